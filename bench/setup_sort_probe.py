"""Time the exact engine's setup sort (exact_setup.hip) alone on 1M x 64 N(0,1)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpitree_amd.ops import native  # noqa: E402

n, F = int(os.environ.get("N", 1_000_000)), int(os.environ.get("F", 64))
hip = native.hip()
X = torch.randn(n, F, device="cuda")
dev = X.device
keys = [torch.empty((F, n), dtype=torch.int32, device=dev) for _ in range(2)]
rows = [torch.empty((F, n), dtype=torch.int32, device=dev) for _ in range(2)]
tb = int(hip.exact_setup_temp_bytes(n, F))
temp = torch.empty(tb, dtype=torch.uint8, device=dev)
chunk = int(hip.exact_setup_chunk())
nc = -(-n // chunk)
cnt = torch.empty((F, nc), dtype=torch.int32, device=dev)
nuniq = torch.empty(F, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream().cuda_stream


def run():
    hip.exact_setup_sort(s, X.data_ptr(), n, F, keys[0].data_ptr(), keys[1].data_ptr(),
                         rows[0].data_ptr(), rows[1].data_ptr(), temp.data_ptr(), tb,
                         cnt.data_ptr(), nuniq.data_ptr(), xs=F, f_lo=0)


for _ in range(3):
    run()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    run()
b.record()
torch.cuda.synchronize()
print(f"setup sort {n}x{F} tile {os.environ.get('MPITREE_SORT_TILE', 'default')}: "
      f"{a.elapsed_time(b) / 20:.3f} ms", flush=True)
