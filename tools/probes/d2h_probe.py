"""D2H copy rate of a finished-tree-sized buffer (6.7 MB) into pinned host memory.

Run under different runtime settings (the tree copy is ~200 us of a 3.3 ms fit):
    python tools/probes/d2h_probe.py [MB]
"""
import os
import sys
import time

import torch

mb = float(sys.argv[1]) if len(sys.argv) > 1 else 6.7
n = int(mb * 1e6)
dev = torch.device("cuda", 0)
src = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
dst = torch.empty(n, dtype=torch.uint8, pin_memory=True)
s = torch.cuda.current_stream()
for chunks in (1, 2, 4):
    streams = [torch.cuda.Stream() for _ in range(chunks)]
    best = 1e9
    for rep in range(30):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step = (n + chunks - 1) // chunks
        for i, st in enumerate(streams):
            st.wait_stream(s)
            with torch.cuda.stream(st):
                dst[i * step:(i + 1) * step].copy_(src[i * step:(i + 1) * step], non_blocking=True)
        for st in streams:
            st.synchronize()
        best = min(best, time.perf_counter() - t0)
    print(f"env SDMA={os.environ.get('HSA_ENABLE_SDMA', '-')} "
          f"BLIT={os.environ.get('GPU_FORCE_BLIT_COPY_SIZE', '-')} chunks={chunks}: "
          f"{mb:.1f} MB in {best * 1e6:.0f} us = {mb / 1e3 / best:.1f} GB/s", flush=True)
