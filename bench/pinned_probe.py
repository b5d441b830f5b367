"""Probe: cost of pinned host allocations and D2H copies of tree-sized buffers."""
import time

import torch

dev = torch.device("cuda", 0)
src = torch.empty(16 << 20, dtype=torch.uint8, device=dev)
for nbytes in (3 << 20, 11 << 20, 64 << 20, 120 << 20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        del h
    t1 = time.perf_counter()
    keep = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
    t2 = time.perf_counter()
    s = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    h = keep[0]
    for _ in range(3):
        h.copy_(s, non_blocking=True)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    for _ in range(10):
        h.copy_(s, non_blocking=True)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"{nbytes >> 20} MB: alloc+free (cached) {(t1 - t0) / 5 * 1e3:.3f} ms, "
          f"3 live allocs {(t2 - t1) / 3 * 1e3:.3f} ms each, "
          f"D2H {(t4 - t3) / 10 * 1e3:.3f} ms = {nbytes / ((t4 - t3) / 10) / 1e9:.1f} GB/s",
          flush=True)
