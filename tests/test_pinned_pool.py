"""The pinned output pool (ops/hip_backend._pinned_out) never hands out a
buffer a fitted tree still views, and reuses buffers nobody views."""
import numpy as np
import torch

import mpitree_amd.ops.hip_backend as hb


def test_pool_reuses_only_unreferenced(monkeypatch):
    real_empty = torch.empty

    def empty(*a, **k):  # no GPU here: plain host memory stands in for pinned
        k.pop("pin_memory", None)
        return real_empty(*a, **k)

    monkeypatch.setattr(torch, "empty", empty)
    monkeypatch.setattr(hb, "_OUT_POOL", [])

    def tree(nbytes):
        t, arr = hb._pinned_out(nbytes)
        return arr[: nbytes // 8 * 8].view(np.int64)  # a column view, as from_packed makes

    a = tree(4096)
    b = tree(4096)
    assert not np.shares_memory(a, b) and len(hb._OUT_POOL) == 2
    a[:] = 7
    del a
    c = tree(4096)  # a's buffer is free again
    assert len(hb._OUT_POOL) == 2 and not np.shares_memory(b, c)
    d = tree(1 << 20)  # larger than every pooled buffer
    assert len(hb._OUT_POOL) == 3
    assert all(not np.shares_memory(x, y) for x, y in ((b, c), (b, d), (c, d)))
