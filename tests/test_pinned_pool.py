"""The zero-copy output pool (ops/hip_backend._zc_out) never hands out a
buffer a fitted tree still views, and reuses buffers nobody views."""
import ctypes

import numpy as np

import mpitree_amd.ops.hip_backend as hb


class _FakeHip:
    """Host memory stands in for mapped pinned memory (no GPU here)."""

    def __init__(self):
        self.live = {}

    def host_alloc(self, n, coherent=True):
        buf = (ctypes.c_uint8 * n)()
        p = ctypes.addressof(buf)
        self.live[p] = buf
        return p

    def host_device_ptr(self, p):
        return p

    def host_free(self, p):
        self.live.pop(p)


def test_pool_reuses_only_unreferenced(monkeypatch):
    fake = _FakeHip()
    monkeypatch.setattr(hb.native, "hip", lambda: fake)
    monkeypatch.setattr(hb, "_ZC_POOL", [])

    def tree(nbytes):
        arr, dptr = hb._zc_out(nbytes)
        assert dptr == arr.ctypes.data
        return arr[: nbytes // 8 * 8].view(np.int64)  # a column view, as from_packed makes

    a = tree(4096)
    b = tree(4096)
    assert not np.shares_memory(a, b) and len(hb._ZC_POOL) == 2
    a[:] = 7
    del a
    c = tree(4096)  # a's buffer is free again
    assert len(hb._ZC_POOL) == 2 and not np.shares_memory(b, c)
    d = tree(1 << 20)  # larger than every pooled buffer
    assert len(hb._ZC_POOL) == 3
    assert all(not np.shares_memory(x, y) for x, y in ((b, c), (b, d), (c, d)))
    # past eight buffers the oldest unreferenced one is released
    keep = [tree(8192 * (i + 2)) for i in range(6)]
    assert len(hb._ZC_POOL) <= 9 and len(fake.live) == len(hb._ZC_POOL)
    del keep
