"""The node-local shared-host tree pool (parallel/shared_tree.py): every rank
makes the same slot choice from the gathered free masks, a slot a rank still
views is never reused, and ranks of one machine see each other's writes after
the flag barrier. Host memory stands in for the HIP registration (no GPU)."""
import multiprocessing as mp

import numpy as np
import pytest

from mpitree_amd.parallel import shared_tree as st


class _FakeHip:
    def host_register(self, p, n):
        return p  # (the device pointer of a mapped host range)

    def host_unregister(self, p):
        pass


class _Comm:
    def __init__(self, rank, P):
        self.rank, self.world_size = rank, P


def _pool(rank=0, P=2, uid=None):
    return st.ShmTreePool(_Comm(rank, P), _FakeHip(), uid if uid is not None else 0x5EED + rank)


def test_choose_reuses_only_slots_free_everywhere():
    pool = _pool()
    a = pool.choose([0, 0], 1000)  # nothing exists: a new slot
    assert a.nbytes - st.HEADER >= 1000 and pool.free_mask() == 1
    view = a.nd[st.HEADER : st.HEADER + 64]  # a tree this rank still holds
    assert pool.free_mask() == 0
    b = pool.choose([pool.free_mask(), 1], 1000)  # busy here: another slot
    assert b is not a
    del view
    assert pool.free_mask() == 3
    # the peer still holds slot 0: slot 1 is the only one free everywhere
    assert pool.choose([3, 2], 1000) is b
    # too small everywhere: a new, larger slot
    c = pool.choose([3, 3], 10 << 20)
    assert c is not a and c is not b and c.nbytes - st.HEADER >= 10 << 20
    for sl in list(pool.slots.values()):
        sl.close()


def test_next_slot_is_agreed_ahead_and_excludes_the_current():
    pool = _pool()
    cur = pool.choose([0, 0], 4096)
    pool.plan_next([pool.free_mask(), pool.free_mask()], cur, 4096)
    nxt = pool.take_next()
    assert nxt is not None and nxt is not cur and pool.take_next() is None
    for sl in list(pool.slots.values()):
        sl.close()


def test_short_dev_shm_refuses_a_new_slot_but_reuses_one():
    pool = _pool()
    a = pool.choose([0, 0], 1 << 20)
    small = [st.SHM_MARGIN, 10 * st.SHM_MARGIN]  # one rank's /dev/shm is nearly full
    # a new slot would not fit beside the margin on that rank: every rank falls back
    assert pool.choose([0, 0], 1 << 20, shm_free=small) is None
    # an existing free slot costs no /dev/shm: it is still chosen
    assert pool.choose([1, 1], 1 << 20, shm_free=small) is a
    pool.plan_next([1, 1], a, 1 << 20, shm_free=small)
    assert pool.take_next() is None
    assert st.shm_free_bytes() >= 0
    for sl in list(pool.slots.values()):
        sl.close()


def _rank_main(rank, uid, q):
    pool = st.ShmTreePool(_Comm(rank, 2), _FakeHip(), uid)
    slot = pool.choose([0, 0], 1 << 16)  # same name on both ranks
    data = slot.nd[st.HEADER : st.HEADER + (1 << 16)].view(np.int64)
    half = data.size // 2
    data[rank * half : (rank + 1) * half] = rank + 1  # this rank's nodes
    pool.barrier(slot)
    q.put((rank, int(data[:half].sum()), int(data[half:].sum()), half))
    del data
    slot.close()


@pytest.mark.timeout(60)
def test_two_ranks_share_one_buffer_through_the_barrier():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = int.from_bytes(np.random.default_rng().bytes(5), "little")
    ps = [ctx.Process(target=_rank_main, args=(r, uid, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=50) for _ in range(2))
    for p in ps:
        p.join(20)
        assert p.exitcode == 0
    for rank, s0, s1, half in got:
        assert s0 == half and s1 == 2 * half  # both ranks' halves, seen by each


def test_pool_belongs_to_the_group_not_the_communicator():
    """Estimators build a communicator per fit: the pool (and its registered
    buffers) is found again through the process group, the host-key all-gather
    runs once."""
    calls = []

    class _G:  # a process group stand-in (weak-referenceable)
        pass

    class _C(_Comm):
        def _all_gather(self, a):
            calls.append(1)
            return np.stack([a, a])

    g = _G()
    a, b = _C(0, 2), _C(0, 2)
    a.group = b.group = g
    p1 = st.pool_for(a, _FakeHip())
    p2 = st.pool_for(b, _FakeHip())
    assert p1 is not None and p1 is p2 and len(calls) == 1
    c = _C(0, 2)
    c.group = _G()  # another group: another pool
    assert st.pool_for(c, _FakeHip()) is not p1 and len(calls) == 2


def test_exact_own_positions_group_jobs_by_owner():
    import torch

    from mpitree_amd.ops.exact_grower import _owners, own_positions

    # jobs {start, count, ...} in finisher order; owners dealt serpentine
    fj = torch.tensor([[0, 5, 0, 0, 0], [10, 3, 0, 0, 0], [20, 4, 0, 0, 0],
                       [30, 2, 0, 0, 0], [40, 1, 0, 0, 0]], dtype=torch.int64)
    own = _owners(5, 2, fj.device)
    pos, sizes = own_positions(fj, own, 2)
    want = {0: [], 1: []}
    for j in range(5):
        want[int(own[j])] += list(range(int(fj[j, 0]), int(fj[j, 0] + fj[j, 1])))
    assert sizes == [len(want[0]), len(want[1])]
    assert pos.tolist() == want[0] + want[1]
