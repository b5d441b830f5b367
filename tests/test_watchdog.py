"""The collective-fit watchdog (parallel/failure.py): one thread per process,
re-armed per fit, polls the failure counter only while a fit is armed, and a
peer's failure sets ABORT. A dict stands in for the c10d store (no processes)."""
import threading
import time

from mpitree_amd.parallel import failure as fl


class _Store:
    def __init__(self):
        self.d = {}
        self.lock = threading.Lock()

    def add(self, k, v):
        with self.lock:
            self.d[k] = self.d.get(k, 0) + v
            return self.d[k]


class _Comm:
    world_size, rank = 2, 0


def _guard(store):
    g = fl.FitGuard(_Comm())
    g.store = store
    g.POLL_S = 0.01
    return g


def test_one_thread_rearmed_per_fit():
    store = _Store()
    before = {t.ident for t in threading.enumerate() if t.name == "mpitree-fit-watchdog"}
    for _ in range(20):
        with _guard(store):
            pass
    after = {t.ident for t in threading.enumerate() if t.name == "mpitree-fit-watchdog"}
    assert len(after - before) <= 1  # (the first fit of the process starts it)
    assert not fl.ABORT.is_set()


def test_peer_failure_sets_abort_while_armed():
    store = _Store()
    g = _guard(store)
    with g:
        store.add(g.pfx + "/nfail", 1)  # a peer failed this fit
        t_end = time.time() + 5
        while not fl.ABORT.is_set() and time.time() < t_end:
            time.sleep(0.01)
        assert fl.ABORT.is_set()
    assert not fl.ABORT.is_set()  # cleared when the fit's guard exits
    # the next fit's guard is watched again (its own counter is clean)
    with _guard(store):
        time.sleep(0.05)
        assert not fl.ABORT.is_set()


def test_stale_loop_never_aborts_the_next_fit():
    """A previous fit's loop that sees its own failure counter after that fit
    ended must not set ABORT for the fit running now."""
    store = _Store()
    old = _guard(store)
    with old:
        pass
    store.add(old.pfx + "/nfail", 1)  # the old fit's counter moves late
    with _guard(store):
        old._done.clear()  # (as if the old loop were still polling)
        t = threading.Thread(target=old._watch, daemon=True)
        t.start()
        time.sleep(0.1)
        assert not fl.ABORT.is_set()
        old._done.set()
        t.join(2)


def test_busy_watcher_is_replaced():
    """A watcher whose previous loop is stuck is abandoned: the next fit gets a
    fresh thread instead of running unwatched."""
    w = fl._watcher()
    w.idle.clear()  # (stuck in a previous guard's loop)
    orig = w.idle.wait
    w.idle.wait = lambda timeout=None: False
    try:
        store = _Store()
        g = _guard(store)
        with g:
            assert fl._WATCHER[0] is not w
            assert fl._WATCHER[0].is_current(g)
    finally:
        w.idle.wait = orig
        w.idle.set()
