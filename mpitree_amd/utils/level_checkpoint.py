"""Level-granular checkpoint / resume of a tree fit.

The reference's only checkpoint is the pickled estimator *after* a fit
(``mpitree/tree/_base.py:22-57``); a fit that dies restarts from the root.
``fit(X, y, checkpoint=path)`` runs the level-wise builder
(:class:`~mpitree_amd.core.levelwise.LevelwiseBuilder`) and, after every
completed level, atomically writes the grower's state to ``path``:

* the node table grown so far (features, bins, links, depths, row counts,
  class counts / target sums, pre-order positions),
* the frontier (start, count, rows, depth, position of every open node) and
  the subtrees deferred to the finisher,
* the row permutation (rows grouped by frontier node),
* a signature of the problem (shapes, hyperparameters, an xxh3-128 digest of
  every binned feature code and target), so a checkpoint is never resumed
  against different data.

A later ``fit`` with the same ``path`` and problem resumes after the last
saved level; its tree is identical to an uninterrupted fit's (the sibling
subtraction of the resumed level is replaced by histogram builds, which give
the same integer histograms). The file is removed when the fit completes.

GPU fits keep the device-driven level loop (``ops/device_grower.py``): after a
level's kernels the grower synchronises once and saves the loop's device state
-- the next frontier's work lists, the level's histograms (the next level
derives siblings from them), the pre-order position space, the finisher jobs
and both row-permutation buffers -- and a resumed fit restores it and carries
on from the next level (:meth:`LevelCheckpoint.save_device`,
:meth:`LevelCheckpoint.load_device`). ``MPITREE_CKPT_EVERY=k`` saves every
k-th level. Multi-GPU fits save one file per rank in two generations (levels
alternate between them); on resume the ranks all-gather which levels they
hold and restart from the newest level every rank has, so a crash between
two ranks' writes never mixes levels.

The exact-threshold list engine (``ops/exact_grower.py``, continuous features)
resumes the same way: after a level's partition it saves both presorted list
buffers of the rank's features (and the regression targets riding with them),
the next frontier, the position space with the resolved thresholds and the
finisher jobs; the resumed level recounts its chunk totals. Its signature
digests the raw feature values.
"""

from __future__ import annotations

import os

import numpy as np

__all__ = ["LevelCheckpoint", "problem_signature"]

_TAB = ("feature", "tbin", "left", "right", "depth", "nsamp", "stats", "pos")
_FR = ("id", "pos", "start", "count", "m", "depth")


def problem_signature(codes, y, params, n_classes: int) -> str:
    """Digest of the fit's full inputs (every binned code and target) and params.

    xxh3-128 over the whole buffers (device tensors are copied to the host
    once); a checkpoint written for different data never matches."""
    import xxhash

    h = xxhash.xxh3_128()

    def host(a):
        try:
            import torch

            if torch.is_tensor(a):
                return a.detach().cpu().numpy()
        except ImportError:  # pragma: no cover
            pass
        return np.asarray(a)

    h.update(repr((tuple(codes.shape), int(n_classes), int(params.criterion), params.max_depth,
                   params.min_samples_split, params.min_samples_leaf)).encode())
    for a in (codes, y):
        h.update(memoryview(np.ascontiguousarray(host(a))).cast("B"))
    return h.hexdigest()


class LevelCheckpoint:
    """One fit's checkpoint file (``path``, ``.npz``)."""

    def __init__(self, path, signature: str = ""):
        self.path = os.fspath(path)
        self.signature = signature
        self.fail_after_level = None  # tests: raise after saving this level
        self.saved_levels = 0
        self.resumed_from = None
        # the saving engine's buffer layout (device loops: finisher rows and buffer
        # dimensions); a saved state of another layout is ignored, never restored
        self.layout = ""

    # ---------------------------------------------------------------- save
    def save(self, level: int, tab, fr: dict, deferred: dict, rows: np.ndarray) -> None:
        arrs = {"sig": np.frombuffer(self.signature.encode(), np.uint8),
                "level": np.array([level], np.int64), "tab_n": np.array([tab.n], np.int64),
                "rows": rows}
        for k in _TAB:
            arrs["tab_" + k] = getattr(tab, k)[: tab.n]
        for k in _FR:
            arrs["fr_" + k] = np.asarray(fr[k])
        for k, parts in deferred.items():
            arrs["def_" + k] = (np.concatenate(parts) if parts
                                else np.zeros(0, np.int64))
        tmp = self.path + ".tmp.npz"
        np.savez(tmp, **arrs)
        os.replace(tmp, self.path)  # atomic: a crash leaves the previous level
        self.saved_levels += 1
        if self.fail_after_level is not None and level >= self.fail_after_level:
            raise CheckpointInterrupt(f"interrupted after level {level} (test hook)")

    # ---------------------------------------------------------------- load
    def load(self):
        """The saved state as a dict, or None (no file / different problem)."""
        if not os.path.exists(self.path):
            return None
        with np.load(self.path, allow_pickle=False) as z:
            if bytes(z["sig"]).decode() != self.signature:
                return None
            st = {k: z[k] for k in z.files}
        self.resumed_from = int(st["level"][0])
        return st

    def restore_table(self, st, tab) -> None:
        n = int(st["tab_n"][0])
        tab._grow(n)
        for k in _TAB:
            getattr(tab, k)[:n] = st["tab_" + k]
        tab.n = n

    @staticmethod
    def restore_frontier(st) -> dict:
        fr = {k: np.asarray(st["fr_" + k], np.int64) for k in _FR}
        K = fr["id"].size
        fr["src"] = np.full(K, -1, np.int64)  # resumed level: every histogram is built
        fr["sib"] = np.full(K, -1, np.int64)
        return fr

    @staticmethod
    def restore_deferred(st, keys) -> dict:
        out = {}
        for k in keys:
            a = st.get("def_" + k)
            out[k] = [np.asarray(a, np.int64)] if a is not None and a.size else []
        return out

    # ------------------------------------------------- device level loop
    def _dev_files(self, rank: int, world: int) -> list:
        self._dev_rw = (rank, world)
        if world <= 1:
            return [self.path]
        return [f"{self.path}.r{rank}of{world}.g{g}.npz" for g in (0, 1)]

    def save_device(self, level: int, arrs: dict, rank: int = 0, world: int = 1) -> None:
        """Write the device loop's state after ``level`` (atomic per file)."""
        files = self._dev_files(rank, world)
        # alternate generations by save count, not level parity: with
        # MPITREE_CKPT_EVERY even every save would land on one file
        dst = files[self.saved_levels % len(files)]
        out = dict(arrs)
        out["sig"] = np.frombuffer(self.signature.encode(), np.uint8)
        out["level"] = np.array([level], np.int64)
        out["device_loop"] = np.array([1], np.int64)
        out["layout"] = np.frombuffer(self.layout.encode(), np.uint8)
        tmp = dst + ".tmp.npz"
        np.savez(tmp, **out)
        os.replace(tmp, dst)
        self.saved_levels += 1
        if self.fail_after_level is not None and level >= self.fail_after_level:
            raise CheckpointInterrupt(f"interrupted after level {level} (test hook)")

    def load_device(self, rank: int = 0, world: int = 1, gather=None):
        """The newest saved device-loop state every rank holds, or None.
        ``gather(int64 array [2]) -> [world, 2]`` all-gathers each rank's saved
        levels (multi-rank fits)."""
        have = {}
        for f in self._dev_files(rank, world):
            if not os.path.exists(f):
                continue
            with np.load(f, allow_pickle=False) as z:
                lay = bytes(z["layout"]).decode() if "layout" in z.files else ""
                if ("device_loop" in z.files and bytes(z["sig"]).decode() == self.signature
                        and lay == self.layout):
                    have[int(z["level"][0])] = f
        if world > 1:
            mine = np.full(2, -1, np.int64)
            lv = sorted(have)[-2:]
            mine[: len(lv)] = lv
            allv = np.asarray(gather(mine)).reshape(world, 2)
            common = set(int(v) for v in allv[0] if v >= 0)
            for r in range(1, world):
                common &= set(int(v) for v in allv[r] if v >= 0)
            level = max(common) if common else -1
        else:
            level = max(have) if have else -1
        if level < 0:
            return None
        with np.load(have[level], allow_pickle=False) as z:
            st = {k: z[k] for k in z.files}
        self.resumed_from = level
        return st

    def clear(self) -> None:
        paths = [self.path, self.path + ".tmp.npz"]
        rw = getattr(self, "_dev_rw", None)
        if rw is not None and rw[1] > 1:
            for f in self._dev_files(*rw):
                paths += [f, f + ".tmp.npz"]
        for p in paths:
            if os.path.exists(p):
                os.remove(p)


class CheckpointInterrupt(RuntimeError):
    """Raised by the ``fail_after_level`` test hook after a checkpoint write."""
