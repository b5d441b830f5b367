"""Host timestamps of one fit's setup steps, 1 GPU vs a simulated ownership rank.

The GPU idles before the first level while the host prepares it (the gaps at
the head of ``profiles/r5/flagship_timeline.txt``); a simulated P = 8 ownership
rank showed twice the 1-GPU gap there. This wraps the setup steps of
``fit_tree`` / ``DeviceGrower.fit`` with perf_counter stamps and prints the
median offset of each from the start of the fit (us), per configuration.

    python bench/host_marks.py [--ranks 1+8] [--fits 20]
"""
from __future__ import annotations

import argparse
import functools
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STAMPS: list = []


def _wrap(obj, name, label):
    fn = getattr(obj, name)

    @functools.wraps(fn)
    def w(*a, **k):
        STAMPS.append((label + ">", time.perf_counter()))
        r = fn(*a, **k)
        STAMPS.append((label + "<", time.perf_counter()))
        return r

    setattr(obj, name, w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1+8")
    ap.add_argument("--fits", type=int, default=20)
    a = ap.parse_args()
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    import sim_own_ranks as so

    from mpitree_amd.core import fit as fitmod
    from mpitree_amd.ops import device_grower as dg
    from mpitree_amd.ops import gpu_prepare as gp
    from mpitree_amd.ops import hip_backend as hb
    from mpitree_amd.utils.datasets import make_classification

    dev = torch.device("cuda", 0)
    X, y = make_classification(1_000_000, 64, n_classes=2, seed=0, device=dev)

    def fit(comm=None):
        return fitmod.fit_tree(X, y, regression=False, criterion=0, max_depth=None,
                               min_samples_split=2, device="cuda", comm=comm)

    for _ in range(2):
        fit()
    dg.REC_DUMP = []
    ref, ref_rows = so.reference_rows(fit, dev, False)
    ref_recs, dg.REC_DUMP = dg.REC_DUMP, None
    ref_pos = ref_rows[:, 0].long().contiguous()
    pool = so.SimPool(so.SimSlot(so.packed_bytes(ref.arrays)))
    for obj, name in [(gp, "prepare"), (hb.HipBackend, "setup"), (hb.HipBackend, "begin_positions"),
                      (dg, "device_loop_supported"), (dg.DeviceGrower, "fit"),
                      (dg.DeviceGrower, "_workspace"), (hb.HipBackend, "assemble_positions"),
                      (hb.HipBackend, "launch_finisher"),
                      (gp._Labels, "__init__"), (gp._Labels, "after_first_sync"),
                      (gp._Labels, "finish"), (hb.DeviceBinning, "__init__"),
                      (hb.DeviceBinning, "launch_bin_early"), (hb.DeviceBinning, "launch_bin"),
                      (hb.DeviceBinning, "finish"), (torch.cuda.Event, "synchronize"),
                      (torch.cuda.Event, "record"), (fitmod, "_validate_X"),
                      (fitmod, "resolve_device"), (fitmod, "_level_checkpoint")]:
        _wrap(obj, name, f"{getattr(obj, '__name__', '')}.{name}")
    orig_ctx = None
    from mpitree_amd.ops import native

    hip = native.hip()
    orig_ctx = hip.GrowCtx

    class Ctx:
        def __init__(self, *a):
            STAMPS.append(("GrowCtx>", time.perf_counter()))
            self._c = orig_ctx(*a)
            STAMPS.append(("GrowCtx<", time.perf_counter()))
            self._first = True

        def __getattr__(self, k):
            return getattr(self._c, k)

        def level(self, s, lvl):
            if self._first:
                STAMPS.append(("first level>", time.perf_counter()))
                self._first = False
            self._c.level(s, lvl)

    hip.GrowCtx = Ctx
    for P in [int(v) for v in a.ranks.replace("+", ",").split(",")]:
        runs = []
        for i in range(a.fits + 2):
            comm = (so.SimOwnComm(P, 0, dev, ref_rows, ref_pos, ref.arrays.max_depth, pool,
                                  ref_recs) if P > 1 else None)
            pool.slot.prefill()
            torch.cuda.synchronize()
            STAMPS.clear()
            t0 = time.perf_counter()
            fit(comm)
            torch.cuda.synchronize()
            if i >= 2:
                runs.append([(k, (t - t0) * 1e6) for k, t in STAMPS])
        keys = [k for k, _ in runs[0]]
        med = {}
        for j, k in enumerate(keys):
            vals = [r[j][1] for r in runs if len(r) > j and r[j][0] == k]
            med[f"{j:02d} {k}"] = round(float(np.median(vals)), 1)
        print(json.dumps(dict(P=P, stamps_us=med)), flush=True)
    hip.GrowCtx = orig_ctx


if __name__ == "__main__":
    main()
