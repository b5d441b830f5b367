"""Per-line host time of the flagship fit's setup path (before the first level).

``host_marks.py`` times whole setup functions; this one traces every line of a
few of them (``sys.settrace`` line events, perf_counter at each) and prints
the median time from each line to the next over the fits, largest first, so
the torch / pybind calls that keep the GPU waiting stand out. The tracer adds
~1 us per line; compare lines with each other, not with host_marks.

    python bench/host_lines.py [--fits 20] [--top 40] [--regression]
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fits", type=int, default=20)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--regression", action="store_true")
    a = ap.parse_args()
    from mpitree_amd.core import fit as fitmod
    from mpitree_amd.core.criterion import Criterion
    from mpitree_amd.ops import device_grower as dg
    from mpitree_amd.ops import gpu_prepare as gp
    from mpitree_amd.ops import hip_backend as hb
    from mpitree_amd.utils.datasets import make_classification, make_regression

    dev = torch.device("cuda", 0)
    if a.regression:
        X, y = make_regression(1_000_000, 64, levels=256, seed=0, device=dev)
    else:
        X, y = make_classification(1_000_000, 64, n_classes=2, levels=256, seed=0, device=dev)

    def fit():
        crit = Criterion.SQUARED_ERROR if a.regression else Criterion.ENTROPY
        return fitmod.fit_tree(X, y, regression=a.regression, criterion=crit,
                               max_depth=None, min_samples_split=2, device="cuda")

    codes = {f.__code__ for f in (fitmod.fit_tree, gp.prepare, gp._Labels.__init__,
                                  gp._Labels.finish, gp._Targets.__init__, gp._Targets.finish,
                                  hb.DeviceBinning.__init__, hb.DeviceBinning.launch_bin,
                                  hb.DeviceBinning.host_tables, hb.DeviceBinning.finish,
                                  hb.HipBackend.setup, hb.HipBackend.begin_positions,
                                  dg.DeviceGrower.fit, dg.device_loop_supported)}
    per = defaultdict(list)
    state = {"last": None, "t": 0.0, "stop": False}

    def tracer(frame, event, arg):
        if frame.f_code not in codes:
            return None

        def local(fr, ev, ar):
            if state["stop"]:
                return None
            if ev == "line":
                now = time.perf_counter()
                if state["last"] is not None:
                    per[state["last"]].append(now - state["t"])
                state["last"] = (fr.f_code.co_filename.split("repo/")[-1], fr.f_lineno)
                state["t"] = time.perf_counter()
                # the first level is enqueued: stop tracing this fit
                if fr.f_code is dg.DeviceGrower.fit.__code__ and "ctx.level" in (
                        _src(fr.f_code.co_filename, fr.f_lineno)):
                    state["stop"] = True
            return local

        return local

    for _ in range(3):
        fit()
    torch.cuda.synchronize()
    runs = 0
    for _ in range(a.fits):
        state.update(last=None, stop=False)
        sys.settrace(tracer)
        fit()
        sys.settrace(None)
        torch.cuda.synchronize()
        runs += 1
    rows = []
    for k, v in per.items():
        v = np.asarray(v) * 1e6
        rows.append((float(np.median(v)) * len(v) / runs, len(v) / runs, k))
    rows.sort(reverse=True)
    print(f"{'us/fit':>8} {'hits':>5}  line")
    for us, hits, (f, ln) in rows[: a.top]:
        print(f"{us:8.1f} {hits:5.1f}  {f}:{ln}  {_src(f, ln).strip()[:90]}")


_SRC: dict = {}


def _src(path, ln):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    full = path if os.path.isabs(path) else os.path.join(root, path)
    lines = _SRC.get(full)
    if lines is None:
        try:
            with open(full) as fh:
                lines = _SRC[full] = fh.read().splitlines()
        except OSError:
            lines = _SRC[full] = []
    return lines[ln - 1] if 0 < ln <= len(lines) else ""


if __name__ == "__main__":
    main()
