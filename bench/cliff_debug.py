"""One wide/many-class fit vs the CPU builder (debugging the finisher's tiled
paths): prints engine, finisher stats and whether the trees are equal.

    python bench/cliff_debug.py --C 200 --F 8 --n 30000
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mpitree_amd import DecisionTreeClassifier  # noqa: E402
from tests.helpers import random_problem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--C", type=int, default=200)
    ap.add_argument("--F", type=int, default=8)
    ap.add_argument("--n", type=int, default=30000)
    ap.add_argument("--levels", type=int, default=48)
    ap.add_argument("--codes", action="store_true", help="compare the device binning first")
    a = ap.parse_args()
    rng = np.random.default_rng(a.C * 1000 + a.F)
    X, y = random_problem(rng, a.n, a.F, a.C, levels=a.levels)
    if a.codes:
        from mpitree_amd.core import fit as fm
        from mpitree_amd.core.binning import fit_bin_mapper
        from mpitree_amd.ops.gpu_prepare import prepare

        prep = prepare(torch.from_numpy(X).cuda(), y, regression=False, max_bins=256,
                       encode_labels=fm._encode_labels, encode_targets=fm._encode_targets,
                       exponent=fm.fixed_point_exponent, sync=True)
        ref = fit_bin_mapper(X, 256).transform(X)
        rm = prep.codes_rm.cpu().numpy()[:, : a.F]
        fmj = prep.codes_fm.cpu().numpy().T
        bad_rm = np.argwhere(rm != ref)
        bad_fm = np.argwhere(fmj != ref)
        print(json.dumps(dict(codes_rm_shape=list(prep.codes_rm.shape),
                              codes_fm_shape=list(prep.codes_fm.shape),
                              rm_bad=int(len(bad_rm)), fm_bad=int(len(bad_fm)),
                              rm_first=bad_rm[:3].tolist(), fm_first=bad_fm[:3].tolist())),
              flush=True)
    cpu = DecisionTreeClassifier(device="cpu").fit(X, y)
    gpu = DecisionTreeClassifier(device="cuda").fit(torch.from_numpy(X).cuda(),
                                                    torch.from_numpy(y).cuda())
    torch.cuda.synchronize()
    ga, ca = gpu.tree_arrays_, cpu.tree_arrays_
    out = dict(C=a.C, F=a.F, n=a.n, engine=gpu.fit_stats_.get("engine"),
               finisher_subtrees=gpu.fit_stats_.get("finisher_subtrees"),
               nodes_gpu=ga.node_count, nodes_cpu=ca.node_count, equal=bool(ga.equal(ca)))
    if not out["equal"] and ga.node_count == ca.node_count:
        for name in ("feature", "threshold_bin", "left", "right", "n_samples", "count"):
            g, c = np.asarray(getattr(ga, name)), np.asarray(getattr(ca, name))
            bad = np.nonzero((g != c).reshape(len(g), -1).any(1))[0]
            if bad.size:
                out["first_diff"] = dict(col=name, node=int(bad[0]), gpu=g[bad[0]].tolist(),
                                         cpu=c[bad[0]].tolist(), n_bad=int(bad.size))
                break
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
