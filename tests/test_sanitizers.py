"""Host sanitizers on the native tree builder.

GPU AddressSanitizer / XNACK runs are not available on the MI355X pool, so the
sanitizer coverage SURVEY §5 asks for is applied to the host code: the exact
builder core (``ops/csrc/cpu_builder_core.h``, the same code the ``_cpu``
extension runs) is compiled into a stand-alone harness with
``-fsanitize=address,undefined`` and fed problems that exercise both scan
paths (dense per-bin counts and sorted pairs), u8 and u16 codes, ties,
constant features, ``min_samples_leaf`` and every criterion. Any heap/stack
overflow, use-after-free, leak or UB aborts the harness; its tree must also
equal the extension's bit for bit.
"""

from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from mpitree_amd.core.criterion import Criterion
from mpitree_amd.ops import native

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "mpitree_amd" / "ops" / "csrc"
DRIVER = Path(__file__).resolve().parent / "native" / "asan_driver.cpp"

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = tmp_path_factory.mktemp("asan") / "asan_driver"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fopenmp",
           "-ffp-contract=off", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           f"-I{CSRC}", str(DRIVER), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(f"sanitizer build failed:\n{r.stderr}")
    return exe


def _run(exe, tmp, codes, y, nbins, C, crit, max_depth=-1, mss=2, msl=1, threads=1):
    n, F = codes.shape
    reg = crit == int(Criterion.SQUARED_ERROR)
    hdr = np.array([n, F, C, crit, max_depth, mss, msl, threads, codes.dtype.itemsize], np.int64)
    inp, out = tmp / "in.bin", tmp / "out.bin"
    with open(inp, "wb") as f:
        f.write(hdr.tobytes())
        f.write(np.ascontiguousarray(codes).tobytes())
        f.write(np.ascontiguousarray(y, np.int64 if reg else np.int32).tobytes())
        f.write(np.ascontiguousarray(nbins, np.int32).tobytes())
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS=str(threads))
    r = subprocess.run([str(exe), str(inp), str(out)], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, f"sanitizer reported an error:\n{r.stderr[-4000:]}"
    raw = np.fromfile(out, dtype=np.int64)
    N = int(raw[0])
    S = 2 if reg else C
    return raw[1:].reshape(N, 6 + S)


def _extension(codes, y, nbins, C, crit, max_depth=-1, mss=2, msl=1, threads=1):
    reg = crit == int(Criterion.SQUARED_ERROR)
    out = native.cpu().build_tree(np.ascontiguousarray(codes),
                                  np.ascontiguousarray(y, np.int64 if reg else np.int32),
                                  np.ascontiguousarray(nbins, np.int32), C, crit, max_depth, mss,
                                  msl, threads)
    return np.concatenate([np.stack([out["feature"], out["bin"], out["depth"], out["left"],
                                     out["right"], out["nsamp"]], 1).astype(np.int64),
                           out["stats"].astype(np.int64)], 1)


CASES = [
    # (n, F, C, levels, code dtype, criterion, max_depth, mss, msl, threads)
    (300, 5, 3, 7, np.uint8, Criterion.ENTROPY, -1, 2, 1, 1),  # sorted-pairs scan
    (4000, 3, 2, 6, np.uint8, Criterion.GINI, -1, 2, 1, 1),  # dense per-bin scan
    (2500, 4, 4, 300, np.uint16, Criterion.ENTROPY, 9, 5, 3, 1),  # u16 codes, depth cap, msl
    (3000, 6, 0, 20, np.uint8, Criterion.SQUARED_ERROR, -1, 2, 2, 1),  # regression
    (20000, 4, 3, 16, np.uint8, Criterion.ENTROPY, -1, 2, 1, 4),  # OpenMP feature scan
    (64, 3, 2, 1, np.uint8, Criterion.ENTROPY, -1, 2, 1, 1),  # constant features: root leaf
]


@pytest.mark.parametrize("case", CASES, ids=[f"n{c[0]}-F{c[1]}-{Criterion(c[5]).name}"
                                             for c in CASES])
def test_builder_under_asan_ubsan(harness, tmp_path, case):
    if not native.has_cpu():
        pytest.skip("native host builder not built")
    n, F, C, levels, dt, crit, md, mss, msl, thr = case
    rng = np.random.default_rng(n + F)
    codes = rng.integers(0, levels, size=(n, F)).astype(dt)
    nbins = np.full(F, max(levels, 1), np.int32)
    if crit == Criterion.SQUARED_ERROR:
        y = (rng.normal(size=n) * 1000).round().astype(np.int64)
        C = 0
    else:
        y = (codes[:, 0].astype(np.int64) + rng.integers(0, 2, size=n)) % C
    got = _run(harness, tmp_path, codes, y, nbins, C, int(crit), md, mss, msl, thr)
    want = _extension(codes, y, nbins, C, int(crit), md, mss, msl, thr)
    np.testing.assert_array_equal(got, want)
    assert got[0, 5] == n  # the root holds every row
