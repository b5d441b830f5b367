"""Build the native extensions in-tree.

* ``mpitree_amd/_hip*.so``: gfx950 kernels (``ops/csrc/*.hip``) + pybind11
  bindings, compiled with ``hipcc --offload-arch=gfx950``. No PyTorch headers,
  no hipify: plain HIP for CDNA4 only.
* ``mpitree_amd/_cpu*.so``: the native host builder (``ops/csrc/cpu_*.cpp``),
  compiled with g++ so CPU-only machines do not need the HIP runtime.

Both builds use ``-ffp-contract=off`` so the shared split criterion
(``criterion.h``) evaluates to identical bits on host and device.

Usage: ``python -m mpitree_amd.ops.build [--force] [--only hip|cpu]``.
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parents[1]
CSRC = PKG / "ops" / "csrc"
BUILD = PKG.parent / "build" / "native"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("MPITREE_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["hist.hip", "split_scan.hip", "partition.hip", "predict.hip", "misc.hip",
               "finish.hip", "finish_reg.hip", "assemble.hip", "binning.hip", "grow.hip",
               "exact2.hip", "exact_setup.hip", "small_fit.hip", "dp_route.hip", "bindings.cpp",
               "exact2_bind.cpp", "grow_bind.cpp"]
CPU_SOURCES = ["cpu_builder.cpp"]
HEADERS = ["common.h", "criterion.h", "cpu_builder_core.h", "grow.h", "tiny_sort.h", "exact2.h"]


def _pybind_includes() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cand = Path(rocm) / "bin" / "hipcc"
    return str(cand) if cand.exists() else "hipcc"


def _digest(files: list[Path], extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for f in sorted(files):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def _run(cmd: list[str]):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def hip_target() -> Path:
    return PKG / f"_hip{EXT}"


def cpu_target() -> Path:
    return PKG / f"_cpu{EXT}"


def build_hip(force: bool = False, verbose: bool = False) -> Path:
    srcs = [CSRC / s for s in HIP_SOURCES if (CSRC / s).exists()]
    deps = srcs + [CSRC / h for h in HEADERS]
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
             "-Wno-unused-result", "-D__HIP_PLATFORM_AMD__"]
    tag = _digest(deps, " ".join(flags) + ARCH)
    out = hip_target()
    stamp = out.with_suffix(".stamp")
    if not force and out.exists() and stamp.exists() and stamp.read_text() == tag:
        return out
    BUILD.mkdir(parents=True, exist_ok=True)
    inc = [f"-I{CSRC}"] + _pybind_includes()
    objs = []

    def compile_one(src: Path) -> Path:
        obj = BUILD / (src.name + ".o")
        cmd = [_hipcc()] + flags + inc + ["-c", str(src), "-o", str(obj)]
        if src.suffix == ".cpp":  # host-only code, still compiled as HIP for the headers
            cmd = [_hipcc()] + flags + inc + ["-x", "hip", "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(compile_one, srcs))
    link = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(out)] + [
        str(o) for o in objs]
    if verbose:
        print(" ".join(link), flush=True)
    _run(link)
    stamp.write_text(tag)
    return out


def build_cpu(force: bool = False, verbose: bool = False) -> Path:
    srcs = [CSRC / s for s in CPU_SOURCES if (CSRC / s).exists()]
    deps = srcs + [CSRC / h for h in HEADERS]
    flags = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fopenmp",
             "-fvisibility=hidden"]
    tag = _digest(deps, " ".join(flags))
    out = cpu_target()
    stamp = out.with_suffix(".stamp")
    if not force and out.exists() and stamp.exists() and stamp.read_text() == tag:
        return out
    cmd = ["g++"] + flags + [f"-I{CSRC}"] + _pybind_includes() + [str(s) for s in srcs] + [
        "-o", str(out)]
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    stamp.write_text(tag)
    return out


def build_all(force: bool = False, verbose: bool = False, only: str | None = None):
    outs = []
    if only in (None, "cpu"):
        outs.append(build_cpu(force, verbose))
    if only in (None, "hip"):
        outs.append(build_hip(force, verbose))
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["hip", "cpu"])
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    for o in build_all(a.force, a.verbose, a.only):
        print(o)


if __name__ == "__main__":
    sys.exit(main())
