#!/bin/bash
# GPU call: per-kernel averages (rocprofv3 kernel trace of a short flagship
# bench) with the in-tree HIP extension and with each variants/<name>.so swapped
# in (tools/build_variant.sh), twice in alternation. Results: gpurun_out/kexp_so.log.
# Usage: bash tools/gpu_kexp_so.sh name ...   (BENCH_ARGS for other configs)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SO=$(ls mpitree_amd/_hip*.so)
cp "$SO" gpurun_out/.base.so
: > gpurun_out/kexp_so.log
prof() {
  rm -rf gpurun_out/kxs
  timeout -k 10 150 rocprofv3 --kernel-trace -d gpurun_out/kxs -o run -- python3 bench.py --steps 5 --warmup 2 $BENCH_ARGS > gpurun_out/kxs.log 2>&1
  DB=$(ls gpurun_out/kxs/*.db gpurun_out/kxs/*/*.db 2>/dev/null | head -1)
  echo "== $1" >> gpurun_out/kexp_so.log
  python tools/rocpd_top.py "$DB" 14 | grep "mt::" >> gpurun_out/kexp_so.log
  rm -rf gpurun_out/kxs
}
for rep in 1 2; do
  prof base
  for v in "$@"; do
    cp "variants/$v.so" "$SO"
    prof "$v"
    cp gpurun_out/.base.so "$SO"
  done
done
rm -f gpurun_out/.base.so
