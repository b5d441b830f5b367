#!/bin/bash
# GPU call: flagship bench + finisher phase profile for the in-tree HIP extension
# and each variants/<name>.so (tools/build_variant.sh), two alternations.
# Results: gpurun_out/ab_fin.log. Usage: bash tools/gpu_ab_fin.sh name ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SO=$(ls mpitree_amd/_hip*.so)
cp "$SO" gpurun_out/.base.so
: > gpurun_out/ab_fin.log
run() {
  echo "== $1" >> gpurun_out/ab_fin.log
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 $BENCH_ARGS 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['tree_nodes'])" >> gpurun_out/ab_fin.log
  if [ -n "$FIN_PROF" ]; then
    timeout -k 10 120 python -u bench/fin_prof.py 2>/dev/null | grep -E "cycle split|cycles per node|wall us" >> gpurun_out/ab_fin.log
  fi
}
for rep in 1 2; do
  cp gpurun_out/.base.so "$SO"
  run base
  for v in "$@"; do
    cp "variants/$v.so" "$SO"
    run "$v"
  done
done
cp gpurun_out/.base.so "$SO"
rm -f gpurun_out/.base.so
