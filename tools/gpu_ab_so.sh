#!/bin/bash
# GPU call: flagship bench with the in-tree HIP extension, then with each
# variants/<name>.so swapped in (tools/build_variant.sh), then the in-tree one
# again. Results: gpurun_out/ab_so.log. Usage: bash tools/gpu_ab_so.sh name ...
# Extra bench arguments: BENCH_ARGS="--regression" bash tools/gpu_ab_so.sh ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SO=$(ls mpitree_amd/_hip*.so)
cp "$SO" gpurun_out/.base.so
: > gpurun_out/ab_so.log
run() {
  echo "== $1" >> gpurun_out/ab_so.log
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 $BENCH_ARGS 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['tree_nodes'])" >> gpurun_out/ab_so.log
}
run base
for v in "$@"; do
  cp "variants/$v.so" "$SO"
  run "$v"
  cp gpurun_out/.base.so "$SO"
done
run base
for v in "$@"; do
  cp "variants/$v.so" "$SO"
  run "$v"
  cp gpurun_out/.base.so "$SO"
done
rm -f gpurun_out/.base.so
