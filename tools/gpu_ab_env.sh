#!/bin/bash
# GPU call: flagship bench under several env settings, alternated twice
# (gpurun_out/ab_env.log). Usage: bash tools/gpu_ab_env.sh "ENV=1" "ENV=2" ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab_env.log
for rep in 1 2; do
  for cfg in "MPITREE_NOOP=0" "$@"; do
    echo "== $cfg" >> gpurun_out/ab_env.log
    env $cfg timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 $BENCH_ARGS 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['tree_nodes'])" >> gpurun_out/ab_env.log
  done
done
