#!/bin/bash
# GPU call (round 4): full GPU suite, host level-enqueue A/B (MPITREE_LEVEL_CTX),
# flagship timeline, regression ownership simulation.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gputests.log 2>&1
: > gpurun_out/ab_ctx.log
for rep in 1 2; do
  for v in 0 1; do
    for args in "" "--n 100000 --features 32 --max-depth 12" "--regression"; do
      echo "ctx=$v args=$args $(MPITREE_LEVEL_CTX=$v timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 $args 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["tree_nodes"])')" >> gpurun_out/ab_ctx.log
    done
  done
done
bash tools/gpu_timeline_bench.sh ctx "--steps 3 --warmup 1" c64 "--steps 2 --warmup 1 --classes 64"
timeout -k 10 300 python -u bench/sim_own_ranks.py --regression --reps 3 > gpurun_out/sim_own_reg.log 2>&1
timeout -k 10 300 python -u bench/sim_own_ranks.py --reps 3 > gpurun_out/sim_own_cls.log 2>&1
timeout -k 10 400 python -u bench/sim_own_ranks.py --n 10000000 --features 128 --reps 2 > gpurun_out/sim_own_10m.log 2>&1
bash tools/gpu_r4_d2h.sh
