#!/bin/bash
# GPU call (round 4): GPU suite; 200k x 512 / C = 64 / flagship numbers; ownership
# variants at P = 4, 8 (finisher jobs at the switch, units per rank).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gputests.log 2>&1
: > gpurun_out/bench_f.log
for args in "" "--n 200000 --features 512" "--classes 64 --steps 3"; do
  echo "args=$args $(timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 $args 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["tree_nodes"], d["config"]["engine"])')" >> gpurun_out/bench_f.log
done
: > gpurun_out/sim_own_var.log
for jobs in 0 1; do
  for upr in 2 4; do
    echo "== jobs_at_switch=$jobs units_per_rank=$upr" >> gpurun_out/sim_own_var.log
    MPITREE_OWN_JOBS=$jobs timeout -k 10 300 python -u bench/sim_own_ranks.py --ranks 1,4,8 --reps 3 \
      --units-per-rank $upr 2>/dev/null >> gpurun_out/sim_own_var.log
  done
done
