#!/bin/bash
# GPU call (round 4): threshold ranks searched on the sorted keys -- exact tests,
# classification + regression exact benches.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "exact" > gpurun_out/gputests_ag.log 2>&1
: > gpurun_out/bench_ag.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --continuous --steps 10 --warmup 2 >> gpurun_out/bench_ag.log 2>&1
  timeout -k 10 200 python bench.py --continuous --regression --steps 5 --warmup 2 >> gpurun_out/bench_ag.log 2>&1
done
