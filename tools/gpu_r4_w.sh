#!/bin/bash
# GPU call (round 4): exact-engine GPU tests after removing the staged partition, then
# the continuous 1M x 64 bench (twice).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "exact" > gpurun_out/gputests_w.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --continuous --steps 10 --warmup 2 >> gpurun_out/bench_w.log 2>&1
done
