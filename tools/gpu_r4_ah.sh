#!/bin/bash
# GPU call (round 4): scatter store loop with 4 entries per lane -- sort test, exact
# tests, exact bench, setup-sort timing and kernel table.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "exact" > gpurun_out/gputests_ah.log 2>&1
: > gpurun_out/bench_ah.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --continuous --steps 10 --warmup 2 >> gpurun_out/bench_ah.log 2>&1
done
bash tools/gpu_timeline_bench.sh exact "--continuous --steps 2 --warmup 1"
