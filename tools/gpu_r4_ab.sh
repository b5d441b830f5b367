#!/bin/bash
# GPU call (round 4): exact engine -- tests, bench, timeline, per-level debug counts.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "exact or probe" > gpurun_out/gputests_ab.log 2>&1
: > gpurun_out/bench_ab.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --continuous --steps 10 --warmup 2 >> gpurun_out/bench_ab.log 2>&1
done
MPITREE_EXACT_SYNC=1 timeout -k 10 200 python bench.py --continuous --steps 1 --warmup 0 > gpurun_out/exact_levels.log 2>&1
bash tools/gpu_timeline_bench.sh exact "--continuous --steps 2 --warmup 1"
