#!/bin/bash
# GPU call (round 4): full GPU suite after the exact-threshold binning probe, then the
# continuous (exact) and flagship benches.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests_z.log 2>&1
: > gpurun_out/bench_z.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --continuous --steps 10 --warmup 2 >> gpurun_out/bench_z.log 2>&1
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 >> gpurun_out/bench_z.log 2>&1
done
