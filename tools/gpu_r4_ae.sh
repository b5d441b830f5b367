#!/bin/bash
# GPU call (round 4): benches after reverting the partition's counter peek.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "exact or tiny" > gpurun_out/gputests_ae.log 2>&1
: > gpurun_out/bench_ae.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 >> gpurun_out/bench_ae.log 2>&1
  timeout -k 10 200 python bench.py --continuous --steps 10 --warmup 2 >> gpurun_out/bench_ae.log 2>&1
  timeout -k 10 200 python bench.py --continuous --n 100000 --features 32 --max-depth 12 --steps 10 --warmup 2 >> gpurun_out/bench_ae.log 2>&1
done
