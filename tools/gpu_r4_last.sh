#!/bin/bash
# GPU call (round 4, last): full GPU suite, smoke, flagship and exact bench lines.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gputests_last.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_last.log 2>&1
: > gpurun_out/bench_last.log
for i in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 >> gpurun_out/bench_last.log 2>&1
  timeout -k 10 200 python -u bench.py --continuous --steps 10 --warmup 2 >> gpurun_out/bench_last.log 2>&1
done
