#!/bin/bash
# GPU call: the GPU test suite (optionally a -k filter) then the flagship bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/gputests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1
fi
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
