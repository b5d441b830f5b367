#!/bin/bash
# Round-3 GPU call: the GPU test suite (optional -k filter), then the flagship
# bench, the continuous-feature (exact engine) bench and the regression bench.
# Usage (via gpurun): bash tools/gpu_r3.sh [pytest -k expression | -]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
K=${1:--}
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/gputests.log 2>&1
elif [ "$K" = "-" ] && [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1
fi
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
timeout -k 10 180 python -u bench.py --steps 5 --warmup 2 --continuous >> gpurun_out/bench.log 2>&1
timeout -k 10 180 python -u bench.py --steps 5 --warmup 2 --regression >> gpurun_out/bench.log 2>&1
