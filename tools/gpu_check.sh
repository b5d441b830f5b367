#!/bin/bash
# One GPU call: the GPU test suite, the flagship bench with an A/B env toggle,
# and a rocprofv3 kernel-trace of the default path. Usage (via gpurun):
#   bash tools/gpu_check.sh [ENV_VAR_TOGGLED_OFF]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AB=${1:-MPITREE_DEVICE_ASSEMBLY}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_on.log 2>&1
env "$AB=0" timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_off.log 2>&1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 >> gpurun_out/bench_on.log 2>&1
rm -rf gpurun_out/prof_on
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_on -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_on.log 2>&1
