#!/bin/bash
# GPU call: finisher phase profile + rocprofv3 kernel stats of the flagship bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u bench/fin_prof.py > gpurun_out/fin_prof.log 2>&1
rm -rf gpurun_out/prof
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof.log 2>&1
