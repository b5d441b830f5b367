#!/bin/bash
# GPU call: exact-engine configurations + a rocprofv3 kernel trace of the 100k one.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench/baseline_configs.py 100k_exact 1m_exact --reps 2 > gpurun_out/exact_bench.log 2>&1
rm -rf gpurun_out/prof_exact
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_exact -o run -- python3 bench/baseline_configs.py 100k_exact --reps 1 > gpurun_out/prof_exact.log 2>&1
