#!/bin/bash
# GPU call (round 4): XCD-grouped partition tickets -- exact tests, then A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "exact" > gpurun_out/gputests_ac.log 2>&1
BENCH_ARGS="--continuous --steps 10 --warmup 2" bash tools/gpu_ab_env.sh "MPITREE_EXACT_PART_GROUPS=0"
