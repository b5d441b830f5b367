#!/bin/bash
# GPU call (round 4): exact engine with byte flags -- exact + distributed GPU tests,
# probe test, then A/B against the bit atomics.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "exact or distributed or probe" > gpurun_out/gputests_aa.log 2>&1
BENCH_ARGS="--continuous --steps 10 --warmup 2" bash tools/gpu_ab_env.sh "MPITREE_EXACT_FLAG_BYTES=0"
