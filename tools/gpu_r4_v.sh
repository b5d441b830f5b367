#!/bin/bash
# GPU call (round 4): exact partition with global row-direction flags (2 workgroups
# per CU) vs the LDS flag copy (1 per CU).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BENCH_ARGS="--continuous --steps 10 --warmup 2" bash tools/gpu_ab_env.sh "MPITREE_EXACT_PART_LDS=0" "MPITREE_EXACT_PART_STAGE=0" "MPITREE_EXACT_PART_LDS=0 MPITREE_EXACT_PART_STAGE=0"
