#!/bin/bash
# GPU call (round 4): 200k x 512 regression hunt (round-3 finisher / scan sources
# swapped in) + the current C = 64 and 200k x 512 numbers.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--n 200000 --features 512" bash tools/gpu_ab_so.sh fin_r3 scan_r3
cp gpurun_out/ab_so.log gpurun_out/ab_512.log
BENCH_ARGS="--classes 64 --steps 3" bash tools/gpu_ab_so.sh fin_r3 scan_r3
cp gpurun_out/ab_so.log gpurun_out/ab_c64.log
