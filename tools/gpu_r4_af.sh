#!/bin/bash
# GPU call (round 4): exact partition ticket padding for F_loc without a 4..16 divisor
# (F = 67): padded (in-tree) vs unpadded (variants/nopad.so), F = 64 control; tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "exact" > gpurun_out/gputests_af.log 2>&1
BENCH_ARGS="--continuous --n 500000 --features 67 --steps 5 --warmup 2" timeout -k 10 600 bash tools/gpu_ab_so.sh nopad
cp gpurun_out/ab_so.log gpurun_out/ab_pad67.log
BENCH_ARGS="--continuous --steps 10 --warmup 2" timeout -k 10 600 bash tools/gpu_ab_so.sh nopad
cp gpurun_out/ab_so.log gpurun_out/ab_pad64.log
