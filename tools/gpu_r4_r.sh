#!/bin/bash
# GPU call (round 4): C = 64 kernel table (8-bit small-node histograms + 128-row waves).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/kx_c64
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kx_c64 -o run -- python3 bench.py --classes 64 --steps 2 --warmup 1 > gpurun_out/kx_c64.log 2>&1
DB=$(ls gpurun_out/kx_c64/*.db gpurun_out/kx_c64/*/*.db 2>/dev/null | head -1)
python tools/rocpd_top.py "$DB" 12 > gpurun_out/c64_kernels.txt
rm -rf gpurun_out/kx_c64
BENCH_ARGS="--classes 64 --steps 2 --warmup 1" bash tools/gpu_ab_env.sh "MPITREE_TINY_ROWS=64" "MPITREE_FINISHER_ROWS=2048"
