#!/bin/bash
# GPU call (round 4): kernel table of the continuous (exact) 1M x 64 fit.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/kx_ex
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kx_ex -o run -- python3 bench.py --continuous --steps 3 --warmup 1 > gpurun_out/kx_ex.log 2>&1
DB=$(ls gpurun_out/kx_ex/*.db gpurun_out/kx_ex/*/*.db 2>/dev/null | head -1)
python tools/rocpd_top.py "$DB" 25 > gpurun_out/exact_kernels.txt
rm -rf gpurun_out/kx_ex
