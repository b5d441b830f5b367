#!/bin/bash
# GPU call: rocprofv3 kernel timeline of one simulated rank of a P-GPU
# subtree-ownership fit (bench/sim_own_ranks.py --only-rank), plus the 1-GPU fit.
# Usage (via gpurun): bash tools/gpu_timeline_own.sh P RANK
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
P=${1:-8}; R=${2:-0}
rm -rf gpurun_out/tl_own
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tl_own -o run -- python3 bench/sim_own_ranks.py --ranks $P --only-rank $R --reps 3 > gpurun_out/tl_own.log 2>&1
DB=$(find gpurun_out/tl_own -name "*.db" | head -1)
python3 tools/rocpd_timeline.py "$DB" --n 400 > gpurun_out/tl_own_P${P}r${R}.txt
rm -rf gpurun_out/tl_own
