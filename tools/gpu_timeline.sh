#!/bin/bash
# GPU call: rocprofv3 kernel trace of the flagship bench and the full dispatch
# timeline of its last fit (gpurun_out/timeline.txt) plus the kernel summary.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS=${1:-}
rm -rf gpurun_out/prof_tl
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_tl -o run -- python3 bench.py --steps 5 --warmup 2 $ARGS > gpurun_out/prof_tl.log 2>&1
DB=$(ls gpurun_out/prof_tl/*.db gpurun_out/prof_tl/*/*.db 2>/dev/null | head -1)
python tools/rocpd_timeline.py "$DB" --n 400 > gpurun_out/timeline.txt 2>&1
python tools/rocpd_top.py "$DB" > gpurun_out/top.txt 2>&1 || true
