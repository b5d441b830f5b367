#!/bin/bash
# GPU call: rocprofv3 kernel trace of bench.py runs -> per-kernel stats and the
# timeline of the last fit. Usage (via gpurun): bash tools/gpu_timeline_bench.sh TAG "bench args"
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  TAG=$1; ARGS=$2; shift 2
  rm -rf gpurun_out/tl_$TAG
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tl_$TAG -o run -- python3 bench.py $ARGS > gpurun_out/tl_$TAG.log 2>&1
  DB=$(find gpurun_out/tl_$TAG -name "*.db" | head -1)
  python3 tools/rocpd_timeline.py "$DB" --n 600 > gpurun_out/tl_$TAG.txt
  python3 tools/rocpd_top.py "$DB" > gpurun_out/tl_$TAG.top.txt 2>&1 || true
  rm -rf gpurun_out/tl_$TAG
done
