#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py runs. Usage (via gpurun):
#   bash tools/gpu_prof_r3.sh TAG "bench args" [TAG2 "bench args2" ...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  TAG=$1; ARGS=$2; shift 2
  rm -rf gpurun_out/prof_$TAG
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py $ARGS > gpurun_out/prof_$TAG.log 2>&1
  find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$TAG.kernel_stats.csv \;
  find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -exec cp {} gpurun_out/prof_$TAG.kernel_trace.csv \;
  rm -rf gpurun_out/prof_$TAG
done
