#!/bin/bash
# GPU call (round 4, last): rocprofv3 kernel tables of the flagship and exact fits.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "flagship|--steps 5 --warmup 2" "exact|--continuous --steps 3 --warmup 1"; do
  TAG=${cfg%%|*}; ARGS=${cfg#*|}
  rm -rf gpurun_out/kt_$TAG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$TAG -o run -- python3 bench.py $ARGS > gpurun_out/kt_$TAG.log 2>&1
  DB=$(find gpurun_out/kt_$TAG -name "*.db" | head -1)
  python3 tools/rocpd_top.py "$DB" 30 > gpurun_out/kernels_final_$TAG.txt
  STATS=$(find gpurun_out/kt_$TAG -name "*kernel_stats.csv" | head -1)
  [ -n "$STATS" ] && cp "$STATS" gpurun_out/kernel_stats_final_$TAG.csv
  rm -rf gpurun_out/kt_$TAG
done
