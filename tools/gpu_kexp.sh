#!/bin/bash
# GPU call: per-kernel averages (rocprofv3 kernel trace of a short flagship bench)
# under each given env setting. Usage: bash tools/gpu_kexp.sh "A=1" "A=2 B=3" ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/kexp.log
i=0
for cfg in "$@"; do
  i=$((i+1))
  rm -rf gpurun_out/kx$i
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/kx$i -o run -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/kx$i.log 2>&1
  DB=$(ls gpurun_out/kx$i/*.db gpurun_out/kx$i/*/*.db 2>/dev/null | head -1)
  echo "== $cfg" >> gpurun_out/kexp.log
  python tools/rocpd_top.py "$DB" 12 | grep "mt::" >> gpurun_out/kexp.log
  rm -rf gpurun_out/kx$i
done
