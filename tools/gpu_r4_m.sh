#!/bin/bash
# GPU call (round 4): many-class tiny kernel (per-node class lists): tests + C = 64 bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider \
  -k "finisher or device_loop or tiny or classifier or many" > gpurun_out/gputests_m.log 2>&1
timeout -k 10 300 python -u bench.py --classes 64 --steps 3 --warmup 1 > gpurun_out/bench_c64.log 2>&1
FIN_PROF_CLASSES=64 MPITREE_FIN_PROF=1 timeout -k 10 300 python -u bench/fin_prof.py > gpurun_out/fin_prof_c64.log 2>&1
BENCH_ARGS="--classes 64 --steps 2 --warmup 1" bash tools/gpu_ab_env.sh "MPITREE_FINISHER_ROWS=512" "MPITREE_FINISHER_ROWS=1024" "MPITREE_FINISHER_ROWS=4096"
