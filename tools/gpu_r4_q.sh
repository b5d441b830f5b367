#!/bin/bash
# GPU call (round 4): many-class finisher with 8-bit counts for <= 255-row nodes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "finisher or device_loop or tiny or classifier or many or wide or published or small" \
  > gpurun_out/gputests_q.log 2>&1
timeout -k 10 300 python -u bench.py --classes 64 --steps 3 --warmup 1 > gpurun_out/bench_c64.log 2>&1
FIN_PROF_CLASSES=64 MPITREE_FIN_PROF=1 timeout -k 10 300 python -u bench/fin_prof.py > gpurun_out/fin_prof_c64.log 2>&1
bash tools/gpu_ab_so.sh head nofence
