#!/bin/bash
# GPU call (round 4): one-sweep setup sort -- sort test, exact GPU tests, continuous
# bench and its kernel table.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "setup_sort" > gpurun_out/gputests_x0.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "exact" > gpurun_out/gputests_x.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --continuous --steps 10 --warmup 2 >> gpurun_out/bench_x.log 2>&1
done
rm -rf gpurun_out/kx_ex
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kx_ex -o run -- python3 bench.py --continuous --steps 3 --warmup 1 > gpurun_out/kx_ex.log 2>&1
DB=$(ls gpurun_out/kx_ex/*.db gpurun_out/kx_ex/*/*.db 2>/dev/null | head -1)
python tools/rocpd_top.py "$DB" 25 > gpurun_out/exact_kernels.txt
rm -rf gpurun_out/kx_ex
