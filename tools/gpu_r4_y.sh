#!/bin/bash
# GPU call (round 4): setup sort (reduce-then-scan) -- test, timing, kernel table,
# exact GPU tests and the continuous bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "setup_sort" > gpurun_out/gputests_y0.log 2>&1 && MPITREE_SORT_TILE=16384 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "setup_sort" >> gpurun_out/gputests_y0.log 2>&1
: > gpurun_out/sort_probe.log
for tl in 8192 16384 8192 16384; do MPITREE_SORT_TILE=$tl timeout -k 10 120 python bench/setup_sort_probe.py >> gpurun_out/sort_probe.log 2>&1; done
rm -rf gpurun_out/kx_sp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/kx_sp -o run -- python3 bench/setup_sort_probe.py > gpurun_out/kx_sp.log 2>&1
DB=$(ls gpurun_out/kx_sp/*.db gpurun_out/kx_sp/*/*.db 2>/dev/null | head -1)
python tools/rocpd_top.py "$DB" 12 > gpurun_out/sort_kernels.txt
rm -rf gpurun_out/kx_sp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "exact" > gpurun_out/gputests_y.log 2>&1
: > gpurun_out/bench_y.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --continuous --steps 10 --warmup 2 >> gpurun_out/bench_y.log 2>&1
done
