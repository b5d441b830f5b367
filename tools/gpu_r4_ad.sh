#!/bin/bash
# GPU call (round 4): batched wave claims (tiny kernels, exact partition exit claims) --
# full GPU suite, flagship + exact benches, small exact timeline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests_ad.log 2>&1
: > gpurun_out/bench_ad.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 >> gpurun_out/bench_ad.log 2>&1
  timeout -k 10 200 python bench.py --continuous --steps 10 --warmup 2 >> gpurun_out/bench_ad.log 2>&1
  timeout -k 10 200 python bench.py --continuous --n 100000 --features 32 --max-depth 12 --steps 10 --warmup 2 >> gpurun_out/bench_ad.log 2>&1
done
bash tools/gpu_timeline_bench.sh small "--continuous --n 100000 --features 32 --max-depth 12 --steps 3 --warmup 2" flag "--steps 3 --warmup 2"
