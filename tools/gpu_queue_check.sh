set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_q.log 2>&1
MPITREE_TINY_QUEUE=0 timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_noq.log 2>&1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 >> gpurun_out/bench_q.log 2>&1
rm -rf gpurun_out/prof_q
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_q.log 2>&1
