#!/bin/bash
# GPU call (round 4, end): the full GPU suite, every BASELINE configuration
# (profiles/r4/baseline_configs_r4c.jsonl) and the flagship bench line.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gputests_final3.log 2>&1
timeout -k 10 600 python -u bench/baseline_configs.py --reps 5 > gpurun_out/baseline_configs_r4c.jsonl 2> gpurun_out/baseline_configs_r4c.err
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_final3.log 2>&1
