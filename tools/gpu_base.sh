#!/bin/bash
# Baseline GPU call: GPU test suite + flagship bench (+ optional extra bench args).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
