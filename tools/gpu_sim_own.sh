#!/bin/bash
# GPU call: distributed GPU tests (gloo ranks sharing the card) + the per-rank
# subtree-ownership simulation. Usage (via gpurun): bash tools/gpu_sim_own.sh [sim args]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_distributed.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_dist.log 2>&1
fi
timeout -k 10 400 python -u bench/sim_own_ranks.py "$@" > gpurun_out/sim_own.jsonl 2> gpurun_out/sim_own.err
