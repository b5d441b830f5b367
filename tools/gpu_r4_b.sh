#!/bin/bash
# GPU call (round 4): probes + the exact-engine GPU tests + regression ownership sim.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_probe_r4.sh
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "exact or many_classes or n_classes or wide_features" \
  > gpurun_out/gputests_exact.log 2>&1
timeout -k 10 120 python -u bench.py --continuous --steps 10 --warmup 2 > gpurun_out/bench_cont.log 2>&1
timeout -k 10 300 python -u bench/sim_own_ranks.py --regression --reps 3 > gpurun_out/sim_own_reg.log 2>&1
