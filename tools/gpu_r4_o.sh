#!/bin/bash
# GPU call (round 4): exact engine with the fused two-class scan (look-back chunk
# totals) -- exact GPU tests, then continuous 1M x 64 A/B against xe_tot + xe_carry.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "exact" > gpurun_out/gputests_o.log 2>&1
: > gpurun_out/ab_fused.log
for rep in 1 2; do
  for v in 1 0; do
    echo "fused=$v $(MPITREE_EXACT_FUSED_SCAN=$v timeout -k 10 300 python -u bench.py --continuous --steps 10 --warmup 2 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["tree_nodes"])')" >> gpurun_out/ab_fused.log
  done
done
