#!/bin/bash
# GPU call (round 4): exact engine GPU tests + staged-partition A/B (continuous
# 1M x 64) + its PMC bytes; multi-rank ownership sim with the new unit default.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "exact or distributed" > gpurun_out/gputests_g.log 2>&1
: > gpurun_out/ab_stage.log
for rep in 1 2; do
  for v in 0 1; do
    echo "stage=$v $(MPITREE_EXACT_PART_STAGE=$v timeout -k 10 300 python -u bench.py --continuous --steps 10 --warmup 2 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["tree_nodes"])')" >> gpurun_out/ab_stage.log
  done
done
PMC_EXACT=1 bash tools/pmc_bytes.sh exact_staged
