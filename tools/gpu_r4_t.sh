#!/bin/bash
# GPU call (round 4): two-class exact engine with partition-counted chunk totals (no
# xe_tot pass after level 0) -- exact GPU tests (1 and multi-rank), continuous A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "exact" > gpurun_out/gputests_t.log 2>&1
: > gpurun_out/ab_part_tot.log
for rep in 1 2; do
  for v in 1 0; do
    echo "part_tot=$v $(MPITREE_EXACT_PART_TOT=$v timeout -k 10 300 python -u bench.py --continuous --steps 10 --warmup 2 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["tree_nodes"])')" >> gpurun_out/ab_part_tot.log
  done
done
