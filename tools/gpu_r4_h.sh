#!/bin/bash
# GPU call (round 4): histogram item size A/B (MPITREE_HIST_ITEMS = 2 items per CU
# vs 1 larger item per CU) on the flagship: bench ms and per-kernel averages.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab_hist_items.log
for rep in 1 2; do
  for v in 2 1; do
    echo "items=$v $(MPITREE_HIST_ITEMS=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["tree_nodes"])')" >> gpurun_out/ab_hist_items.log
  done
done
bash tools/gpu_kexp.sh "MPITREE_HIST_ITEMS=2" "MPITREE_HIST_ITEMS=1"
