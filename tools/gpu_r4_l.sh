#!/bin/bash
# GPU call (round 4): payload finisher with / without in-place sibling subtraction
# (variants/nosub.so) against the gather path, plus the no-subtraction profile.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_ab_so.sh nosub
for rep in 1 2; do
  echo "gather $(MPITREE_FIN_PAYLOAD=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["tree_nodes"])')" >> gpurun_out/ab_so.log
done
SO=$(ls mpitree_amd/_hip*.so); cp "$SO" /tmp/base.so; cp variants/nosub.so "$SO"
MPITREE_FIN_PROF=1 timeout -k 10 200 python -u bench/fin_prof.py > gpurun_out/fin_prof_nosub.log 2>&1 || true
cp /tmp/base.so "$SO"
