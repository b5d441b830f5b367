#!/bin/bash
# GPU call (round 4): payload finisher (row codes move with the partition, sibling
# histogram subtraction in place) -- finisher GPU tests, then bench A/B against
# the gather path (MPITREE_FIN_PAYLOAD=0) and the finisher phase profile.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider \
  -k "finisher or device_loop or tiny or classifier or assembly or iris or large_multiitem or many_features" \
  > gpurun_out/gputests_j.log 2>&1
: > gpurun_out/ab_payload.log
for rep in 1 2; do
  for v in 0 1; do
    echo "payload=$v $(MPITREE_FIN_PAYLOAD=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["tree_nodes"])')" >> gpurun_out/ab_payload.log
  done
done
MPITREE_FIN_PROF=1 timeout -k 10 200 python -u bench/fin_prof.py > gpurun_out/fin_prof_payload.log 2>&1 || true
