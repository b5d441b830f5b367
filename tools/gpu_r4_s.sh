#!/bin/bash
# GPU call (round 4): flagship re-sweeps after this round's finisher changes --
# finisher compile-time variants and the finisher job size.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "assembly or classifier or predict or proba or iris or many or oracle or export or feature_parallel or exact_feature" \
  > gpurun_out/gputests_s.log 2>&1
bash tools/gpu_ab_so.sh unroll8 unroll2 pair2 handoff4
cp gpurun_out/ab_so.log gpurun_out/ab_fin_variants.log
bash tools/gpu_ab_env.sh "MPITREE_FINISHER_ROWS=4096" "MPITREE_FINISHER_ROWS=12000" "MPITREE_FINISHER_ROWS=16384"
