#!/bin/bash
# GPU call (round 4): finisher phase profiles, payload path vs gather path.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 1 0; do
  MPITREE_FIN_PAYLOAD=$v MPITREE_FIN_PROF=1 timeout -k 10 200 python -u bench/fin_prof.py > gpurun_out/fin_prof_p$v.log 2>&1
done
