#!/bin/bash
# GPU call: flagship bench under several env settings (A/B), then the timeline
# profile of the default path. Usage: bash tools/gpu_ab.sh "ENV=1" "ENV=2" ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab.log
for cfg in "" "$@" ""; do
  echo "== $cfg" >> gpurun_out/ab.log
  env $cfg timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])" >> gpurun_out/ab.log
done
bash tools/gpu_timeline.sh
