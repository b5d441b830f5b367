#!/bin/bash
# GPU call (round 4): GPU suite, benches of the cliff shapes, C = 64 timeline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gputests.log 2>&1
: > gpurun_out/bench_d.log
for args in "" "--classes 64 --steps 3" "--n 200000 --features 512" "--continuous --steps 10" \
            "--regression --steps 10"; do
  echo "args=$args $(timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 $args 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["tree_nodes"], d["config"]["engine"])')" >> gpurun_out/bench_d.log
done
bash tools/gpu_timeline_bench.sh c64 "--steps 2 --warmup 3 --classes 64"
