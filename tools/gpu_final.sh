#!/bin/bash
# GPU call: what the driver runs at round end (GPU suite, smoke, 1-GPU bench),
# plus the regression and 10M x 128 bench lines and the flagship kernel table.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_tests.sh
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --regression > gpurun_out/bench_reg.log 2>&1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --n 10000000 --features 128 --strategy data > gpurun_out/bench_10m.log 2>&1
bash tools/gpu_prof_configs.sh flagship reg
