#!/bin/bash
# GPU call: the full GPU test suite, every BASELINE configuration's bench line,
# rocprofv3 kernel tables of each, the finisher phase profile and two PMC passes
# over the flagship fit. Outputs land in gpurun_out/ (copy summaries to profiles/).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_tests.sh
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --regression > gpurun_out/bench_reg.log 2>&1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --n 10000000 --features 128 --strategy data > gpurun_out/bench_10m.log 2>&1
timeout -k 10 300 python -u bench/baseline_configs.py iris sweep_gpu 100k 1m 1m_exact 1m_reg 10m --reps 5 > gpurun_out/baseline_configs.jsonl 2>&1
bash tools/gpu_prof_configs.sh fin flagship reg 10m exact
bash tools/pmc_two.sh
