#!/bin/bash
# GPU call: feature-parallel per-rank simulation, every BASELINE configuration's
# measured row, and rocprofv3 kernel tables of each configuration.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 240 python -u bench/sim_fp_ranks.py > gpurun_out/sim_fp.jsonl 2> gpurun_out/sim_fp.err
timeout -k 10 300 python -u bench/baseline_configs.py iris sweep_gpu 100k 1m 1m_exact 1m_reg 10m --reps 5 > gpurun_out/baseline_configs.jsonl 2>&1
bash tools/gpu_prof_configs.sh fin flagship reg 10m exact
