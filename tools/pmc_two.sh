#!/bin/bash
# Two PMC passes (issue/wait + LDS) over bench/pmc_fit.py; env (PMC_REG, PMC_N, PMC_F) passes through.
# Summarise: python tools/pmc_report.py --fits 2 gpurun_out/pmcA gpurun_out/pmcB
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/pmcA gpurun_out/pmcB
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmcA -o run -- python bench/pmc_fit.py > gpurun_out/pmcA.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmcB -o run -- python bench/pmc_fit.py > gpurun_out/pmcB.log 2>&1
python tools/pmc_report.py --fits 2 gpurun_out/pmcA gpurun_out/pmcB > gpurun_out/pmc_report.md
