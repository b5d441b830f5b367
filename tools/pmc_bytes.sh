#!/bin/bash
# Four PMC passes over bench/pmc_fit.py (env PMC_REG / PMC_EXACT / PMC_N / PMC_F pass
# through): issue / wait buckets, LDS conflicts, then FETCH_SIZE and WRITE_SIZE in passes of
# their own (FETCH_SIZE takes 3 of the 4 TCC slots, WRITE_SIZE 2). Each pass runs under its
# own kill timeout. Report: gpurun_out/pmc_report_<TAG>.md
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-flag}
for p in A B C D; do rm -rf gpurun_out/pmc$p; done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmcA -o run -- python bench/pmc_fit.py > gpurun_out/pmcA.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmcB -o run -- python bench/pmc_fit.py > gpurun_out/pmcB.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcC -o run -- python bench/pmc_fit.py > gpurun_out/pmcC.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcD -o run -- python bench/pmc_fit.py > gpurun_out/pmcD.log 2>&1
python tools/pmc_report.py --fits 2 gpurun_out/pmcA gpurun_out/pmcB gpurun_out/pmcC gpurun_out/pmcD > gpurun_out/pmc_report_$TAG.md
for p in A B C D; do rm -rf gpurun_out/pmc$p; done
