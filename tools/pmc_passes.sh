#!/bin/bash
# PMC counter passes over one flagship fit (bench/pmc_fit.py); one rocprofv3 run per pass,
# each within the per-block slot limits (SQ 8, TCC 4: FETCH_SIZE and WRITE_SIZE apart).
# Summarise: python tools/pmc_report.py --fits 2 gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmc1 -o run -- python bench/pmc_fit.py > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc2 -o run -- python bench/pmc_fit.py > gpurun_out/pmc2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc3 -o run -- python bench/pmc_fit.py > gpurun_out/pmc3.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc4 -o run -- python bench/pmc_fit.py > gpurun_out/pmc4.log 2>&1
