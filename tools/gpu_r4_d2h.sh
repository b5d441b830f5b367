#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/d2h.log
timeout -k 10 60 python -u tools/probes/d2h_probe.py >> gpurun_out/d2h.log 2>&1
HSA_ENABLE_SDMA=0 timeout -k 10 60 python -u tools/probes/d2h_probe.py >> gpurun_out/d2h.log 2>&1
GPU_FORCE_BLIT_COPY_SIZE=0 timeout -k 10 60 python -u tools/probes/d2h_probe.py >> gpurun_out/d2h.log 2>&1
