#!/bin/bash
# GPU call (round 4): grid-barrier vs launch-chain probe, finisher phase profile,
# node-size census of the flagship tree.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probes/gridbar_probe 1 200 4096 > gpurun_out/gridbar.log 2>&1
timeout -k 10 60 ./tools/probes/gridbar_probe 2 200 4096 >> gpurun_out/gridbar.log 2>&1
timeout -k 10 60 ./tools/probes/gridbar_probe 1 200 64 >> gpurun_out/gridbar.log 2>&1
timeout -k 10 120 python -u bench/fin_prof.py > gpurun_out/fin_prof.log 2>&1
timeout -k 10 120 python -u bench/node_sizes.py > gpurun_out/node_sizes.log 2>&1
