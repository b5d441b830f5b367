#!/bin/bash
# Short GPU probes: pinned-copy costs and a flagship fit phase breakdown.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u bench/pinned_probe.py > gpurun_out/probe.log 2>&1
