#!/bin/bash
# Bench-only GPU call: flagship, continuous, regression (no tests).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 >> gpurun_out/bench.log 2>&1
timeout -k 10 180 python -u bench.py --steps 5 --warmup 2 --continuous >> gpurun_out/bench.log 2>&1
timeout -k 10 180 python -u bench.py --steps 5 --warmup 2 --regression >> gpurun_out/bench.log 2>&1
