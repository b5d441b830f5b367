#!/bin/bash
# Multi-rank rehearsal of bench.py on the one-GPU box: 2 and 4 ranks share the
# card, collectives over gloo (RCCL refuses two ranks on one GPU).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for P in 2 4; do
  MPITREE_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $P --master-addr 127.0.0.1 --master-port 2951$P bench.py --gpus $P \
    --steps 5 --warmup 2 > gpurun_out/bench_gloo$P.log 2>&1
done
