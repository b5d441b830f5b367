# Finisher job-size sweeps (MPITREE_FINISHER_ROWS) on the BASELINE shapes; results
# in gpurun_out/ab_*.log (copied to profiles/r6/).
set -e
rm -f gpurun_out/ab.log
BENCH_ARGS="--continuous --max-bins 1024 --steps 5 --warmup 2" bash tools/gpu.sh "ab:MPITREE_FINISHER_ROWS=1024;MPITREE_FINISHER_ROWS=2048;MPITREE_FINISHER_ROWS=3000"
mv gpurun_out/ab.log gpurun_out/ab_q1024b.log
BENCH_ARGS="--n 200000 --features 512 --no-continuous --steps 10 --warmup 2" bash tools/gpu.sh "ab:MPITREE_FINISHER_ROWS=256;MPITREE_FINISHER_ROWS=320;MPITREE_FINISHER_ROWS=384"
mv gpurun_out/ab.log gpurun_out/ab_f512b.log
