# Finisher job-size sweeps (MPITREE_FINISHER_ROWS) on the BASELINE shapes; results
# in gpurun_out/ab_*.log (copied to profiles/r6/).
set -e
rm -f gpurun_out/ab.log
BENCH_ARGS="--n 100000 --features 32 --max-depth 12 --no-continuous --steps 20 --warmup 3" bash tools/gpu.sh "ab:MPITREE_FINISHER_ROWS=4096;MPITREE_FINISHER_ROWS=8192;MPITREE_FINISHER_ROWS=16384"
mv gpurun_out/ab.log gpurun_out/ab_100k_b.log
BENCH_ARGS="--n 100000 --features 32 --no-continuous --steps 20 --warmup 3" bash tools/gpu.sh "ab:MPITREE_FINISHER_ROWS=4096;MPITREE_FINISHER_ROWS=8192"
mv gpurun_out/ab.log gpurun_out/ab_100k_full.log
