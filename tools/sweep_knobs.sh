# Level-loop / finisher knob sweeps on the BASELINE shapes; gpurun_out/ab_*.log.
set -e
rm -f gpurun_out/ab.log
BENCH_ARGS="--no-continuous --steps 20 --warmup 3" bash tools/gpu.sh "ab:MPITREE_HIST_ITEMS=1"
mv gpurun_out/ab.log gpurun_out/ab_hi_flag.log
BENCH_ARGS="--n 100000 --features 32 --max-depth 12 --no-continuous --steps 20 --warmup 3" bash tools/gpu.sh "ab:MPITREE_HIST_ITEMS=1"
mv gpurun_out/ab.log gpurun_out/ab_hi_100k.log
BENCH_ARGS="--n 200000 --features 512 --no-continuous --steps 10 --warmup 2" bash tools/gpu.sh "ab:MPITREE_HIST_ITEMS=1"
mv gpurun_out/ab.log gpurun_out/ab_hi_f512.log
BENCH_ARGS="--continuous --max-bins 1024 --steps 5 --warmup 2" bash tools/gpu.sh "ab:MPITREE_HIST_ITEMS=1"
mv gpurun_out/ab.log gpurun_out/ab_hi_q1024.log
