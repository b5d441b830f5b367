# Level-loop / finisher knob sweeps on the BASELINE shapes; gpurun_out/ab_*.log.
set -e
rm -f gpurun_out/ab.log
BENCH_ARGS="--classes 300 --no-continuous --steps 2 --warmup 1" bash tools/gpu.sh "ab:MPITREE_HIST_ITEMS=2"
mv gpurun_out/ab.log gpurun_out/ab_hi_c300.log
