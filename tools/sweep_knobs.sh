# Level-loop / finisher knob sweeps on the BASELINE shapes; gpurun_out/ab_*.log.
set -e
rm -f gpurun_out/ab.log
BENCH_ARGS="--regression --no-continuous --steps 10 --warmup 2" bash tools/gpu.sh "ab:MPITREE_FIN_GRID=256;MPITREE_FIN_GRID=512;MPITREE_FIN_GRID=1024"
mv gpurun_out/ab.log gpurun_out/ab_reg_grid.log
BENCH_ARGS="--classes 300 --no-continuous --steps 2 --warmup 1" bash tools/gpu.sh "ab:MPITREE_TINY_LPT=0"
mv gpurun_out/ab.log gpurun_out/ab_c300_lpt.log
