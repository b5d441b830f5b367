# Level-loop / finisher knob sweeps on the BASELINE shapes; gpurun_out/ab_*.log.
set -e
rm -f gpurun_out/ab.log
BENCH_ARGS="--classes 300 --no-continuous --steps 2 --warmup 1" bash tools/gpu.sh "ab:so=nohcap"
mv gpurun_out/ab.log gpurun_out/ab_hcap_c300.log
BENCH_ARGS="--classes 64 --no-continuous --steps 5 --warmup 2" bash tools/gpu.sh "ab:so=nohcap"
mv gpurun_out/ab.log gpurun_out/ab_hcap_c64.log
BENCH_ARGS="--no-continuous --steps 20 --warmup 3" bash tools/gpu.sh "ab:so=nohcap"
mv gpurun_out/ab.log gpurun_out/ab_hcap_flag.log
