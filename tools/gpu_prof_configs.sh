#!/bin/bash
# GPU call: rocprofv3 kernel traces of the BASELINE configurations (flagship,
# regression, 10M x 128 data-parallel on one rank, 1M x 64 exact thresholds) and
# the block finisher's phase profile.
# Usage: tools/gpu_prof_configs.sh [flagship] [reg] [10m] [exact] [fin]   (default: all)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(fin flagship reg 10m exact)
prof() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  rm -rf "gpurun_out/prof_$name"
  timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$name" -o run -- "$@" \
    > "gpurun_out/prof_$name.log" 2>&1
  local db
  db=$(find "gpurun_out/prof_$name" -name 'run_results.db' -print -quit)
  if [ -n "$db" ]; then
    python tools/rocpd_top.py "$db" 40 > "gpurun_out/prof_$name.top.txt"
    python tools/rocpd_summary.py "$db" > "gpurun_out/prof_$name.summary.md"
    python tools/rocpd_timeline.py "$db" --n 120 > "gpurun_out/prof_$name.timeline.txt" || true
  fi
  find "gpurun_out/prof_$name" -name '*kernel_stats.csv' -exec cp {} "gpurun_out/prof_$name.kernel_stats.csv" \;
  rm -rf "gpurun_out/prof_$name"  # the databases exceed what gpurun copies back
}
for a in "${ARGS[@]}"; do
  case $a in
    fin) timeout -k 10 120 python -u bench/fin_prof.py > gpurun_out/fin_prof.log 2>&1 ;;
    flagship) prof flagship 180 python3 bench.py --steps 5 --warmup 2 ;;
    reg) prof reg 240 python3 bench.py --steps 3 --warmup 1 --regression ;;
    10m) prof 10m 300 python3 bench.py --steps 2 --warmup 1 --n 10000000 --features 128 --strategy data ;;
    exact) prof exact 300 python3 bench/baseline_configs.py 1m_exact --reps 2 ;;
  esac
done
