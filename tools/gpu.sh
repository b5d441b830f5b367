#!/bin/bash
# The one GPU runner (replaces the round-3/4 one-shot tools/gpu_*.sh scripts).
#
#   gpurun -- bash tools/gpu.sh STEP [STEP ...]
#
# Every step runs under its own time limit and the chain stops at the first
# failing step (set -e): after a fault, an abort or a time limit nothing more
# touches the GPU in that call. Outputs land in gpurun_out/ (copy the summaries
# worth keeping to profiles/). Steps (arguments after ':' separated by ','):
#
#   tests[:K]            GPU test suite (optionally pytest -k K)       -> gputests.log
#   dist                 distributed GPU tests (gloo ranks, one card)  -> gputests_dist.log
#   bench[:ARGS]         bench.py --steps 20 --warmup 3 ARGS           -> bench.log (appended)
#   ab:CFG1;CFG2;...     bench under each setting, alternated twice     -> ab.log
#                        (CFG: "ENV=1 ENV2=x"; "so=NAME" swaps in variants/NAME.so from
#                        tools/build_variant.sh; "dir=PATH" runs PATH/bench.py, a whole
#                        tree from tools/snapshot_tree.sh; BENCH_ARGS: extra bench.py args)
#   configs[:NAMES]      bench/baseline_configs.py NAMES --reps 5       -> baseline_configs.jsonl
#   prof:NAME[:ARGS]     rocprofv3 kernel trace + stats of bench.py ARGS
#                        -> prof_NAME.{top,summary,timeline,lastfit}.txt, kernel_stats.csv
#   profpy:NAME:SCRIPT[:ARGS]  the same for python3 SCRIPT ARGS (e.g. bench/sim_own_ranks.py)
#   fin                  block-finisher phase profile (bench/fin_prof.py) -> fin_prof.log
#   pmc[:ARGS]           two PMC passes over bench/pmc_fit.py ARGS      -> pmc_report.md
#   sim:ARGS             bench/sim_own_ranks.py ARGS                    -> sim_own.jsonl
#   simx:ARGS            bench/sim_exact_ranks.py ARGS                  -> sim_exact.jsonl
#   simdp:ARGS           bench/sim_dp_ranks.py ARGS (data parallel)     -> sim_dp.jsonl
#   py:SCRIPT[:ARGS]     python -u SCRIPT ARGS (150 s)                  -> py_<script>.log
#
# ARGS use ',' for spaces: "bench:--continuous,--steps,10" runs
# bench.py --steps 20 --warmup 3 --continuous --steps 10 (argparse: last wins).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out

args_of() { echo "${1//,/ }"; }

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
    python tools/rocpd_timeline.py "$db" --n 400 > "gpurun_out/prof_$name.timeline.txt" || true
    python tools/rocpd_timeline.py "$db" --agg > "gpurun_out/prof_$name.lastfit.txt" || true
  fi
  find "gpurun_out/prof_$name" -name '*kernel_stats.csv' -exec cp {} "gpurun_out/prof_$name.kernel_stats.csv" \;
  rm -rf "gpurun_out/prof_$name"  # the databases exceed what gpurun copies back
}

for step in "$@"; do
  name=${step%%:*}
  rest=""
  [ "$name" != "$step" ] && rest=${step#*:}
  echo "== step $step ($(date +%T))"
  case $name in
    tests)
      if [ -n "$rest" ]; then
        timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
          -p no:cacheprovider -k "$rest" > gpurun_out/gputests.log 2>&1
      else
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
          -p no:cacheprovider > gpurun_out/gputests.log 2>&1
      fi ;;
    dist)
      timeout -k 10 600 python -u -m pytest tests/test_distributed.py -m gpu -x -v --timeout 240 \
        --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_dist.log 2>&1 ;;
    bench)
      # shellcheck disable=SC2046
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 $(args_of "$rest") \
        >> gpurun_out/bench.log 2>> gpurun_out/bench.err ;;
    ab)
      IFS=';' read -r -a cfgs <<< "$rest"
      SO=$(ls mpitree_amd/_hip*.so)
      cp "$SO" gpurun_out/.base.so
      for rep in 1 2; do
        for cfg in "base=1" "${cfgs[@]}"; do
          echo "== $cfg" >> gpurun_out/ab.log
          envs=$cfg
          script=bench.py
          if [[ $cfg == so=* ]]; then cp "variants/${cfg#so=}.so" "$SO"; envs="base=1"; fi
          if [[ $cfg == dir=* ]]; then script="${cfg#dir=}/bench.py"; envs="base=1"; fi
          # shellcheck disable=SC2086
          env $envs timeout -k 10 150 python -u "$script" --steps 20 --warmup 3 $BENCH_ARGS \
            2>>gpurun_out/ab.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); \
print(d['ms_per_step'], d['config']['tree_nodes'])" >> gpurun_out/ab.log
          cp gpurun_out/.base.so "$SO"
        done
      done
      rm -f gpurun_out/.base.so ;;
    configs)
      # shellcheck disable=SC2046
      timeout -k 10 900 python -u bench/baseline_configs.py $(args_of "$rest") --reps 5 \
        >> gpurun_out/baseline_configs.jsonl 2>> gpurun_out/baseline_configs.err ;;
    prof)
      pname=${rest%%:*}
      pargs=""
      [ "$pname" != "$rest" ] && pargs=${rest#*:}
      # shellcheck disable=SC2046
      prof "$pname" 240 python3 bench.py --steps 5 --warmup 2 $(args_of "$pargs") ;;
    profpy)
      pname=${rest%%:*}
      r2=${rest#*:}
      script=${r2%%:*}
      sargs=""
      [ "$script" != "$r2" ] && sargs=${r2#*:}
      # shellcheck disable=SC2046
      prof "$pname" 300 python3 "$script" $(args_of "$sargs") ;;
    fin)
      timeout -k 10 150 python -u bench/fin_prof.py > gpurun_out/fin_prof.log 2>&1 ;;
    pmc)
      rm -rf gpurun_out/pmcA gpurun_out/pmcB
      # shellcheck disable=SC2046
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace \
        --output-format csv -d gpurun_out/pmcA -o run -- python bench/pmc_fit.py $(args_of "$rest") \
        > gpurun_out/pmcA.log 2>&1
      # shellcheck disable=SC2046
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
        SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM \
        --output-format csv -d gpurun_out/pmcB -o run -- python bench/pmc_fit.py $(args_of "$rest") \
        > gpurun_out/pmcB.log 2>&1
      python tools/pmc_report.py --fits 2 gpurun_out/pmcA gpurun_out/pmcB > gpurun_out/pmc_report.md ;;
    sim)
      # shellcheck disable=SC2046
      timeout -k 10 400 python -u bench/sim_own_ranks.py $(args_of "$rest") \
        >> gpurun_out/sim_own.jsonl 2>> gpurun_out/sim_own.err ;;
    simx)
      # shellcheck disable=SC2046
      timeout -k 10 400 python -u bench/sim_exact_ranks.py $(args_of "$rest") \
        >> gpurun_out/sim_exact.jsonl 2>> gpurun_out/sim_exact.err ;;
    simdp)
      # shellcheck disable=SC2046
      timeout -k 10 600 python -u bench/sim_dp_ranks.py $(args_of "$rest") \
        >> gpurun_out/sim_dp.jsonl 2>> gpurun_out/sim_dp.err ;;
    py)
      script=${rest%%:*}
      sargs=""
      [ "$script" != "$rest" ] && sargs=${rest#*:}
      base=$(basename "$script" .py)
      # shellcheck disable=SC2046
      timeout -k 10 150 python -u "$script" $(args_of "$sargs") > "gpurun_out/py_$base.log" 2>&1 ;;
    *)
      echo "tools/gpu.sh: unknown step '$step'" >&2
      exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
