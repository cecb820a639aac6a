#!/bin/bash
# One GPU call: parity tests, smoke, bench, rocprofv3 kernel trace.  Each GPU step has its own
# time limit; test failures (exit 1) do not stop the chain, crashes/timeouts (>=124) do.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a $OUT/steps.log
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name; stopping" | tee -a $OUT/steps.log; exit $rc; fi
  return 0
}
STEPS=,${STEPS:-tests,smoke,bench,prof},
[[ $STEPS == *,tests,* ]] && step tests 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300
[[ $STEPS == *,smoke,* ]] && step smoke 300 python __graft_entry__.py smoke
[[ $STEPS == *,bench,* ]] && step bench 600 python bench.py
[[ $STEPS == *,prof,* ]] && step prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline
[[ $STEPS == *,pmcF,* ]] && step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
[[ $STEPS == *,pmcW,* ]] && step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
[[ $STEPS == *,cfgs,* ]] && step cfgs 900 python tools/bench_configs.py
[[ $STEPS == *,sol,* ]] && step sol 120 tools/bin/sol_stream
[[ $STEPS == *,cfgprof,* ]] && step cfgprof 900 rocprofv3 --kernel-trace --stats -d $OUT/cfgprof -o cfgs --output-format csv -- python3 tools/bench_configs.py --steps 5 --warmup 1
echo "=== done" | tee -a $OUT/steps.log
