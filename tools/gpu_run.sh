#!/bin/bash
# One parameterised GPU call (replaces the per-call tools/r02*.sh scripts of round 2).
#
#   tools/gpu_run.sh TAG STEP [STEP ...]
#
# A STEP is "name:limit_s:command ..." (command runs from the repo root, output to
# gpurun_out/TAG_name.log) or one of the shorthands:
#   tests        pytest -m gpu (thread timeouts, so a hang names its test)
#   smoke        __graft_entry__.py smoke
#   bench        python bench.py (the driver's default line)
#   prof         rocprofv3 --kernel-trace --stats of bench.py (gpurun_out/TAG_prof/)
#   pmcF / pmcW  FETCH_SIZE / WRITE_SIZE passes of bench.py (one counter group per pass)
#   cfgs         tools/bench_configs.py (every secondary config)
#   sq:CONFIGS   SQ instruction / wait counters of tools/bench_configs.py --configs CONFIGS
#   sq2:CONFIGS  second SQ group (active / LDS / bank conflicts) + GRBM_GUI_ACTIVE
#   kt:CONFIGS   rocprofv3 --kernel-trace --stats of tools/bench_configs.py --configs CONFIGS
#
# Every GPU step runs under its own time limit; a test failure (rc 1) does not stop the chain,
# anything else non-zero does (fault, abort, timeout: start nothing more on the GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}; shift
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
SQ2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
BC="python3 tools/bench_configs.py --steps 3 --warmup 1"

run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $TAG/$name ($(date +%T)): $*" | tee -a $OUT/${TAG}_steps.log
  timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $TAG/$name rc=$rc" | tee -a $OUT/${TAG}_steps.log
  tail -2 "$OUT/${TAG}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name; stopping" | tee -a $OUT/${TAG}_steps.log; exit $rc; fi
  if [ $rc -eq 1 ] && [[ $name != tests* ]]; then echo "rc=1 in $name; stopping" | tee -a $OUT/${TAG}_steps.log; exit 1; fi
  return 0
}

for S in "$@"; do
  case "$S" in
    tests)  run tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    tests:*) run tests 900 python -u -m pytest ${S#tests:} -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke)  run smoke 300 python __graft_entry__.py smoke ;;
    bench)  run bench 600 python bench.py ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o bench --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline ;;
    pmcF)   run pmcF 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/${TAG}_pmcF -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    pmcW)   run pmcW 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/${TAG}_pmcW -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    cfgs)   run cfgs 900 python3 tools/bench_configs.py ;;
    cfgs:*) run cfgs 900 python3 tools/bench_configs.py --configs ${S#cfgs:} ;;
    sq:*)   run sq_${S#sq:} 150 rocprofv3 --pmc $SQ1 -d $OUT/${TAG}_sq -o ${S#sq:} --output-format csv -- $BC --configs ${S#sq:} ;;
    sq2:*)  run sq2_${S#sq2:} 150 rocprofv3 --pmc $SQ2 -d $OUT/${TAG}_sq2 -o ${S#sq2:} --output-format csv -- $BC --configs ${S#sq2:} ;;
    kt:*)   run kt_${S#kt:} 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_kt -o ${S#kt:} --output-format csv -- $BC --configs ${S#kt:} ;;
    *:*:*)  IFS=: read -r name lim cmd <<< "$S"; run "$name" "$lim" bash -c "$cmd" ;;
    *)      echo "unknown step $S"; exit 2 ;;
  esac
done
echo "=== $TAG done" | tee -a $OUT/${TAG}_steps.log
