cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/r02o_sq_head -o head --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02o_sq_head.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/r02o_sq_det -o det --output-format csv -- python3 tools/bench_configs.py --configs cfg3_detect --steps 3 --warmup 1 > gpurun_out/r02o_sq_det.log 2>&1 || exit $?
timeout -k 10 120 tools/bin/sol_stream 65536 20 > gpurun_out/r02o_sol.log 2>&1 || exit $?
C="python3 tools/bench_configs.py --configs cfg4 --cfg4-global 32768 --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02o_pmcF -o cfg4 --output-format csv -- $C > gpurun_out/r02o_pmcF.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02o_pmcW -o cfg4 --output-format csv -- $C > gpurun_out/r02o_pmcW.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/r02o_sq_cfg4 -o cfg4 --output-format csv -- $C > gpurun_out/r02o_sq_cfg4.log 2>&1 || exit $?
echo done
