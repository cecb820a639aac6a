cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/bin/sol_stream 65536 20 > gpurun_out/r02h_sol.log 2>&1 || exit $?
C="python3 tools/bench_configs.py --configs cfg4 --cfg4-global 32768 --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02h_pmcF -o cfg4 --output-format csv -- $C > gpurun_out/r02h_pmcF.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02h_pmcW -o cfg4 --output-format csv -- $C > gpurun_out/r02h_pmcW.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/r02h_pmcSQ -o cfg4 --output-format csv -- $C > gpurun_out/r02h_pmcSQ.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02h_kt -o cfg4 --output-format csv -- $C > gpurun_out/r02h_kt.log 2>&1
