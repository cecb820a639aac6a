cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_postproc.py tests/test_gpu_synth.py -m gpu -k "backend or receiver" > gpurun_out/r02am_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02am_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_configs.py --configs backend --steps 10 --warmup 2 > gpurun_out/r02am_cfg.log 2>&1 || exit $?
grep -o '"ms": [0-9.]*\|"hbm_frac": [0-9.]*' gpurun_out/r02am_cfg.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02am_prof -o be --output-format csv -- python3 tools/bench_configs.py --configs backend --steps 3 --warmup 1 > gpurun_out/r02am_prof.log 2>&1
echo done
