cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_exact.py -m gpu -k "backend or receiver or rtl or minn" > gpurun_out/r02aw_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02aw_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_configs.py --configs backend,cfg2b --steps 10 --warmup 2 > gpurun_out/r02aw_cfg.log 2>&1 || exit $?
grep -o '"config": "[a-z0-9_]*"\|"ms": [0-9.]*' gpurun_out/r02aw_cfg.log | paste - -
echo done
