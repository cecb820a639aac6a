cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_wire.py tests/test_gpu_exact.py tests/test_gpu_parity.py -m gpu > gpurun_out/r02i_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02i_prof -o cfgs --output-format csv -- python3 tools/bench_configs.py --configs cfg2a,cfg2a_cp12,cfg2b,cfg2b_cp12 --steps 20 --warmup 3 > gpurun_out/r02i_cfgs.log 2>&1
echo "cfgs rc=$?"
