cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_zc_rocfft.py -m gpu > gpurun_out/r02j_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r02j_prof -o cfgs --output-format csv -- python3 tools/bench_configs.py --configs cfg5,cfg5_rocfft,cfg5_rocfft_dense --steps 5 --warmup 1 > gpurun_out/r02j_cfgs.log 2>&1
echo "cfgs rc=$?"
