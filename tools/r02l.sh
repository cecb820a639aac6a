cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py -m gpu > gpurun_out/r02l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
OFS_ZC_METHOD=fft timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02l_prof -o mf --output-format csv -- python3 tools/bench_configs.py --configs zc_mf,zc_mf_direct --steps 5 --warmup 1 > gpurun_out/r02l_cfgs.log 2>&1
echo "cfgs rc=$?"
