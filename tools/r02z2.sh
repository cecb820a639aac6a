cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py -m gpu -k "zc" > gpurun_out/r02z2_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for v in r1 r2; do
OFS_LIB=build/libofdmsync_$v.so timeout -k 10 300 python tools/bench_configs.py --configs zc_detect,zc_detect_state --steps 10 --warmup 2 > gpurun_out/r02z2_cfgs_$v.log 2>&1 || exit $?
done
echo done
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py -m gpu -k "zc_freq" > gpurun_out/r02z2_tests_zf.log 2>&1 || { echo "zf tests rc=$?"; exit 1; }
for v in zf0 zf1; do
OFS_LIB=build/libofdmsync_$v.so timeout -k 10 300 python tools/bench_configs.py --configs zc_freq_fp64 --steps 5 --warmup 1 > gpurun_out/r02z2_cfgs_$v.log 2>&1 || exit $?
done
echo done2
