cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py -m gpu -k "zc_cfar or zc_detect or bit_identical or preamble" > gpurun_out/r02z8_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for v in s8 s16 s8r1 s4; do
OFS_LIB=build/libofdmsync_$v.so timeout -k 10 300 python tools/bench_configs.py --configs zc_detect,zc_detect_state --steps 10 --warmup 2 > gpurun_out/r02z8_cfgs_$v.log 2>&1 || exit $?
done
echo done
