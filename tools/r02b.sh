cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_detect_only.py tests/test_gpu_fp64_wave.py tests/test_gpu_headline_parity.py -m gpu > gpurun_out/r02b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02b_prof -o cfgs --output-format csv -- python3 tools/bench_configs.py --configs cfg3_T4096,aa_refshape_c64,aa_refshape_c128 --steps 10 --warmup 2 > gpurun_out/r02b_cfgs.log 2>&1
echo "cfgs rc=$?"
