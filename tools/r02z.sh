cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py -m gpu -k "zc" > gpurun_out/r02z_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python tools/bench_configs.py --configs zc_detect,zc_detect_state,zc_detect_seq --steps 10 --warmup 2 > gpurun_out/r02z_cfgs.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02z_prof -o cfgs --output-format csv -- python3 tools/bench_configs.py --configs zc_detect,zc_detect_state --steps 5 --warmup 1 > gpurun_out/r02z_prof.log 2>&1
echo done
