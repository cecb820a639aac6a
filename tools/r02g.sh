cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_synth.py tests/test_gpu_detect_only.py -m gpu > gpurun_out/r02g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python bench.py --steps 50 > gpurun_out/r02g_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02g_prof -o bench --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/r02g_prof.log 2>&1
echo "prof rc=$?"
