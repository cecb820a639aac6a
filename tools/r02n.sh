cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_fullsize.py -m gpu > gpurun_out/r02n_tests.log 2>&1
echo "tests rc=$?"
