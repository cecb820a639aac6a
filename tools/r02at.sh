cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py -m gpu -k "zc_cfar" > gpurun_out/r02at_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02at_tests.log; [ $rc -ne 0 ] && exit $rc
OFS_ZC_NODMA=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py -m gpu -k "zc_cfar" > gpurun_out/r02at_tests2.log 2>&1
rc=$?; echo "tests nodma rc=$rc"; tail -1 gpurun_out/r02at_tests2.log
echo done
