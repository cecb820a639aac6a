cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r02bi_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r02bi_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r02bi_smoke.log 2>&1; echo "smoke rc=$?"
echo done
