cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r02ac_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02ac_tests.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r02ac_smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 400 python bench.py > gpurun_out/r02ac_bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/r02ac_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02ac_prof -o bench --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/r02ac_prof.log 2>&1 || exit $?
echo done
