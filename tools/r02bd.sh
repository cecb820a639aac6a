cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r02bd_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r02bd_smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 400 python bench.py > gpurun_out/r02bd_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02bd_prof -o bench --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/r02bd_prof.log 2>&1 || exit $?
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/r02bd_cfgs.log 2>&1; echo "cfgs rc=$?"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r02bd_cfgprof -o cfgs --output-format csv -- python3 tools/bench_configs.py --steps 3 --warmup 1 > gpurun_out/r02bd_cfgprof.log 2>&1
echo "cfgprof rc=$?"
