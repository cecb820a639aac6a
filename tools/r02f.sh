cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r02f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r02f_bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02f_prof -o cfgs --output-format csv -- python3 tools/bench_configs.py --configs aa_refshape_c64,aa_refshape_c128,cfg3_T4096,cfg4,cfg5 --steps 10 --warmup 2 > gpurun_out/r02f_cfgs.log 2>&1
echo "cfgs rc=$?"
