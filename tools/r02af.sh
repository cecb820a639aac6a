cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_wire.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "rtl or minn or wire or cfg2" > gpurun_out/r02af_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02af_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/rtl_ab.py --libs build/libofdmsync_spec.so,build/libofdmsync_walk.so > gpurun_out/r02af_ab0.log 2>&1 || { cat gpurun_out/r02af_ab0.log | tail -5; exit 1; }
cat gpurun_out/r02af_ab0.log
timeout -k 10 200 python tools/rtl_ab.py --libs build/libofdmsync_spec.so,build/libofdmsync_walk.so --mode 1 > gpurun_out/r02af_ab1.log 2>&1 || { tail -5 gpurun_out/r02af_ab1.log; exit 1; }
cat gpurun_out/r02af_ab1.log
timeout -k 10 200 python tools/rtl_ab.py --libs build/libofdmsync_spec.so,build/libofdmsync_walk.so --Q 128 --T 3000 --B 2000 > gpurun_out/r02af_ab2.log 2>&1 || { tail -5 gpurun_out/r02af_ab2.log; exit 1; }
cat gpurun_out/r02af_ab2.log
timeout -k 10 200 python tools/bench_configs.py --configs cfg2b,cfg2b_cp12 --steps 20 --warmup 3 > gpurun_out/r02af_cfgs.log 2>&1 || exit $?
grep -o '"config": "[a-z0-9_]*"\|"ms": [0-9.]*' gpurun_out/r02af_cfgs.log | paste - -
echo done
