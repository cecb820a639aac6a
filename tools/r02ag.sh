cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=ofdm-sync-math_amd/ofdm_sync_amd/libofdmsync.so
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_wire.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "rtl or minn or wire or cfg2" > gpurun_out/r02ag_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02ag_tests.log; [ $rc -ne 0 ] && exit $rc
for extra in "" "--mode 1" "--Q 128 --T 3000 --B 2000" "--Q 128 --T 3000 --B 2000 --mode 1" "--shift 0"; do
  timeout -k 10 200 python tools/rtl_ab.py --libs build/libofdmsync_prev.so,$L $extra > gpurun_out/r02ag_ab.log 2>&1 || { tail -5 gpurun_out/r02ag_ab.log; exit 1; }
  echo "== $extra"; grep -v amdgpu.ids gpurun_out/r02ag_ab.log
done
timeout -k 10 200 python tools/bench_configs.py --configs cfg2b,cfg2b_cp12 --steps 20 --warmup 3 > gpurun_out/r02ag_cfgs.log 2>&1 || exit $?
grep -o '"config": "[a-z0-9_]*"\|"ms": [0-9.]*' gpurun_out/r02ag_cfgs.log | paste - -
echo done
