cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
for v in base w4 w4pd1 pd2; do
  OFS_LIB=build/libofdmsync_$v.so timeout -k 10 200 python tools/bench_configs.py --configs cfg2a,cfg2a_cp12 --steps 30 --warmup 3 > gpurun_out/r02ah_$v.log 2>&1 || { tail -3 gpurun_out/r02ah_$v.log; exit 1; }
  echo "$v $(grep -o '"ms": [0-9.]*' gpurun_out/r02ah_$v.log | tr '\n' ' ')"
done
done
echo done
L=ofdm-sync-math_amd/ofdm_sync_amd/libofdmsync.so
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_wire.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "rtl or minn or wire or cfg2" > gpurun_out/r02ah_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02ah_tests.log; [ $rc -ne 0 ] && exit $rc
for extra in "" "--mode 1" "--T 1001"; do
  timeout -k 10 200 python tools/rtl_ab.py --libs build/libofdmsync_prev.so,$L $extra > gpurun_out/r02ah_ab.log 2>&1 || { tail -5 gpurun_out/r02ah_ab.log; exit 1; }
  echo "== $extra"; grep -v amdgpu.ids gpurun_out/r02ah_ab.log
done
echo done2
