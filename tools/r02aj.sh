cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py tests/test_gpu_parity.py -m gpu -k "zc_freq or zcfreq or freq" > gpurun_out/r02aj_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02aj_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in g64 g32 g16; do
  OFS_LIB=build/libofdmsync_$v.so timeout -k 10 200 python tools/bench_configs.py --configs zc_freq_fp64 --steps 10 --warmup 2 > gpurun_out/r02aj_$v.log 2>&1 || { tail -3 gpurun_out/r02aj_$v.log; exit 1; }
  echo "$v $(grep -o '"ms": [0-9.]*' gpurun_out/r02aj_$v.log | tr '\n' ' ')"
done
done
echo done
