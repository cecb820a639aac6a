cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py tests/test_gpu_zc_rocfft.py tests/test_gpu_fullsize.py -m gpu -k "zc_freq or cfg5 or rocfft or zc" > gpurun_out/r02au_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02au_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
for v in winbi winasm; do
  OFS_LIB=build/libofdmsync_$v.so timeout -k 10 200 python tools/bench_configs.py --configs cfg5 --steps 10 --warmup 2 > gpurun_out/r02au_x.log 2>&1 || { tail -3 gpurun_out/r02au_x.log; exit 1; }
  echo "$v $(grep -o '"ms": [0-9.]*' gpurun_out/r02au_x.log | tr '\n' ' ')"
done
done
echo done
