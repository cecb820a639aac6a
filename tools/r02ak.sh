cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py tests/test_gpu_parity.py tests/test_gpu_zc_rocfft.py -m gpu -k "zc_freq or zcfreq or freq or rocfft" > gpurun_out/r02ak_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02ak_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in build/libofdmsync_zfold.so ofdm-sync-math_amd/ofdm_sync_amd/libofdmsync.so build/libofdmsync_g8.so build/libofdmsync_g16.so; do
  OFS_LIB=$v timeout -k 10 200 python tools/bench_configs.py --configs zc_freq_fp64 --steps 10 --warmup 2 > gpurun_out/r02ak_x.log 2>&1 || { tail -3 gpurun_out/r02ak_x.log; exit 1; }
  echo "$(basename $v) $(grep -o '"ms": [0-9.]*' gpurun_out/r02ak_x.log | tr '\n' ' ')"
done
done
echo done
