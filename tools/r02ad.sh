cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_zc_rocfft.py -m gpu > gpurun_out/r02ad_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02ad_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_configs.py --configs cfg5_rocfft_dense,cfg5 --steps 5 --warmup 1 > gpurun_out/r02ad_dense.log 2>&1 || exit $?
for c in 512 1024 2048 4096 8192; do
  OFS_ZC_FFT_CHUNK=$c timeout -k 10 200 python tools/bench_configs.py --configs cfg5_rocfft_chunked --steps 5 --warmup 1 > gpurun_out/r02ad_chunk$c.log 2>&1 || exit $?
  grep -o '"ms": [0-9.]*' gpurun_out/r02ad_chunk$c.log | tr '\n' ' '; echo " chunk=$c"
done
OFS_ZC_FFT_CHUNK=2048 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02ad_prof -o chunk --output-format csv -- python3 tools/bench_configs.py --configs cfg5_rocfft_chunked --steps 3 --warmup 1 > gpurun_out/r02ad_prof.log 2>&1 || exit $?
echo done
