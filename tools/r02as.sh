cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py tests/test_gpu_postproc.py tests/test_gpu_parity.py -m gpu -k "zc" > gpurun_out/r02as_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02as_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in dma nodma; do
  if [ $v = nodma ]; then export OFS_ZC_NODMA=1; else unset OFS_ZC_NODMA; fi
  timeout -k 10 200 python tools/bench_configs.py --configs zc_detect,zc_detect_state --steps 10 --warmup 2 > gpurun_out/r02as_x.log 2>&1 || { tail -3 gpurun_out/r02as_x.log; exit 1; }
  echo "$v $(grep -o '"ms": [0-9.]*' gpurun_out/r02as_x.log | tr '\n' ' ')"
done
done
echo done
