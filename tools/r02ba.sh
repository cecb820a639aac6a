cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OFS_LIB=build/libofdmsync_wf64.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_winfast.py -m gpu > gpurun_out/r02ba_t.log 2>&1
rc=$?; echo "tests wf64 rc=$rc"; tail -1 gpurun_out/r02ba_t.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in wf256 wf64 wf128; do
  OFS_LIB=build/libofdmsync_$v.so timeout -k 10 200 python tools/bench_configs.py --configs cfg4,cfg4_2br --cfg4-global 32768 --steps 10 --warmup 2 > gpurun_out/r02ba_x.log 2>&1 || { tail -3 gpurun_out/r02ba_x.log; exit 1; }
  echo "$v $(grep -o '"ms": [0-9.]*' gpurun_out/r02ba_x.log | tr '\n' ' ')"
done
done
echo done
