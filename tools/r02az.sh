cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in be512 be1024; do
  OFS_LIB=build/libofdmsync_$v.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "backend or receiver" > gpurun_out/r02az_t_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -1 gpurun_out/r02az_t_$v.log; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
for v in be256 be512 be1024; do
  OFS_LIB=build/libofdmsync_$v.so timeout -k 10 200 python tools/bench_configs.py --configs backend --steps 10 --warmup 2 > gpurun_out/r02az_x.log 2>&1 || { tail -3 gpurun_out/r02az_x.log; exit 1; }
  echo "$v $(grep -o '"ms": [0-9.]*' gpurun_out/r02az_x.log | tr '\n' ' ')"
done
done
echo done
