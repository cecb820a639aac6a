cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base nowalk nohelp nochain; do
  OFS_LIB=build/libofdmsync_$v.so timeout -k 10 200 python tools/bench_configs.py --configs zc_detect,zc_detect_state --steps 10 --warmup 2 > gpurun_out/r02ar_x.log 2>&1 || { tail -3 gpurun_out/r02ar_x.log; exit 1; }
  echo "$v $(grep -o '"ms": [0-9.]*' gpurun_out/r02ar_x.log | tr '\n' ' ')"
done
echo done
