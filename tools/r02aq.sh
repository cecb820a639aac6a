cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
for v in w4 w8 w8g8; do
  OFS_LIB=build/libofdmsync_$v.so timeout -k 10 200 python tools/bench_configs.py --configs zc_freq_fp64 --steps 10 --warmup 2 > gpurun_out/r02aq_x.log 2>&1 || { tail -3 gpurun_out/r02aq_x.log; exit 1; }
  echo "$v $(grep -o '"ms": [0-9.]*' gpurun_out/r02aq_x.log | tr '\n' ' ')"
done
done
echo done
