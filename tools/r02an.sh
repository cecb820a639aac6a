cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
for v in scmbase scmw2; do
  OFS_LIB=build/libofdmsync_$v.so timeout -k 10 200 python tools/bench_configs.py --configs cfg4_2br,cfg4 --cfg4-global 32768 --steps 10 --warmup 2 > gpurun_out/r02an_$v.log 2>&1 || { tail -3 gpurun_out/r02an_$v.log; exit 1; }
  echo "$v $(grep -o '"ms": [0-9.]*' gpurun_out/r02an_$v.log | tr '\n' ' ')"
done
done
echo done
