#!/bin/bash
# Sweep fast-path variants on the GPU box: library build (occupancy bound) x samples-per-lane.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for LIB in ${LIB_LIST:-build/libofdmsync_w0.so build/libofdmsync_w4.so build/libofdmsync_w5.so}; do
  for E in ${E_LIST:-4 2 8}; do
    echo "=== lib=$LIB E=$E" >> gpurun_out/tune.log
    OFS_LIB=$PWD/$LIB OFS_FAST_E=$E timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/tune_one.log 2>&1
    rc=$?
    tail -1 gpurun_out/tune_one.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('value', d['value'], 'frac', d['roofline']['frac'], 'ms', d['ms_per_step'])" >> gpurun_out/tune.log 2>&1 || tail -3 gpurun_out/tune_one.log >> gpurun_out/tune.log
    if [ $rc -ge 124 ]; then echo "fatal rc=$rc" >> gpurun_out/tune.log; exit $rc; fi
  done
done
exit 0
