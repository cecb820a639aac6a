# Diagnostic: interleaved A/B of two library builds (OFS_LIB) over tools/bench_configs.py configs,
# then a GPU test subset.  Usage on the GPU box:
#   bash tools/lib_cfg_ab.sh build/libofdmsync_a.so build/libofdmsync_b.so cfg2a,cfg4 "tests/test_gpu_parity.py"
set -e
mkdir -p gpurun_out
A=$1; B=$2; CFGS=$3; TESTS=$4
for r in 1 2 3; do
  for L in $A $B; do
    n=$(basename $L .so)
    OFS_LIB=$L timeout -k 10 240 python -u tools/bench_configs.py --configs $CFGS > gpurun_out/ab_${n}_$r.jsonl 2>&1
  done
done
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > gpurun_out/ab_tests.log 2>&1
fi
