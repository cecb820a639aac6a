# Diagnostic: interleaved A/B of two library builds (OFS_LIB) on the small exact configs, then the
# corr / parity / fullsize / wire / exact GPU tests.  Usage on the GPU box: bash tools/rtl_ab.sh
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
  for L in rtlold rtlnew; do
    OFS_LIB=build/libofdmsync_$L.so timeout -k 10 120 python -u tools/bench_configs.py --configs cfg2b,cfg2b_cp12,cfg2a,cfg3_2ant > gpurun_out/rtl_ab_${L}_$r.jsonl 2>&1
  done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_corr.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_wire.py tests/test_gpu_exact.py > gpurun_out/rtl_tests.log 2>&1
