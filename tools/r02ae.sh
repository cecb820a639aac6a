cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_zc_rocfft.py -m gpu > gpurun_out/r02ae_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02ae_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_configs.py --configs cfg5_rocfft_dense --steps 5 --warmup 1 > gpurun_out/r02ae_dense.log 2>&1 || exit $?
grep -o '"ms": [0-9.]*' gpurun_out/r02ae_dense.log
for p in metric smooth full; do
  OFS_CFG2B_PARTS=$p timeout -k 10 200 python tools/bench_configs.py --configs cfg2b --steps 20 --warmup 3 > gpurun_out/r02ae_cfg2b_$p.log 2>&1 || exit $?
  echo "cfg2b $p $(grep -o '"ms": [0-9.]*' gpurun_out/r02ae_cfg2b_$p.log)"
done
for w in 1 2; do
  OFS_RTL_WPB=$w timeout -k 10 200 python tools/bench_configs.py --configs cfg2b --steps 20 --warmup 3 > gpurun_out/r02ae_cfg2b_w$w.log 2>&1 || exit $?
  echo "cfg2b wpb=$w $(grep -o '"ms": [0-9.]*' gpurun_out/r02ae_cfg2b_w$w.log)"
done
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/r02ae_sq -o cfg2b --output-format csv -- python3 tools/bench_configs.py --configs cfg2b --steps 3 --warmup 1 > gpurun_out/r02ae_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_CVT -d gpurun_out/r02ae_sq2 -o cfg2b --output-format csv -- python3 tools/bench_configs.py --configs cfg2b --steps 3 --warmup 1 > gpurun_out/r02ae_sq2.log 2>&1
echo "sq2 rc=$?"
echo done
