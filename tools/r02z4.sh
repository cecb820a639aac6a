cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in r2 nochain; do
OFS_LIB=build/libofdmsync_$v.so timeout -k 10 300 python tools/bench_configs.py --configs zc_detect --steps 10 --warmup 2 > gpurun_out/r02z4_cfgs_$v.log 2>&1 || exit $?
done
OFS_LIB=build/libofdmsync_r2.so timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/r02z4_pmc -o zc --output-format csv -- python3 tools/bench_configs.py --configs zc_detect --steps 2 --warmup 1 > gpurun_out/r02z4_pmc.log 2>&1
echo done
