cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in r2 nowalk nohelp none; do
OFS_LIB=build/libofdmsync_$v.so timeout -k 10 300 python tools/bench_configs.py --configs zc_detect,zc_detect_state --steps 10 --warmup 2 > gpurun_out/r02z3_cfgs_$v.log 2>&1 || exit $?
done
for v in zf0 zf1; do
OFS_LIB=build/libofdmsync_$v.so timeout -k 10 300 python tools/bench_configs.py --configs zc_freq_fp64 --steps 5 --warmup 1 > gpurun_out/r02z3_cfgs_$v.log 2>&1 || exit $?
done
echo done
