cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=build/libofdmsync_al0.so,build/libofdmsync_al2.so
timeout -k 10 200 python tools/lib_ab.py --op scminn --libs $L --B 32768 --T 4096 --L 1024 --na 1 > gpurun_out/r02t_ab_cfg4.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --op scminn --libs $L --B 16384 --T 4096 --L 1024 --na 2 > gpurun_out/r02t_ab_cfg4_2br.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --op scminn --libs $L --B 32768 --T 4001 --L 512 --na 1 > gpurun_out/r02t_ab_odd.log 2>&1
echo done
