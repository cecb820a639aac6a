cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=build/libofdmsync_peelffpd2.so,build/libofdmsync_l0.so,build/libofdmsync_l1.so,build/libofdmsync_l2.so,build/libofdmsync_l2w4.so,build/libofdmsync_l2pd4.so
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 65536 --T 4096 --L 512 --na 1 > gpurun_out/r02e_ab_t4096.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 16384 --T 5315 --L 512 --na 2 > gpurun_out/r02e_ab_ref.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 65536 --T 2048 --L 256 --na 1 > gpurun_out/r02e_ab_t2048.log 2>&1 || exit $?
