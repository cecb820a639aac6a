cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=build/libofdmsync_old.so,build/libofdmsync_oldpd2.so,build/libofdmsync_peelff.so,build/libofdmsync_peelnoff.so,build/libofdmsync_peelffpd2.so,build/libofdmsync_peelnoffpd2.so
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 65536 --T 4096 --L 512 --na 1 > gpurun_out/r02d_ab_t4096.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 16384 --T 5315 --L 512 --na 2 > gpurun_out/r02d_ab_ref.log 2>&1 || exit $?
