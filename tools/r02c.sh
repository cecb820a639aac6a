cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=build/libofdmsync_base.so,build/libofdmsync_pd2.so,build/libofdmsync_pd8.so,build/libofdmsync_w4.so,build/libofdmsync_w4pd8.so,build/libofdmsync_w2pd8.so
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 65536 --T 4096 --L 512 --na 1 > gpurun_out/r02c_ab_t4096.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 16384 --T 5315 --L 512 --na 2 > gpurun_out/r02c_ab_ref.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 16384 --T 5316 --L 512 --na 2 > gpurun_out/r02c_ab_ref_even.log 2>&1 || exit $?
