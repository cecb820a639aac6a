cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=build/libofdmsync_s64.so,build/libofdmsync_s32.so
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 65536 --T 1024 --L 512 --na 1 --no-check > gpurun_out/r02p_ab_head.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 65536 --T 1024 --L 512 --na 1 --detect-only --no-check > gpurun_out/r02p_ab_det.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 65536 --T 4096 --L 512 --na 1 --no-check > gpurun_out/r02p_ab_t4096.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --libs $L --B 16384 --T 5315 --L 512 --na 2 --no-check > gpurun_out/r02p_ab_ref.log 2>&1 || exit $?
OFS_LIB=build/libofdmsync_s32.so timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_headline_parity.py tests/test_gpu_parity.py -m gpu -k "aa" > gpurun_out/r02p_tests.log 2>&1
echo "tests rc=$?"
