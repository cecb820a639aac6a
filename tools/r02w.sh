cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=build/libofdmsync_aaold.so,build/libofdmsync_aanew.so
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_headline_parity.py tests/test_gpu_parity.py tests/test_gpu_detect_only.py tests/test_gpu_fullsize.py -m gpu > gpurun_out/r02w_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for E in 2 4; do
OFS_FAST_E=$E timeout -k 10 200 python tools/lib_ab.py --no-check --libs $L --B 65536 --T 1024 --L 512 --na 1 > gpurun_out/r02w_ab_head_E$E.log 2>&1 || exit $?
OFS_FAST_E=$E timeout -k 10 200 python tools/lib_ab.py --no-check --detect-only --libs $L --B 65536 --T 1024 --L 512 --na 1 > gpurun_out/r02w_ab_det_E$E.log 2>&1 || exit $?
done
timeout -k 10 200 python tools/lib_ab.py --no-check --libs $L --B 65536 --T 4096 --L 512 --na 1 > gpurun_out/r02w_ab_t4096.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --no-check --libs $L --B 16384 --T 5315 --L 512 --na 2 > gpurun_out/r02w_ab_ref.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --no-check --detect-only --libs $L --B 65536 --T 4096 --L 512 --na 1 > gpurun_out/r02w_ab_t4096_det.log 2>&1
echo done
