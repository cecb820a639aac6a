cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=build/libofdmsync_pk0.so,build/libofdmsync_pk1.so
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_winfast.py tests/test_gpu_fullsize.py -m gpu > gpurun_out/r02u_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 200 python tools/lib_ab.py --op scminn --no-check --libs $L --B 32768 --T 4096 --L 1024 --na 1 > gpurun_out/r02u_ab_cfg4.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --op scminn --no-check --libs $L --B 16384 --T 4096 --L 1024 --na 2 > gpurun_out/r02u_ab_cfg4_2br.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --op scminn --no-check --libs $L --B 32768 --T 4001 --L 512 --na 1 > gpurun_out/r02u_ab_odd.log 2>&1
echo done
