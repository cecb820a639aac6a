cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=build/libofdmsync_old.so,build/libofdmsync_new.so
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_winfast.py tests/test_gpu_parity.py -m gpu > gpurun_out/r02v_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for op in sc comb minn; do
timeout -k 10 200 python tools/lib_ab.py --op $op --no-check --libs $L --B 32768 --T 4096 --L 1024 --na 1 > gpurun_out/r02v_ab_$op.log 2>&1 || exit $?
done
timeout -k 10 200 python tools/lib_ab.py --op sc --no-check --libs $L --B 16384 --T 4096 --L 1024 --na 2 > gpurun_out/r02v_ab_sc2.log 2>&1 || exit $?
timeout -k 10 200 python tools/lib_ab.py --op minn --no-check --libs $L --B 32768 --T 4001 --L 512 --na 1 > gpurun_out/r02v_ab_minn_odd.log 2>&1
echo done
