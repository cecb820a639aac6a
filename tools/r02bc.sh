cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py tests/test_gpu_parity.py -m gpu -k "fft or zc" > gpurun_out/r02bc_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r02bc_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_configs.py --configs zc_mf,zc_mf --steps 10 --warmup 2 > gpurun_out/r02bc_x.log 2>&1 || exit $?
grep -o '"ms": [0-9.]*' gpurun_out/r02bc_x.log | tr '\n' ' '
echo done
