cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_corr.py -m gpu -k "park" > gpurun_out/r02ab_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python tools/bench_configs.py --configs park_fp32,park_fp64 --steps 5 --warmup 1 > gpurun_out/r02ab_cfgs.log 2>&1 || exit $?
OFS_PARK_DIRECT=1 timeout -k 10 300 python tools/bench_configs.py --configs park_fp32,park_fp64 --steps 5 --warmup 1 > gpurun_out/r02ab_cfgs_direct.log 2>&1
echo done
