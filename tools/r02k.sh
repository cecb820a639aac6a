cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02k_prof -o cfgs --output-format csv -- python3 tools/bench_configs.py --configs park_fp32,park_fp64,zc_mf,zc_freq_fp64,zc_detect --steps 5 --warmup 1 > gpurun_out/r02k_cfgs.log 2>&1
echo "cfgs rc=$?"
C="python3 tools/bench_configs.py --configs cfg5_rocfft,cfg5_rocfft_dense --cfg5-global 262144 --steps 2 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02k_pmcF -o fft --output-format csv -- $C > gpurun_out/r02k_pmcF.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02k_pmcW -o fft --output-format csv -- $C > gpurun_out/r02k_pmcW.log 2>&1 || exit $?
