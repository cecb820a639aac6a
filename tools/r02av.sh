cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/lib_ab.py --libs build/libofdmsync_st1.so,build/libofdmsync_st0.so --B 65536 --T 1024 --L 512 --na 1 --rounds 8 > gpurun_out/r02av_ab.log 2>&1 || { tail -5 gpurun_out/r02av_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r02av_ab.log
timeout -k 10 400 python tools/lib_ab.py --libs build/libofdmsync_st1.so,build/libofdmsync_st0.so --B 65536 --T 1024 --L 512 --na 2 --rounds 6 > gpurun_out/r02av_ab2.log 2>&1 || { tail -5 gpurun_out/r02av_ab2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r02av_ab2.log
timeout -k 10 400 python tools/lib_ab.py --libs build/libofdmsync_st1.so,build/libofdmsync_st0.so --B 65536 --T 1024 --L 128 --na 1 --rounds 6 > gpurun_out/r02av_ab3.log 2>&1 || { tail -5 gpurun_out/r02av_ab3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r02av_ab3.log
echo done
