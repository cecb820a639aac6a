cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/lib_ab.py --libs build/libofdmsync_hbase.so,build/libofdmsync_hilp.so,build/libofdmsync_hmc.so --B 65536 --T 1024 --L 512 --na 1 --rounds 6 > gpurun_out/r02bg_ab.log 2>&1 || { tail -5 gpurun_out/r02bg_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r02bg_ab.log
timeout -k 10 400 python tools/lib_ab.py --libs build/libofdmsync_hbase.so,build/libofdmsync_hilp.so,build/libofdmsync_hmc.so --B 65536 --T 4096 --L 512 --na 1 --rounds 4 > gpurun_out/r02bg_ab2.log 2>&1 || { tail -5 gpurun_out/r02bg_ab2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r02bg_ab2.log
echo done
