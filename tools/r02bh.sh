cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for extra in "" "--shift 0" "--Q 128 --T 3000 --B 2000"; do
  timeout -k 10 200 python tools/rtl_ab.py --libs build/libofdmsync_rbase.so,build/libofdmsync_rwalk.so $extra > gpurun_out/r02bh_ab.log 2>&1 || { tail -5 gpurun_out/r02bh_ab.log; exit 1; }
  echo "== $extra"; grep -v amdgpu.ids gpurun_out/r02bh_ab.log
done
echo done
