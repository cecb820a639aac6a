# Diagnostic: interleaved A/B/... of several library builds (OFS_LIB) over tools/bench_configs.py configs.
#   bash tools/lib_cfg_abn.sh ROUNDS CONFIGS build/libofdmsync_a.so build/libofdmsync_b.so ...
set -e
mkdir -p gpurun_out
R=$1; CFGS=$2; shift 2
for r in $(seq 1 $R); do
  for L in "$@"; do
    n=$(basename $L .so)
    OFS_LIB=$L timeout -k 10 240 python -u tools/bench_configs.py --configs $CFGS > gpurun_out/abn_${n}_$r.jsonl 2>&1
    echo "$n $r $(grep -o '"ms": [0-9.]*' gpurun_out/abn_${n}_$r.jsonl | tr '\n' ' ')"
  done
done
