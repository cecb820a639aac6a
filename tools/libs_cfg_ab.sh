# Diagnostic: interleaved A/B of N library builds (OFS_LIB) over tools/bench_configs.py configs, lib
# order rotated per round.  Usage on the GPU box:
#   bash tools/libs_cfg_ab.sh TAG build/libofdmsync_a.so,build/libofdmsync_b.so,... cfg2a,cfg4 [ROUNDS]
# Output: gpurun_out/TAG_<lib>_<round>.jsonl
set -e
mkdir -p gpurun_out
TAG=$1; IFS=, read -ra LIBS <<< "$2"; CFGS=$3; ROUNDS=${4:-3}
n=${#LIBS[@]}
for ((r = 0; r < ROUNDS; r++)); do
  for ((i = 0; i < n; i++)); do
    L=${LIBS[$(( (i + r) % n ))]}
    OFS_LIB=$L timeout -k 10 240 python -u tools/bench_configs.py --configs $CFGS > gpurun_out/${TAG}_$(basename $L .so)_$r.jsonl 2>&1
  done
done
