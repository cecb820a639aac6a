#!/bin/bash
# Compile one csrc/*.hip for gfx950 and print per-kernel register / LDS / scratch usage.
#   tools/ru.sh corr [kernel-name-filter]
cd "$(dirname "$0")/.."
f=${1:-corr}
out=/tmp/ru_$f.txt
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude ${RU_FLAGS} -c ofdm-sync-math_amd/csrc/$f.hip \
  -o /tmp/ru_$f.o -Rpass-analysis=kernel-resource-usage > $out 2>&1
rc=$?
grep -E "error" $out | head -20
grep -E "Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy|LDS Size|VGPRs Spill" $out | sed 's/.*remark: //; s/ \[-Rpass.*//' \
  | paste - - - - - - - | grep -E "${2:-.}" | sed 's/Function Name: //'
exit $rc
