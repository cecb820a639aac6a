#!/bin/bash
# Build tuning variants of libofdmsync.so (occupancy bound of the fast kernel) into build/.
cd "$(dirname "$0")/.."
mkdir -p build
for W in ${WAVES_LIST:-0 4 5}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -DOFS_FAST_WAVES=$W \
     -o build/libofdmsync_w$W.so ofdm-sync-math_amd/csrc/*.hip &
done
wait
ls -la build/
