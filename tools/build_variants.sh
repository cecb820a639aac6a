#!/bin/bash
# Build tuning variants of libofdmsync.so into build/: VARIANTS is a list of name=flags,
# e.g. "w0= nt=-DOFS_STORE_NT=1 aux2=-DOFS_DMA_AUX=2".
cd "$(dirname "$0")/.."
mkdir -p build
VARIANTS=${VARIANTS:-"w0= w4=-DOFS_FAST_WAVES=4 w5=-DOFS_FAST_WAVES=5"}
for V in $VARIANTS; do
  NAME=${V%%=*}; FLAGS=${V#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude $FLAGS \
     -o build/libofdmsync_$NAME.so ofdm-sync-math_amd/csrc/*.hip -L/opt/rocm/lib -lrocfft -Wl,-rpath,/opt/rocm/lib &
done
wait
ls -la build/
