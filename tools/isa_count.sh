#!/bin/bash
# Static VALU / SALU / memory instruction counts of one kernel (gfx950 ISA), per source line.
#   tools/isa_count.sh aa_fast _ZN12_GLOBAL__N_114aa_fast_kernelILi4ELi2EEEv10AaFastArgs [EXTRA_FLAGS]
f=$1; sym=$2; shift 2
d=$(mktemp -d)
( cd $d && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I/root/repo/include -gline-tables-only \
    --save-temps "$@" -c /root/repo/ofdm-sync-math_amd/csrc/$f.hip -o $d/x.o 2>/dev/null )
awk "/^$sym:/,/s_endpgm/" $d/$f-hip-amdgcn-amd-amdhsa-gfx950.s > $d/k.s
python3 - $d/k.s <<'PY'
import re, sys, collections
cur=None; cnt=collections.Counter(); n=collections.Counter()
for line in open(sys.argv[1]):
    m=re.match(r'\s+\.loc\s+(\d+)\s+(\d+)',line)
    if m: cur=(int(m.group(1)),int(m.group(2))); continue
    s=line.strip()
    for p in ('v_','s_','ds_','global_','buffer_'):
        if s.startswith(p): n[p]+=1
    if s.startswith('v_'): cnt[cur]+=1
print(dict(n)); print(cnt.most_common(12))
PY
rm -rf $d
