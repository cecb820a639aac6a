#!/bin/bash
# Static VALU / SALU / memory instruction counts of one kernel (gfx950 ISA), per source line.
#   tools/isa_count.sh aa_fast _ZN12_GLOBAL__N_114aa_fast_kernelILi4ELi2EEEv10AaFastArgs [EXTRA_FLAGS]
f=$1; sym=$2; shift 2
d=$(mktemp -d)
( cd $d && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I/root/repo/include -gline-tables-only \
    --save-temps "$@" -c /root/repo/ofdm-sync-math_amd/csrc/$f.hip -o $d/x.o 2>/dev/null )
awk "/^$sym:/,/s_endpgm/" $d/$f-hip-amdgcn-amd-amdhsa-gfx950.s > $d/k.s
python3 - $d/k.s $d/$f-hip-amdgcn-amd-amdhsa-gfx950.s <<'PY'
import re, sys, collections, os
files={}
for line in open(sys.argv[2]):
    m=re.match(r'\s+\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?',line)
    if m: files[int(m.group(1))]=os.path.basename(m.group(3) or m.group(2))
cur=None; cnt=collections.Counter(); n=collections.Counter()
for line in open(sys.argv[1]):
    m=re.match(r'\s+\.loc\s+(\d+)\s+(\d+)',line)
    if m: cur=(files.get(int(m.group(1)),m.group(1)),int(m.group(2))); continue
    s=line.strip()
    for p in ('v_','s_','ds_','global_','buffer_'):
        if s.startswith(p): n[p]+=1
    if s.startswith('v_'): cnt[cur]+=1
print(dict(n))
for k,v in cnt.most_common(int(os.environ.get('TOPN','12'))): print(v, k)
PY
rm -rf $d
