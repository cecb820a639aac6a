"""Static instruction counts of the loops of one kernel in a gfx950 .s (diagnostic tooling).
    python tools/loop_isa.py file.s symbol"""
import re, sys
lines = open(sys.argv[1]).read().split('\n')
sym = sys.argv[2]
start = next(i for i, l in enumerate(lines) if l.startswith(sym + ':'))
end = next(i for i in range(start, len(lines)) if 's_endpgm' in lines[i])
lines = lines[start:end + 1]
labels = {}
for i, l in enumerate(lines):
    m = re.match(r'^(\.LBB\d+_\d+):', l)
    if m:
        labels[m.group(1)] = i
cnt = lambda body, p: sum(1 for x in body if x.strip().startswith(p))
print('kernel', 'valu', cnt(lines, 'v_'), 'salu', cnt(lines, 's_'), 'vgpr', [l for l in lines if 'NumVgprs' in l][:1])
for i, l in enumerate(lines):
    m = re.search(r's_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
    if m and labels.get(m.group(2), 1e9) < i:
        body = lines[labels[m.group(2)]:i + 1]
        print(m.group(2), len(body), 'valu', cnt(body, 'v_'), 'salu', cnt(body, 's_'), 'global', cnt(body, 'global_'),
              'f64', sum(1 for x in body if '_f64' in x), 'dpp', sum(1 for x in body if '_dpp' in x))
