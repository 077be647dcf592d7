#!/usr/bin/env python3
"""Dev: instruction mix of every loop of one kernel in a hipcc device assembly (.s) file.
usage: tools/dev/loopmix.py file.s <kernel-name substring>"""
import collections
import sys

lines = open(sys.argv[1]).read().split('\n')
name = sys.argv[2]
s = [i for i, l in enumerate(lines) if name in l and l.split(';')[0].rstrip().endswith(':') and not l.startswith(('\t', ' ', '.'))]
if not s:
    sys.exit(f'kernel {name} not found')
s = s[0]
e = next(i for i in range(s, len(lines)) if lines[i].startswith('.Lfunc_end'))
k = lines[s:e]
print(lines[s][:120], len(k), 'lines')
for i, l in enumerate(k):
    if 'Loop Header' not in l:
        continue
    lab = l.split(':')[0]
    js = [x for x in range(i + 1, len(k)) if lab in k[x] and ('s_branch' in k[x] or 's_cbranch' in k[x])]
    if not js:
        continue
    j = js[-1]
    c = collections.Counter()
    for ln in k[i:j + 1]:
        ln = ln.strip()
        if not ln or ln.startswith((';', '.')):
            continue
        op = ln.split()[0]
        if op.startswith('v_mfma'):
            kk = 'mfma'
        elif op.startswith('v_'):
            kk = 'valu'
        elif op.startswith('s_waitcnt'):
            kk = 'waitcnt'
        elif op.startswith('s_'):
            kk = 'salu'
        elif op.startswith('ds_'):
            kk = 'ds'
        elif ('global_load' in op or 'buffer_load' in op) and ' lds' in ' ' + ln.replace(',', ' '):
            kk = 'dma'
        elif op.startswith(('global_', 'buffer_')):
            kk = 'vmem'
        else:
            kk = op
        c[kk] += 1
    print(f'  loop {lab} (depth: {l.split("Depth=")[-1]}) {j - i} lines: {dict(c)}')
