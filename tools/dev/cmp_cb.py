#!/usr/bin/env python3
"""Dev: side-by-side table of tools/conv_bench.py JSON logs (fwd | dgrad | wgrad ms; * = fastest).
usage: tools/dev/cmp_cb.py a.log b.log ..."""
import json
import os
import sys

runs = sys.argv[1:]
names = [os.path.basename(os.path.dirname(r)) + '/' + os.path.basename(r)[:-4] for r in runs]
d = {}
tot = {n: [0.0, 0.0, 0.0] for n in names}
for r, n in zip(runs, names):
    for line in open(r):
        if line.startswith('{'):
            for L in json.loads(line)['layers']:
                v = (L['fwd_ms'], L['dgrad_ms'], L['wgrad_ms'])
                d.setdefault(L['layer'], {})[n] = v
                for i in range(3):
                    tot[n][i] += v[i]
print('\n'.join(f'  [{i}] {n}' for i, n in enumerate(names)))
for k, r in list(d.items()) + [('TOTAL', tot)]:
    s = f'{k:26s}'
    for i in range(3):
        vals = [r[n][i] if n in r else float('nan') for n in names]
        b = min(vals)
        s += ' |' + ''.join(('*' if v == b else ' ') + f'{v:7.3f}' for v in vals)
    print(s)
