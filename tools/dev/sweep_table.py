#!/usr/bin/env python3
"""Tabulate tools/conv_bench.py JSON lines of several runs side by side (fwd/dgrad ms per layer).
    python tools/dev/sweep_table.py dir name1 name2 ...   (reads dir/<name>.log)"""
import json
import sys

d, names = sys.argv[1], sys.argv[2:]
rows = {}
for n in names:
    for line in open(f'{d}/{n}.log'):
        if line.startswith('{'):
            for L in json.loads(line)['layers']:
                rows.setdefault(L['layer'], {})[n] = (L['fwd_ms'], L['dgrad_ms'], L['wgrad_ms'])
print(f"{'layer':28s}" + ''.join(f"{n:>17s}" for n in names))
for k, v in rows.items():
    print(f"{k:28s}" + ''.join(f"{v[n][0]:8.3f}/{v[n][1]:7.3f} " if n in v else ' ' * 17 for n in names))
