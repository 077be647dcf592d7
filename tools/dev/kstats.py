#!/usr/bin/env python3
"""Dev: per-kernel-name duration histogram of one rocprofv3 kernel-trace DB, grouped by grid size (the last
``--steps`` steps' window of tools/rocpd_summary.py is not applied: all dispatches).
usage: tools/dev/kstats.py run_results.db <name substring> [--steps N]"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
pat = sys.argv[2]
steps = int(sys.argv[sys.argv.index('--steps') + 1]) if '--steps' in sys.argv else 1
rows = db.execute('select name, duration, grid_x, workgroup_x from kernels').fetchall()
g = collections.defaultdict(list)
for n, d, gx, wx in rows:
    if pat in n:
        g[(n.split('(')[0][-50:], gx // max(wx, 1), wx)].append(d / 1e3)
tot = 0
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    tot += sum(v)
    print(f'{k[0]:50s} blocks={k[1]:8d} wg={k[2]:4d} n={len(v) / steps:6.1f}/step  med={v[len(v) // 2]:8.1f} us  '
          f'sum/step={sum(v) / steps / 1e3:7.2f} ms')
print(f'total/step {tot / steps / 1e3:.2f} ms')
