#!/usr/bin/env python3
"""Summarise a rocprofv3 ``*_results.db`` (rocpd SQLite) into a per-kernel time table.

Usage: python tools/rocpd_summary.py path/to/results.db [--top 40] [--steps N] [--group] [--window]
``--group`` buckets kernels into families (conv fwd / dgrad / wgrad / BN / elementwise ...).
``--window``: only the last ``--steps`` steady-state steps, marker to marker (the once-per-step fused
optimizer kernel, ``--marker``) -- excludes warmup / graph-capture work (e.g. the setup copies).
``--sequence``: instead, every launch of the last step in issue order (index, ms, grid, name) -- which
launch of a kernel family is which layer.
"""
import argparse
import collections
import re
import sqlite3

FAMILIES = [
    ('conv(MIOpen/ours)', r'conv|igemm|Conv|naive_conv|implicit|gemm|Cijk|MIOpen|xdlops|batched_transpose|transpose'),
    ('batchnorm', r'[Bb]atch[Nn]orm|bn_|welford|MIOpenBatchNorm'),
    ('elementwise', r'elementwise|vectorized|unrolled_elementwise|Elementwise'),
    ('reduce', r'reduce|Reduce'),
    ('optimizer/foreach', r'foreach|multi_tensor|adam|Adam'),
    ('upsample/pool', r'upsample|pool|Pool'),
    ('loss', r'nll|softmax|log_softmax|cross'),
    ('copy', r'copy|Copy|fill'),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--top', type=int, default=40)
    ap.add_argument('--steps', type=int, default=1)
    ap.add_argument('--group', action='store_true')
    ap.add_argument('--window', action='store_true')
    ap.add_argument('--marker', default=r'adam_kernel|sgd_kernel|Adam')
    ap.add_argument('--sequence', action='store_true')
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    if a.sequence:
        try:
            seq = db.execute('select name, start, end, grid_size_x, workgroup_size_x from kernels order by start').fetchall()
        except sqlite3.OperationalError:
            seq = [r + (0, 0) for r in db.execute('select name, start, end from kernels order by start').fetchall()]
        marks = [i for i, r in enumerate(seq) if re.search(a.marker, r[0])]
        if len(marks) < 2:
            raise SystemExit('--sequence: marker found fewer than 2 times')
        for i, (name, s0, e0, gx, wx) in enumerate(seq[marks[-2] + 1:marks[-1] + 1]):
            nm = re.sub(r'\(anonymous namespace\)::', '', name)
            nm = re.sub(r'\((ConvArgs|FusedBwdArgs|WgradPtrs|unsigned|float|long|const|\(anon).*$', '', nm)
            print(f'{i:5d} {(e0 - s0) / 1e6:8.3f} {gx // max(wx, 1):7d}  {nm[:110]}')
        return
    rows = db.execute('select name, start, end from kernels order by start').fetchall()
    if a.window:
        marks = [i for i, r in enumerate(rows) if re.search(a.marker, r[0])]
        if len(marks) < a.steps + 1:
            raise SystemExit(f'--window: marker found {len(marks)} times, need {a.steps + 1}')
        rows = rows[marks[-a.steps - 1] + 1:marks[-1] + 1]
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for name, s, e in rows:
        tot[name] += (e - s) / 1e6
        cnt[name] += 1
    total = sum(tot.values())
    span = (max(r[2] for r in rows) - min(r[1] for r in rows)) / 1e6 if rows else 0
    print(f'kernels={len(rows)} busy_ms={total:.2f} span_ms={span:.2f} per_step_busy_ms={total / a.steps:.2f}')
    if a.group:
        fam = collections.defaultdict(float)
        fcnt = collections.Counter()
        for n, t in tot.items():
            for fname, pat in FAMILIES:
                if re.search(pat, n):
                    break
            else:
                fname = 'other'
            fam[fname] += t
            fcnt[fname] += cnt[n]
        for f, t in sorted(fam.items(), key=lambda x: -x[1]):
            print(f'{t:10.2f} ms {100 * t / total:5.1f}% {fcnt[f]:7d}  {f}')
        print()
    for n, t in sorted(tot.items(), key=lambda x: -x[1])[:a.top]:
        print(f'{t:10.2f} ms {100 * t / total:5.1f}% {cnt[n]:6d}  {n[:150]}')


if __name__ == '__main__':
    main()
