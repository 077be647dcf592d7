#!/usr/bin/env python3
"""Where does a training step's wall time go that no kernel accounts for?

Reads a rocprofv3 ``*_results.db`` (rocpd SQLite, ``--kernel-trace``), cuts the trace into steps at a
marker kernel that runs once per step (default: the fused Adam kernel), and for the last ``--steps``
steps prints span, kernel-busy time (union of intervals, so concurrent streams are not double counted),
idle time, a histogram of the idle gaps between consecutive kernels, and the largest gaps with the
kernels on either side.

Usage: python tools/rocpd_timeline.py results.db [--marker adam] [--steps 5] [--top 25]
"""
import argparse
import collections
import re
import sqlite3


def short(name):
    name = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return re.sub(r'\(.*', '', name)[:60]


def union_busy(iv):
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    return busy


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--marker', default=r'adam|Adam')
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--top', type=int, default=25)
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute('select name, start, end from kernels order by start').fetchall()
    marks = [i for i, r in enumerate(rows) if re.search(a.marker, r[0])]
    if len(marks) < 2:
        print(f'marker {a.marker!r} found {len(marks)} times; need >= 2')
        return
    bounds = list(zip(marks[:-1], marks[1:]))[-a.steps:]
    print(f'kernels={len(rows)} marker hits={len(marks)}; analysing the last {len(bounds)} steps '
          f'(marker to marker)')
    gap_hist = collections.Counter()
    gap_total = collections.Counter()
    top = []
    edges = [0, 5, 10, 20, 50, 100, 1000, 10 ** 9]
    for k, (i0, i1) in enumerate(bounds):
        seg = rows[i0 + 1:i1 + 1]
        iv = [(s, e) for _, s, e in seg]
        span = (seg[-1][2] - rows[i0][2]) / 1e6
        busy = union_busy(iv) / 1e6
        print(f'step {k}: kernels={len(seg)} span={span:.2f} ms busy={busy:.2f} ms idle={span - busy:.2f} ms '
              f'({100 * (span - busy) / span:.1f}%)')
        prev_end, prev_name = rows[i0][2], rows[i0][0]
        for name, s, e in seg:
            g = (s - prev_end) / 1e3   # us
            if g > 0:
                for lo, hi in zip(edges[:-1], edges[1:]):
                    if lo <= g < hi:
                        gap_hist[(lo, hi)] += 1
                        gap_total[(lo, hi)] += g
                        break
                top.append((g, prev_name, name))
            if e > prev_end:
                prev_end, prev_name = e, name
    n = len(bounds)
    print('\nidle gaps between kernels, per step:')
    for lo, hi in zip(edges[:-1], edges[1:]):
        c = gap_hist[(lo, hi)]
        print(f'  {lo:>5}-{hi if hi < 10 ** 9 else "inf":>5} us: {c / n:8.1f} gaps  {gap_total[(lo, hi)] / n / 1e3:8.2f} ms')
    print(f'\nlargest {a.top} gaps (us, kernel before -> kernel after):')
    for g, p, q in sorted(top, reverse=True)[:a.top]:
        print(f'  {g:9.1f}  {short(p)}  ->  {short(q)}')
    pair = collections.Counter()
    pair_t = collections.Counter()
    for g, p, q in top:
        key = (short(p), short(q))
        pair[key] += 1
        pair_t[key] += g
    print('\nidle time by (kernel before -> kernel after) family, per step:')
    for key, t in sorted(pair_t.items(), key=lambda x: -x[1])[:a.top]:
        print(f'  {t / n / 1e3:8.2f} ms {pair[key] / n:7.1f}x  {key[0]}  ->  {key[1]}')


if __name__ == '__main__':
    main()
