#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 ``--pmc`` run (rocpd SQLite ``*_results.db``).

Usage: python tools/pmc_summary.py gpurun_out/pmcX/pmc_results.db [--filter conv] [--top 20]
Prints, per kernel (short name), the dispatch count, mean duration and the mean of every collected
counter per dispatch, plus derived ratios when their inputs were collected:
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * n_SIMD)    (fraction of SIMD-cycles in MFMA)
  lds_util    = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE * n_CU)             (LDS array busy fraction)
  bank_confl  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  hbm_TBps    = FETCH_SIZE (KB, doubled per the gfx950 half-count) / duration
"""
import argparse
import collections
import re
import sqlite3

N_CU, N_SIMD, N_XCD = 256, 1024, 8


def short(name):
    name = re.sub(r'\(anonymous namespace\)::', '', name)
    m = re.match(r'(?:void )?([\w:]+)(<[^()]*>)?', name)
    return (m.group(1) + (m.group(2) or '')) if m else name[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--filter', default='')
    ap.add_argument('--top', type=int, default=30)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = db.execute('select dispatch_id, kernel_name, counter_name, value, duration from counters_collection').fetchall()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(dict)
    for did, kn, cn, v, d in rows:
        k = short(kn)
        if a.filter and a.filter not in k:
            continue
        per[k][cn] += v
        disp[k].add(did)
        dur[k][did] = d
    out = []
    for k, cs in per.items():
        n = len(disp[k])
        t = sum(dur[k].values()) / n
        avg = {c: v / n for c, v in cs.items()}
        out.append((t * n, k, n, t, avg))
    for tot, k, n, t, avg in sorted(out, reverse=True)[:a.top]:
        g = avg.get('GRBM_GUI_ACTIVE')
        if g:
            g = g / N_XCD   # GRBM_GUI_ACTIVE is summed over the 8 XCDs: per-XCD busy cycles of the dispatch
        der = []
        if g and 'SQ_VALU_MFMA_BUSY_CYCLES' in avg:
            der.append(f"mfma_util={avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (g * N_SIMD):.3f}")
        if g and 'SQ_LDS_IDX_ACTIVE' in avg:
            der.append(f"lds_util={avg['SQ_LDS_IDX_ACTIVE'] / (g * N_CU):.3f}")
        if avg.get('SQ_LDS_IDX_ACTIVE') and 'SQ_LDS_BANK_CONFLICT' in avg:
            der.append(f"bank_confl={avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE']:.3f}")
        if 'FETCH_SIZE' in avg and t > 0:
            der.append(f"hbm_TBps={2 * avg['FETCH_SIZE'] * 1024 / t / 1e3:.2f}")
        print(f'{k[:70]:70s} n={n:4d} {t / 1e3:9.1f}us  ' + ' '.join(der))
        print('      ' + ' '.join(f'{c}={v:.3g}' for c, v in sorted(avg.items())))


if __name__ == '__main__':
    main()
