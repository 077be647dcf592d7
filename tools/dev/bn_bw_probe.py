"""Dev: achieved HBM bandwidth of the BatchNorm passes at the DUCKNet-17 bs320 level shapes, against a plain
copy (torch clone) of the same bytes -- how far each pass is from its byte floor.

    python tools/dev/bn_bw_probe.py [--batch 320] [--levels 1,2,3,4,5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from medical_segmentation_pytorch_amd.ops._ext import require  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=320)
    ap.add_argument('--levels', default='1,2,3,4,5')
    ap.add_argument('--iters', type=int, default=10)
    args = ap.parse_args()
    C = require()
    dev = torch.device('cuda:0')
    for lv in (int(v) for v in args.levels.split(',')):
        hw = 352 >> (lv - 1)
        c = 17 << (lv - 1)
        Cp = (c + 7) // 8 * 8
        P = args.batch * hw * hw
        nbytes = P * Cp * 2
        mk = lambda: (torch.randn(P, Cp, device=dev) * 0.5).bfloat16()   # noqa: E731
        stats = torch.zeros(4, Cp, device=dev)
        stats[0] = 1.1
        stats[1] = 0.05
        stats[3] = 1.0
        coef = torch.randn(3, Cp, device=dev) * 0.01
        y, dz, dy = mk(), mk(), torch.empty(P, Cp, dtype=torch.bfloat16, device=dev)
        res = {'level': lv, 'P': P, 'Cp': Cp, 'tensor_MB': round(nbytes / 1e6, 1)}
        ms = timed(lambda: y.clone(), args.iters)
        res['copy'] = (round(ms, 3), round(2 * nbytes / ms / 1e9, 2))
        part = torch.empty(C.bn_partial_blocks(P, Cp), 2, Cp, device=dev)
        ms = timed(lambda: C.bn_act_bwd_partial(dz, y, stats, part, P, Cp, True), args.iters)
        res['bwd_partial'] = (round(ms, 3), round(2 * nbytes / ms / 1e9, 2))
        ms = timed(lambda: C.bn_act_bwd_apply(dz, y, stats, coef, dy, P, Cp, True), args.iters)
        res['bwd_apply'] = (round(ms, 3), round(3 * nbytes / ms / 1e9, 2))
        ys = [mk() for _ in range(6)]
        out = torch.empty_like(y)
        sts = [stats] * 6
        for k in (2, 6):
            ms = timed(lambda: C.sum_stats(ys[:k], out, part, P, Cp, sts[:k], (1 << k) - 1), args.iters)
            res[f'sum_stats{k}'] = (round(ms, 3), round((k + 1) * nbytes / ms / 1e9, 2))
        del ys, out
        res['unit'] = '(ms, TB/s)'
        print(json.dumps(res), flush=True)
        del y, dz, dy
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
