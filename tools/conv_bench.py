#!/usr/bin/env python3
"""Per-layer microbenchmark of the implicit-GEMM conv kernels (fwd / dgrad / wgrad) on the
DUCKNet-17 layer shapes at the headline config (batch 16, 352x352), vs MIOpen (torch bf16
channels_last).  Prints time, achieved TFLOP/s (useful FLOPs, unpadded) and a JSON summary.

    python tools/conv_bench.py [--batch 16] [--size 352] [--iters 20] [--miopen]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from medical_segmentation_pytorch_amd.ops.conv import Branch, ConvPlan, conv  # noqa: E402


def layers(b=17):
    L = []
    for lvl, c in enumerate([b, 2 * b, 4 * b, 8 * b, 16 * b]):
        L.append((f'L{lvl + 1} 3x3 {c}->{c}', lvl, c, c, (3, 3), 1, (1, 1), (1, 1), 1))
        L.append((f'L{lvl + 1} 3x3d3 {c}->{c}', lvl, c, c, (3, 3), 1, (3, 3), (3, 3), 1))
        L.append((f'L{lvl + 1} 1x7 {c}->{c}', lvl, c, c, (1, 7), 1, (0, 3), (1, 1), 1))
        L.append((f'L{lvl + 1} fused8 {c}->8x{c}', lvl, c, c, (3, 3), 1, (1, 1), (1, 1), 8))
        # DUCK first-conv decompositions: the 5 3x3 convs (in 1, 2 or 3 launches) + the 3 1x1 shortcuts
        for gsz in (5, 3, 2):
            L.append((f'L{lvl + 1} fused{gsz} {c}->{gsz}x{c}', lvl, c, c, (3, 3), 1, (1, 1), (1, 1), gsz))
        L.append((f'L{lvl + 1} fused3-1x1 {c}->3x{c}', lvl, c, c, (1, 1), 1, (0, 0), (1, 1), 3))
        L.append((f'L{lvl + 1} 3x3s2 {c}->{2 * c}', lvl, c, 2 * c, (3, 3), 2, (1, 1), (1, 1), 1))
    # the first DUCK reads the 3-channel image (in_bn(x)): its first convs at 3 -> b
    L.append((f'L1in fused8 3->8x{b}', 0, 3, b, (3, 3), 1, (1, 1), (1, 1), 8))
    L.append((f'L1in fused5 3->5x{b}', 0, 3, b, (3, 3), 1, (1, 1), (1, 1), 5))
    L.append((f'L1in fused3-1x1 3->3x{b}', 0, 3, b, (1, 1), 1, (0, 0), (1, 1), 3))
    L.append(('L6 3x3 544->544', 5, 32 * b, 32 * b, (3, 3), 1, (1, 1), (1, 1), 1))
    L.append(('L6 fused2 544->2x544', 5, 32 * b, 32 * b, (3, 3), 1, (1, 1), (1, 1), 2))
    return L


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--size', type=int, default=352)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--miopen', action='store_true')
    ap.add_argument('--halo', type=int, default=1, help='1: halo-tiled stride-1 kernel where eligible, 0: gather only')
    ap.add_argument('--split', type=int, default=1, help='halo split-bank tile image: 0 never, 1 occupancy-preserving '
                    '(default), 2 wherever it fits (csrc/conv.hip halo_phys)')
    ap.add_argument('--gemm-cfg', type=int, default=-1, help='force one LDS-DMA GEMM tile configuration (A/B)')
    ap.add_argument('--only', default='', help='substring filter on layer names')
    ap.add_argument('--levels', default='', help='comma list of levels to run (e.g. 3,4,5,6)')
    ap.add_argument('--prologue', action='store_true',
                    help='input is a deferred BN(+ReLU) output: fwd / wgrad apply the BN prologue while staging')
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    from medical_segmentation_pytorch_amd.ops import _ext
    C = _ext.require()
    C.conv_set_halo(bool(a.halo))
    C.conv_set_halo_split(a.split)
    C.conv_gemm_force_cfg(a.gemm_cfg)
    res = []
    tot = {'fwd': 0.0, 'dgrad': 0.0, 'wgrad': 0.0}
    for name, lvl, ci, co, k, s, p, d, groups in layers():
        if a.only and a.only not in name:
            continue
        if a.levels and str(lvl + 1) not in a.levels.split(','):
            continue
        hw = a.size >> lvl
        n = a.batch
        convs = [nn.Conv2d(ci, co, k, s, p, d, bias=False).to(dev) for _ in range(groups)]
        br = [Branch(c.weight, g, 0, k[0] * k[1]) for g, c in enumerate(convs)]
        plan = ConvPlan(k[0], k[1], ci, co, br, stride=s, padding=p, dilation=d, Go=groups)
        x = torch.randn(n, hw, hw, plan.Cgi, device=dev).to(torch.bfloat16)
        x[..., ci:] = 0
        oh, ow = plan.out_hw(hw, hw)
        dims = plan.fwd_dims(n, hw, hw, oh, ow)
        dy, dx = [t[0] for t in plan.taps_fwd], [t[1] for t in plan.taps_fwd]
        wp = plan.pack_fwd(dev)
        ys = [torch.empty(n, oh, ow, plan.Cgo, device=dev, dtype=torch.bfloat16) for _ in range(groups)]
        nblk = C.conv_stat_blocks(dims, dy, dx)
        part = torch.empty(nblk, 2, plan.rows, device=dev)
        xc, xr = [], 0
        if a.prologue:   # BN stats rows (scale, shift, mean, invstd) of the input channels
            st = torch.zeros(4, plan.Cgi, device=dev)
            st[0, :ci] = torch.rand(ci, device=dev) + 0.5
            st[1, :ci] = torch.randn(ci, device=dev) * 0.1
            xc, xr = [st], 1
        t_f = timeit(lambda: C.conv_fwd([x], wp, ys, None, part, dims, dy, dx, False, xc, xr), a.iters)
        wd, Kp_d = plan.pack_dgrad(dev)
        gys = [torch.randn_like(y, dtype=torch.float32).to(torch.bfloat16) for y in ys]
        dxs = [torch.empty_like(x)]
        dims_d = [n, oh, ow, plan.Go, plan.Cgo, hw, hw, 1, plan.Cgi, ci, plan.T, Kp_d, s]
        bdy, bdx = [t[0] for t in plan.taps_bwd], [t[1] for t in plan.taps_bwd]
        t_d = timeit(lambda: C.conv_fwd(gys, wd, dxs, None, None, dims_d, bdy, bdx, s > 1), a.iters)
        dwp = torch.empty(C.conv_wgrad_replicas(dims, dy, dx, False, False, bool(xc)) * plan.rows * plan.T * plan.Cip, device=dev)
        t_w = timeit(lambda: C.conv_wgrad(gys, [x], dwp, dims, dy, dx, False, xc, xr), a.iters)
        flops = 2.0 * n * oh * ow * co * ci * k[0] * k[1] * groups
        row = {'layer': name, 'fwd_ms': round(t_f, 4), 'dgrad_ms': round(t_d, 4), 'wgrad_ms': round(t_w, 4),
               'fwd_tflops': round(flops / t_f / 1e9, 1), 'dgrad_tflops': round(flops / t_d / 1e9, 1),
               'wgrad_tflops': round(flops / t_w / 1e9, 1)}
        if a.miopen:
            xm = torch.randn(n, ci, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
            wm = torch.randn(co * groups, ci, *k, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
            row['miopen_fwd_ms'] = round(timeit(lambda: F.conv2d(xm, wm, None, s, p, d), a.iters), 4)
        row['halo_fwd'] = bool(C.conv_uses_halo(dims, dy, dx, False))
        row['halo_dgrad'] = bool(C.conv_uses_halo(dims_d, bdy, bdx, s > 1))
        res.append(row)
        tot['fwd'] += t_f; tot['dgrad'] += t_d; tot['wgrad'] += t_w
        print(f"{name:28s} fwd {t_f:7.3f} ms ({row['fwd_tflops']:6.1f} TF)  dgrad {t_d:7.3f} ({row['dgrad_tflops']:6.1f})"
              f"  wgrad {t_w:7.3f} ({row['wgrad_tflops']:6.1f})" +
              (f"  miopen-fwd {row['miopen_fwd_ms']:7.3f}" if a.miopen else ''), flush=True)
    print(json.dumps({'batch': a.batch, 'size': a.size, 'halo': a.halo, 'split': a.split, 'layers': res, 'totals_ms': tot}))


if __name__ == '__main__':
    main()
