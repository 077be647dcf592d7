#!/usr/bin/env python3
"""Dev: time one conv_bwd_fused launch (csrc/conv_bwd.hip) at the DUCKNet-17 L1 chain-conv shape (17 -> 24
padded channels, 3x3, deferred dY + x prologue + BN epilogue: the <8, true, true, true> instantiation).
python tools/dev/fused_bwd_bench.py [batch] [size] [dilation] [go]  (go = 2: the ResidualBlock's 3x3 + 1x1 pair)   (MSP_C_SO=<variant .so> for knock-out builds)"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from medical_segmentation_pytorch_amd.ops._ext import require  # noqa: E402
from medical_segmentation_pytorch_amd.ops.conv import Branch, ConvPlan, _taps  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 320
    s = int(sys.argv[2]) if len(sys.argv) > 2 else 352
    dil = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    go = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    fwd = len(sys.argv) > 5 and sys.argv[5] == 'fwd'
    C = require()
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    m = nn.Conv2d(17, 17, 3, 1, dil, dil, bias=False).to(dev)
    branches = [Branch(m.weight, 0, 0, 9)]
    if go == 2:
        branches.append(Branch(nn.Conv2d(17, 17, 1, bias=False).to(dev).weight, 1, 4, 1))
    plan = ConvPlan(3, 3, 17, 17, branches, padding=(dil, dil), dilation=(dil, dil), Go=go)
    cp = plan.Cgi
    dims = plan.fwd_dims(n, s, s, s, s)
    tdy, tdx = _taps(plan.taps_fwd)
    nblk = C.conv_bwd_fused_blocks(dims, tdy, tdx)
    wd, kp = plan.pack_dgrad(dev)

    def t(c):
        return torch.randn(n, s, s, c, device=dev).to(torch.bfloat16)
    dz, y2, x = t(cp), t(cp), t(cp)
    y1 = x if os.environ.get('FB_SEPARATE_Y1') != '1' else t(cp)   # the chain case: BN1's input IS x
    st = torch.rand(4, cp, device=dev) + 0.5
    coef = torch.randn(3, cp, device=dev) * 0.1
    dxt = torch.empty_like(x)
    part = torch.empty(nblk, 2, cp, device=dev)
    dwp = torch.empty(nblk * plan.rows * plan.T * plan.Cip, device=dev)

    kw2 = dict(dz2=t(cp), gy2=t(cp), gs2=st, gk2=coef, grelu2=True, t1=4) if go == 2 else {}

    if fwd:   # the forward mode (conv_fwd_fused): y = conv(relu(BN(x))) + BN statistics
        wp = plan.pack_fwd(dev)
        fd = plan.fwd_dims(n, s, s, s, s)
        fdy, fdx = _taps(plan.taps_fwd)
        assert C.conv_fwd_fused_ok(fd, fdy, fdx)
        fpart = torch.empty(C.conv_stat_blocks(fd, fdy, fdx), 2, plan.rows, device=dev)
        xin, yout = t(cp), torch.empty(n, s, s, plan.Cgo, device=dev, dtype=torch.bfloat16)

    def run():
        if fwd:
            C.conv_fwd([xin], wp, [yout], None, fpart, fd, fdy, fdx, False, [st], 1)
            return
        C.conv_bwd_fused(dz, y2, st, coef, True, x, st, True, wd, kp, dxt, y1, coef, True, part, dwp, dims, tdy, tdx,
                         **kw2)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    a.record()
    for _ in range(reps):
        run()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    px = n * s * s
    hbm = px * cp * 2 * (4 + 1 + 2 * (go - 1)) * 1.2   # dz, y2 (per group), x, y1 (+ halo) read, dx written
    if fwd:
        hbm = px * cp * 2 * (1.2 + 1)   # x (+ halo) read, y written
    print(f'{"conv_fwd_fused" if fwd else "conv_bwd_fused"} N={n} {s}x{s} d={dil} go={go} blocks={nblk}: {ms:.3f} ms  (~{hbm / ms / 1e9:.2f} TB/s of '
          f'{hbm / 1e9:.2f} GB)  variant={os.environ.get("MSP_C_SO", "default")}')


if __name__ == '__main__':
    main()
