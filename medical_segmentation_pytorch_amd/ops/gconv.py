"""Grouped convolution on the HIP kernels (``csrc/gconv.hip``): ResNeXt's grouped 3x3 (torchvision
``Bottleneck.conv2``, groups 32) inside the fused graph -- the last conv that used to run on MIOpen.

NHWC bf16 maps with C % 8 == 0 (unpadded: ResNeXt widths are multiples of 8); fp32 weights repacked to
[T][C][CG] per call.  The weight gradient is reduced over pixel slices in a fixed order (``colsum``):
bitwise deterministic.  Reference: models/__init__.py:8-10 (smp encoders, resnext50_32x4d).
"""
from __future__ import annotations

import torch

from ._ext import require


def _taps(conv):
    kh, kw = conv.kernel_size
    (ph, pw), (dh, dw) = tuple(conv.padding), tuple(conv.dilation)
    dy = [r * dh - ph for r in range(kh) for _ in range(kw)]
    dx = [c * dw - pw for _ in range(kh) for c in range(kw)]
    return dy, dx


def _out_size(n, k, s, p, d):
    return (n + 2 * p - d * (k - 1) - 1) // s + 1


class _GConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, cfg):
        C = require()
        x = x.contiguous()
        (kh, kw), (sh, sw), (ph, pw), (dh, dw), groups, dy, dx = cfg
        N, H, W, Cc = x.shape
        CG = Cc // groups
        T = kh * kw
        # w[t][co][cil] = W[co][cil][r][c]
        wp = weight.detach().float().reshape(Cc, CG, T).permute(2, 0, 1).contiguous()
        oh, ow = _out_size(H, kh, sh, ph, dh), _out_size(W, kw, sw, pw, dw)
        y = torch.empty(N, oh, ow, Cc, dtype=torch.bfloat16, device=x.device)
        C.gconv_fwd(x, wp, y, CG, sh, dy, dx)
        ctx.save_for_backward(x, wp)
        ctx.cfg = (kh, kw, sh, CG, T, dy, dx)
        return y

    @staticmethod
    def backward(ctx, g):
        C = require()
        x, wp = ctx.saved_tensors
        kh, kw, stride, CG, T, dy, dx = ctx.cfg
        g = g.contiguous()
        N, H, W, Cc = x.shape
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            C.gconv_dgrad(g, wp, gx, CG, stride, dy, dx)
        gw = None
        if ctx.needs_input_grad[1]:
            P = N * g.shape[1] * g.shape[2]
            nib = CG // 8 if CG >= 8 else 1
            S = C.gconv_wgrad_slices(P, Cc, CG, T)
            part = torch.empty(S, T * (Cc // 8) * nib * 64, dtype=torch.float32, device=x.device)
            C.gconv_wgrad(x, g, part, CG, stride, dy, dx)
            red = torch.empty(part.shape[1], dtype=torch.float32, device=x.device)
            C.colsum(part, red, False)
            nob = Cc // 8
            red = red.view(T, nib, nob, 8, 8)   # [t][input block][output block][e][k]
            if CG >= 8:   # cil = 8*ib + k
                gw = red.permute(2, 3, 1, 4, 0).reshape(Cc, CG, T)
            else:         # the 8-channel block holds 8/CG groups: output e reads inputs (e//CG)*CG + cil
                e = torch.arange(8, device=x.device)
                idx = ((e // CG) * CG).view(8, 1) + torch.arange(CG, device=x.device).view(1, CG)
                sel = torch.gather(red[:, 0], 3, idx.view(1, 1, 8, CG).expand(T, nob, 8, CG))
                gw = sel.permute(1, 2, 3, 0).reshape(Cc, CG, T)
            gw = gw.reshape(Cc, CG, kh, kw).contiguous()
        return gx, gw, None


def gconv(x, conv: torch.nn.Conv2d):
    """``conv`` (groups > 1, in == out channels, no bias) on an NHWC bf16 map [N, H, W, C]."""
    assert conv.groups > 1 and conv.in_channels == conv.out_channels and conv.bias is None
    assert x.shape[-1] == conv.in_channels and conv.in_channels % 8 == 0, 'grouped conv input must be unpadded'
    dy, dx = _taps(conv)
    cfg = (tuple(conv.kernel_size), tuple(conv.stride), tuple(conv.padding), tuple(conv.dilation), conv.groups, dy,
           dx)
    assert conv.stride[0] == conv.stride[1], 'gconv: square stride'
    return _GConv.apply(x, conv.weight, cfg)


def gconv_reference(x, conv):
    import torch.nn.functional as F
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), conv.weight.float(), None, conv.stride, conv.padding, conv.dilation,
                 conv.groups)
    return y.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()
