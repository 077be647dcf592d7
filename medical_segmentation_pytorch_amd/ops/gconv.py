"""Grouped convolution on the HIP kernels (``csrc/gconv.hip``): ResNeXt's grouped 3x3 (torchvision
``Bottleneck.conv2``, groups 32) inside the fused graph -- the last conv that used to run on MIOpen.

NHWC bf16 maps with C % 8 == 0 (unpadded: ResNeXt widths are multiples of 8); fp32 weights repacked to
[T][C][CG] per call.  3x3 convs with C % 16 == 0 and CG <= 64 (depthwise included) run forward and data-gradient on the MFMA
kernel (``gconv_mfma``: block-diagonal weights over a max(16, CG)-channel window, packed per MFMA lane by
``_mfma_pack``) and so does the weight-gradient (``gconv_wgrad_mfma``: the dense 16-co x 9-tap x window
tiles, reduced over pixel slices by ``colsum``, block diagonal gathered by ``_wgrad_diag_index``); env
MSP_GCONV_MFMA=0 keeps the VALU kernels (A/B).  The weight gradient is reduced over pixel slices in a fixed order (``colsum``):
bitwise deterministic.  Reference: models/__init__.py:8-10 (smp encoders, resnext50_32x4d).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ._ext import require

_MFMA = os.environ.get('MSP_GCONV_MFMA', '1') != '0'
# smallest group width on the MFMA path (env MSP_GCONV_MFMA_MINCG, A/B).  Depthwise (CG = 1) included: only
# 1/16 of the MFMA work is useful, but the VALU kernels are slower still -- smp-Unet MobileNetV2 bs64
# 2020 -> 2947 img/s (profiles/r05/gconv/bench_smp_unet_mobilenetv2_bs64_*.json)
_MFMA_MINCG = int(os.environ.get('MSP_GCONV_MFMA_MINCG', '1'))
_PACK_IDX = {}


def _mfma_ok(C, CG, T):
    # the MFMA kernels take a window of KW = max(16, CG) in {16, 32, 64} channels that holds whole groups:
    # CG must divide 16 or be 32 / 64 (CG = 24, 48 would hit a kernel check, CG = 12 would straddle windows)
    return (_MFMA and T == 9 and C % 16 == 0 and _MFMA_MINCG <= CG <= 64
            and (16 % CG == 0 or CG in (32, 64)))


def _mfma_pack_index(C, CG, T, trans, device):
    """Gather index into [T*C*CG + 1] (the last slot a zero) building the MFMA A operands: [C/16][NST][64][8]
    with lane l = row l % 16 (output channel co = 16*ob + l % 16), k = 32*s + 8*(l // 16) + j -> tap k // KW,
    window channel (co // KW) * KW + k % KW; block-diagonal (other groups and padding taps read the zero).
    fwd: w[tap][co][cin - g(co)]; trans (data-gradient, output channel = an input channel ci): w[tap][cin][ci - g(ci)]."""
    key = (C, CG, T, trans, str(device))
    idx = _PACK_IDX.get(key)
    if idx is None:
        KW = max(16, CG)
        nst = (T * KW + 31) // 32
        ob = np.arange(C // 16).reshape(-1, 1, 1, 1)
        st = np.arange(nst).reshape(1, -1, 1, 1)
        ln = np.arange(64).reshape(1, 1, -1, 1)
        j = np.arange(8).reshape(1, 1, 1, -1)
        co = 16 * ob + ln % 16
        k = 32 * st + 8 * (ln // 16) + j
        tap = k // KW
        cin = (co // KW) * KW + k % KW
        ok = (tap < T) & (cin // CG == co // CG)
        if trans:
            flat = tap * C * CG + cin * CG + (co - (co // CG) * CG)
        else:
            flat = tap * C * CG + co * CG + (cin - (cin // CG) * CG)
        flat = np.where(ok, flat, T * C * CG)
        idx = torch.from_numpy(flat.reshape(-1).astype(np.int64)).to(device)
        _PACK_IDX[key] = idx
    return idx


def _wgrad_diag_index(C, CG, T, device):
    """Gather index from the MFMA weight-gradient tiles red [C/16][T*KW/16][16 co][16 ch] (tile = tap * KW/16 +
    16-ch sub-block of the co block's KW window) to dW [C][CG][T] (the block diagonal)."""
    key = ('wg', C, CG, T, str(device))
    idx = _PACK_IDX.get(key)
    if idx is None:
        KW = max(16, CG)
        co = np.arange(C).reshape(-1, 1, 1)
        cil = np.arange(CG).reshape(1, -1, 1)
        t = np.arange(T).reshape(1, 1, -1)
        wch = (co // CG) * CG + cil - (co // KW) * KW
        tile = t * (KW // 16) + wch // 16
        flat = (((co // 16) * (T * KW // 16) + tile) * 16 + co % 16) * 16 + wch % 16
        idx = torch.from_numpy(np.broadcast_to(flat, (C, CG, T)).reshape(-1).astype(np.int64)).to(device)
        _PACK_IDX[key] = idx
    return idx


def _mfma_pack(wp, C, CG, T, trans):
    flat = torch.cat([wp.reshape(-1), wp.new_zeros(1)])
    return flat[_mfma_pack_index(C, CG, T, trans, wp.device)].to(torch.bfloat16)


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
        if _mfma_ok(Cc, CG, T):
            C.gconv_mfma(x, _mfma_pack(wp, Cc, CG, T, False), y, max(16, CG), sh, False, dy, dx)
        else:
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
            if _mfma_ok(Cc, CG, T):
                C.gconv_mfma(g, _mfma_pack(wp, Cc, CG, T, True), gx, max(16, CG), stride, True, dy, dx)
            else:
                C.gconv_dgrad(g, wp, gx, CG, stride, dy, dx)
        gw = None
        if ctx.needs_input_grad[1] and _mfma_ok(Cc, CG, T):
            P = N * g.shape[1] * g.shape[2]
            KW = max(16, CG)
            S = C.gconv_wgrad_mfma_slices(P, Cc)
            part = torch.empty(S, (Cc // 16) * (T * KW // 16) * 256, dtype=torch.float32, device=x.device)
            C.gconv_wgrad_mfma(x, g, part, KW, stride, dy, dx)
            red = torch.empty(part.shape[1], dtype=torch.float32, device=x.device)
            C.colsum(part, red, False)
            gw = red[_wgrad_diag_index(Cc, CG, T, x.device)].view(Cc, CG, kh, kw)
        elif ctx.needs_input_grad[1]:
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
