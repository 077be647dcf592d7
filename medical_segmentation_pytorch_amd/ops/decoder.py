"""Autograd ops over the decoder-hub kernels (``csrc/decoder.hip``) for NHWC bf16 feature maps.

These are the non-conv operations of the smp decoders the reference can train (``models/__init__.py:8-10``:
FPN, DeepLabV3/V3+, Linknet, PSPNet, Unet++ ...): bilinear resizing (``F.interpolate`` /
``nn.UpsamplingBilinear2d``), ``nn.GroupNorm(+ReLU)`` (FPN), ``nn.AdaptiveAvgPool2d`` (PSPNet bins,
ASPP / PAN global pooling) and depthwise convolution (DeepLabV3+ ``SeparableConv2d``).  Every backward
is a deterministic gather / fixed-order reduction.  Each op has a plain-torch fp32 oracle for the tests.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._ext import require


def _scale(i, o, align, sf=None):
    """PyTorch's bilinear source scale (aten area_pixel_compute_scale)."""
    if align:
        return (i - 1) / (o - 1) if o > 1 else 0.0
    return 1.0 / sf if sf else i / o


class _Resize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, OH, OW, align, sh, sw, out):
        C = require()
        x = x.contiguous()
        N, H, W, Cp = x.shape
        accum = out is not None
        y = out if accum else torch.empty(N, OH, OW, Cp, dtype=x.dtype, device=x.device)
        C.resize_bilinear(x, y, sh, sw, align, accum=accum)
        ctx.geo = (H, W, align, sh, sw)
        ctx.accum = accum
        if accum:
            ctx.mark_dirty(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = require()
        H, W, align, sh, sw = ctx.geo
        dy = dy.contiguous()
        dx = torch.empty(dy.shape[0], H, W, dy.shape[3], dtype=dy.dtype, device=dy.device)
        C.resize_bilinear(dy, dx, sh, sw, align, backward=True)
        return dx, None, None, None, None, None, (dy if ctx.accum else None)


def resize_bilinear(x, size=None, scale_factor=None, align_corners=False, out=None):
    """``F.interpolate(x, size|scale_factor, mode='bilinear', align_corners)`` on an NHWC bf16 map;
    ``out``: accumulate into this [N, OH, OW, Cp] tensor (``out += up(x)``, in place)."""
    N, H, W, Cp = x.shape
    if size is None:
        OH, OW = int(H * scale_factor), int(W * scale_factor)
    else:
        OH, OW = size
    sf = scale_factor if size is None else None
    sh, sw = _scale(H, OH, align_corners, sf), _scale(W, OW, align_corners, sf)
    return _Resize.apply(x, OH, OW, bool(align_corners), float(sh), float(sw), out)


def resize_bilinear_reference(x, size=None, scale_factor=None, align_corners=False):
    y = F.interpolate(x.permute(0, 3, 1, 2).float(), size=size, scale_factor=scale_factor, mode='bilinear',
                      align_corners=align_corners)
    return y.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


# ------------------------------------------------------------------------------------------------ GroupNorm
class _GroupNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, G, C, eps, relu, gamma, beta):
        Cx = require()
        x = x.contiguous()
        N, H, W, Cp = x.shape
        HW = H * W
        nblk = Cx.nc_sums_blocks(HW, Cp)
        part = torch.empty(N, nblk, 2, Cp, dtype=torch.float32, device=x.device)
        Cx.nc_sums(x, None, None, False, part)
        tab = torch.empty(N, 4, Cp, dtype=torch.float32, device=x.device)
        Cx.gn_finalize(part, C, G, eps, gamma.detach().float().contiguous() if gamma is not None else None,
                       beta.detach().float().contiguous() if beta is not None else None, HW, tab)
        z = torch.empty_like(x)
        Cx.affine_nc(x, tab, 4, z, relu)
        ctx.save_for_backward(x, tab, gamma)
        ctx.cfg = (G, C, relu, gamma is not None, beta is not None)
        return z

    @staticmethod
    def backward(ctx, dz):
        Cx = require()
        x, tab, gamma = ctx.saved_tensors
        G, C, relu, has_g, has_b = ctx.cfg
        dz = dz.contiguous()
        N, H, W, Cp = x.shape
        HW = H * W
        nblk = Cx.nc_sums_blocks(HW, Cp)
        part = torch.empty(N, nblk, 2, Cp, dtype=torch.float32, device=x.device)
        Cx.nc_sums(x, dz, tab, relu, part)
        dgamma = torch.zeros(C, dtype=torch.float32, device=x.device) if has_g else None
        dbeta = torch.zeros(C, dtype=torch.float32, device=x.device) if has_b else None
        coef = torch.empty(N, 3, Cp, dtype=torch.float32, device=x.device)
        Cx.gn_bwd_finalize(part, C, G, gamma.detach().float().contiguous() if has_g else None, tab, HW, dgamma,
                           dbeta, coef)
        dx = torch.empty_like(x)
        Cx.affine_nc_bwd(dz, x, tab, coef, dx, relu)
        return dx, None, None, None, None, dgamma, dbeta


def group_norm_act(x, gn: torch.nn.GroupNorm, relu=True):
    """``act(GroupNorm(x))`` (nn.GroupNorm semantics: biased variance over (H, W, C/G) per image and group)
    on an NHWC bf16 map with ``gn.num_channels`` real channels; returns a materialised NHWC bf16 map."""
    assert gn.num_channels % gn.num_groups == 0
    return _GroupNormAct.apply(x, gn.num_groups, gn.num_channels, float(gn.eps), bool(relu), gn.weight, gn.bias)


def group_norm_act_reference(x, gn, relu=True):
    C = gn.num_channels
    y = F.group_norm(x[..., :C].permute(0, 3, 1, 2).float(), gn.num_groups, gn.weight, gn.bias, gn.eps)
    if relu:
        y = torch.relu(y)
    out = torch.zeros_like(x)
    out[..., :C] = y.permute(0, 2, 3, 1).to(torch.bfloat16)
    return out


# ------------------------------------------------------------------------------------------------ pooling
class _AdaptiveAvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, OH, OW):
        C = require()
        x = x.contiguous()
        N, H, W, Cp = x.shape
        y = torch.empty(N, OH, OW, Cp, dtype=x.dtype, device=x.device)
        C.adaptive_avgpool(x, y)
        ctx.hw = (H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = require()
        dy = dy.contiguous()
        H, W = ctx.hw
        dx = torch.empty(dy.shape[0], H, W, dy.shape[3], dtype=dy.dtype, device=dy.device)
        C.adaptive_avgpool(dy, dx, backward=True)
        return dx, None, None


def adaptive_avgpool(x, out_hw):
    oh, ow = (out_hw, out_hw) if isinstance(out_hw, int) else out_hw
    return _AdaptiveAvgPool.apply(x, int(oh), int(ow))


def adaptive_avgpool_reference(x, out_hw):
    y = F.adaptive_avg_pool2d(x.permute(0, 3, 1, 2).float(), out_hw)
    return y.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


# ------------------------------------------------------------------------------------------------ depthwise
def _taps(kh, kw, padding, dilation):
    ph, pw = padding
    dh, dw = dilation
    return [r * dh - ph for r in range(kh) for c in range(kw)], [c * dw - pw for r in range(kh) for c in range(kw)]


class _DwConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, kh, kw, padding, dilation):
        Cx = require()
        x = x.contiguous()
        N, H, W, Cp = x.shape
        C = weight.shape[0]
        T = kh * kw
        wt = torch.zeros(T, Cp, dtype=torch.float32, device=x.device)
        wt[:, :C] = weight.detach().float().reshape(C, T).t()
        bt = None
        if bias is not None:
            bt = torch.zeros(Cp, dtype=torch.float32, device=x.device)
            bt[:C] = bias.detach().float()
        dy, dx = _taps(kh, kw, padding, dilation)
        y = torch.empty_like(x)
        Cx.dwconv_fwd(x, wt, bt, y, dy, dx)
        ctx.save_for_backward(x, wt)
        ctx.cfg = (C, kh, kw, dy, dx, bias is not None)
        return y

    @staticmethod
    def backward(ctx, g):
        Cx = require()
        x, wt = ctx.saved_tensors
        C, kh, kw, dy, dx, has_b = ctx.cfg
        g = g.contiguous()
        N, H, W, Cp = x.shape
        T = kh * kw
        gx = torch.empty_like(x)
        Cx.dwconv_fwd(g, wt, None, gx, [-v for v in dy], [-v for v in dx])   # dX[p] = sum_t w_t dY[p - off_t]
        nblk = Cx.dwconv_wgrad_blocks(N * H * W, Cp)
        part = torch.empty(nblk, T + 1, Cp, dtype=torch.float32, device=x.device)
        Cx.dwconv_wgrad(x, g, part, dy, dx)
        red = torch.empty(T + 1, Cp, dtype=torch.float32, device=x.device)
        Cx.colsum(part, red, False)
        gw = red[:T, :C].t().reshape(C, 1, kh, kw).contiguous()
        gb = red[T, :C].contiguous() if has_b else None
        return gx, gw, gb, None, None, None, None


def dwconv(x, conv: torch.nn.Conv2d):
    """Depthwise ``conv`` (groups == in == out channels, stride 1) on an NHWC bf16 map."""
    kh, kw = conv.kernel_size
    assert conv.groups == conv.in_channels == conv.out_channels and tuple(conv.stride) == (1, 1)
    # the kernel writes a 'same'-sized map (y = empty_like(x)): any other padding would be silently
    # shifted / cropped, so it is refused here
    (ph, pw), (dh, dw) = tuple(conv.padding), tuple(conv.dilation)
    if 2 * ph != dh * (kh - 1) or 2 * pw != dw * (kw - 1):
        raise ValueError(f'dwconv: only same-size depthwise convs are fused (kernel {kh}x{kw}, padding '
                         f'{(ph, pw)}, dilation {(dh, dw)})')
    C = conv.in_channels
    if conv.bias is None and (kh, kw) == (3, 3) and x.shape[-1] == C and C % 16 == 0:
        # unpadded 3x3 without bias (smp SeparableConv2d's depthwise): the MFMA grouped-conv kernels
        # (ops/gconv.py, CG = 1; any dilation) -- forward, data- and weight-gradient
        from .gconv import gconv
        return gconv(x, conv)
    return _DwConv.apply(x, conv.weight, conv.bias, kh, kw, tuple(conv.padding), tuple(conv.dilation))


def dwconv_reference(x, conv):
    C = conv.out_channels
    y = F.conv2d(x[..., :C].permute(0, 3, 1, 2).float(), conv.weight.float(),
                 conv.bias.float() if conv.bias is not None else None, conv.stride, conv.padding, conv.dilation,
                 conv.groups)
    out = torch.zeros_like(x)
    out[..., :C] = y.permute(0, 2, 3, 1).to(torch.bfloat16)
    return out
