"""Pooling / decoder-merge / residual-tail ops on the HIP kernels (``csrc/pool.hip``).

* :func:`maxpool` -- ``nn.MaxPool2d(k, s, p)`` on NHWC bf16 (UNet encoder ``models/unet.py:49`` of the
  reference; the ResNet stem of the smp encoders).  The forward keeps a one-byte winning-tap index
  per element; the backward gathers (deterministic, no atomics).
* :func:`up2_cat` -- smp ``UnetDecoderBlock``: ``cat([interpolate(x, 2, 'nearest'), skip], 1)`` written
  once into a dense channel range (the following conv then sees one ordinary input).
* :func:`add_act` -- the ResNet block tail ``relu(bn(conv(x)) + identity)`` on materialised inputs;
  :func:`res_tail` -- the same from the deferred BN outputs in one pass (training).
"""
from __future__ import annotations

import torch

from ._ext import require
from .bn import materialize, need_grads
from .fm import cpad


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        C = require()
        x = x.contiguous()
        n, h, w, cp = x.shape
        oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        y = torch.empty(n, oh, ow, cp, dtype=torch.bfloat16, device=x.device)
        idx = torch.empty(n, oh, ow, cp, dtype=torch.uint8, device=x.device)
        C.maxpool_fwd(x, y, idx, k, s, p)
        ctx.save_for_backward(idx)
        ctx.cfg = (k, s, p, x.shape)
        return y

    @staticmethod
    def backward(ctx, g):
        C = require()
        need_grads([g])
        (idx,) = ctx.saved_tensors
        k, s, p, shape = ctx.cfg
        dx = torch.empty(shape, dtype=torch.bfloat16, device=g.device)
        C.maxpool_bwd(g.contiguous(), idx, dx, k, s, p)
        return dx, None, None, None


class _Up2Cat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, low, skip, cl, cs):
        C = require()
        low = low.contiguous()
        n, h, w, cpl = low.shape
        out = torch.empty(n, 2 * h, 2 * w, cpad(cl + cs), dtype=torch.bfloat16, device=low.device)
        C.up2_cat(low, skip.contiguous() if skip is not None else None, out, cl, cs)
        ctx.cfg = (low.shape, None if skip is None else skip.shape, cl, cs)
        return out

    @staticmethod
    def backward(ctx, g):
        C = require()
        need_grads([g])
        lshape, sshape, cl, cs = ctx.cfg
        g = g.contiguous()
        dlow = torch.empty(lshape, dtype=torch.bfloat16, device=g.device)
        dskip = torch.empty(sshape, dtype=torch.bfloat16, device=g.device) if sshape is not None else None
        C.up2_cat_bwd(g, dlow, dskip, cl, cs)
        return dlow, dskip, None, None


class _AddAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, relu):
        C = require()
        a, b = a.contiguous(), b.contiguous()
        z = torch.empty_like(a)
        C.add_act(a, b, z, relu)
        ctx.relu = relu
        if relu:
            ctx.save_for_backward(z)
        return z

    @staticmethod
    def backward(ctx, dz):
        need_grads([dz])
        if not ctx.relu:
            return dz, dz, None
        C = require()
        (z,) = ctx.saved_tensors
        g = torch.empty_like(z)
        C.relu_bwd(dz.contiguous(), z, g)
        return g, g, None


class _ResTail(torch.autograd.Function):
    """relu(o + r): o a deferred BN output (the block's last BN), r the identity -- a plain tensor or the
    deferred downsample BN -- in ONE pass (``bn_add_act``; no materialised o / r).  Backward: g = dz * (z > 0)
    is the gradient of both o and r (the deferred aliases take dL/d(BN output)); with ``park`` the identity's
    share is parked for conv1, which shares the block input x and adds it in its data-gradient epilogue
    (``ops.conv.park_input_grad``) instead of autograd adding two bf16 tensors."""

    @staticmethod
    def forward(ctx, a_t, a_stats, a_relu, b_t, b_stats, b_relu, park):
        C = require()
        a_t, b_t = a_t.contiguous(), b_t.contiguous()
        z = torch.empty_like(a_t)
        C.bn_add_act(a_t, a_stats, a_relu, b_t, b_stats, b_relu, z, True)
        ctx.save_for_backward(z)
        ctx.park = park and b_stats is None
        ctx.b_ref = b_t if ctx.park else None
        return z

    @staticmethod
    def backward(ctx, dz):
        need_grads([dz])
        C = require()
        (z,) = ctx.saved_tensors
        g = torch.empty_like(z)
        C.relu_bwd(dz.contiguous(), z, g)
        if ctx.park:
            from .conv import park_input_grad
            park_input_grad(ctx.b_ref, g)
            ctx.b_ref = None
            return g, None, None, None, None, None, None
        return g, None, None, g, None, None, None


def res_tail(o, idt, park_identity=False):
    """ResNet block tail ``relu(o + idt)``: fused when ``o`` is a deferred BN output (training), else the
    materialised add_act.  ``park_identity``: ``idt`` is the block input and conv1 (one of ours) reads it."""
    from .bn import Deferred, need_stats
    if not isinstance(o, Deferred):
        return add_act(materialize(o), materialize(idt), relu=True)
    need_stats([o, idt])
    if isinstance(idt, Deferred):
        return _ResTail.apply(o.t, o.stats, bool(o.relu), idt.t, idt.stats, bool(idt.relu), False)
    return _ResTail.apply(o.t, o.stats, bool(o.relu), idt, None, False, bool(park_identity))


def maxpool(x, k=3, s=2, p=1):
    return _MaxPool.apply(x, int(k), int(s), int(p))


def up2_cat(low, skip, cl, cs):
    """``low`` [N,h,w,cpad(cl)], ``skip`` [N,2h,2w,cpad(cs)] or None -> [N,2h,2w,cpad(cl+cs)]."""
    return _Up2Cat.apply(low, skip, int(cl), int(cs) if skip is not None else 0)


def add_act(a, b, relu=True):
    return _AddAct.apply(a, b, bool(relu))


# ------------------------------------------------------------------------------------------------ oracles
def maxpool_reference(x, k=3, s=2, p=1):
    import torch.nn.functional as F
    y = F.max_pool2d(x.permute(0, 3, 1, 2).float(), k, s, p)
    return y.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


def up2_cat_reference(low, skip, cl, cs):
    import torch.nn.functional as F
    up = F.interpolate(low[..., :cl].permute(0, 3, 1, 2).float(), scale_factor=2, mode='nearest')
    parts = [up] + ([skip[..., :cs].permute(0, 3, 1, 2).float()] if skip is not None else [])
    cat = torch.cat(parts, 1).permute(0, 2, 3, 1)
    n, h, w, c = cat.shape
    out = torch.zeros(n, h, w, cpad(c), dtype=torch.bfloat16, device=low.device)
    out[..., :c] = cat.to(torch.bfloat16)
    return out
