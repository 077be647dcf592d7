"""Layout conversion and glue ops on the HIP kernels (``csrc/elementwise.hip``)."""
from __future__ import annotations

import os

import torch

from ._ext import require
from .fm import cpad


class _ToFM(torch.autograd.Function):
    """NCHW fp32 -> NHWC bf16 padded (model input boundary)."""

    @staticmethod
    def forward(ctx, x):
        C = require()
        x = x.contiguous().float()
        n, c, h, w = x.shape
        y = torch.empty(n, h, w, cpad(c), dtype=torch.bfloat16, device=x.device)
        C.nchw_to_nhwc(x, y, cpad(c))
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, g):
        C = require()
        n, c, h, w = ctx.shape
        out = torch.empty(n, c, h, w, dtype=torch.float32, device=g.device)
        C.nhwc_to_nchw(g.contiguous(), out, cpad(c))
        return out


class _FromFM(torch.autograd.Function):
    """NHWC bf16 padded -> NCHW fp32 with ``c`` logical channels (logits boundary)."""

    @staticmethod
    def forward(ctx, fm, c):
        C = require()
        fm = fm.contiguous()
        n, h, w, cp = fm.shape
        out = torch.empty(n, c, h, w, dtype=torch.float32, device=fm.device)
        C.nhwc_to_nchw(fm, out, cp)
        ctx.cp = cp
        return out

    @staticmethod
    def backward(ctx, g):
        C = require()
        g = g.contiguous().float()
        n, c, h, w = g.shape
        out = torch.empty(n, h, w, ctx.cp, dtype=torch.bfloat16, device=g.device)
        C.nchw_to_nhwc(g, out, ctx.cp)
        return out, None


class _Up2Add(torch.autograd.Function):
    """nearest-2x(low) + skip  (reference models/ducknet.py:82-84); pro = deferred-BN prologues."""

    @staticmethod
    def forward(ctx, pro, park, low, skip):
        C = require()
        low, skip = low.contiguous(), skip.contiguous()
        n, h, w, cp = low.shape
        assert skip.shape == (n, 2 * h, 2 * w, cp), (low.shape, skip.shape)
        out = torch.empty_like(skip)
        C.up2_add(low, skip, out, n, h, w, cp, pro[0], pro[1])
        ctx.shape = (n, h, w, cp)
        ctx.skip_ref = skip if park else None
        return out

    @staticmethod
    def backward(ctx, g):
        from .bn import need_grads
        C = require()
        need_grads([g])
        n, h, w, cp = ctx.shape
        g = g.contiguous()
        dlow = torch.empty(n, h, w, cp, dtype=torch.bfloat16, device=g.device)
        C.pool2_sum(g, dlow, n, h, w, cp)
        if ctx.skip_ref is not None and ctx.needs_input_grad[3]:
            # the skip's other reader (the encoder's downsample conv) adds its data-gradient to g in its
            # epilogue (ops.conv.park_input_grad) -- no autograd bf16 add of the two contributions
            from .conv import park_input_grad
            park_input_grad(ctx.skip_ref, g)
            ctx.skip_ref = None
            return None, None, dlow, None
        return None, None, dlow, g


class _AddN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pro, *xs):
        C = require()
        xs = [x.contiguous() for x in xs]
        out = torch.empty_like(xs[0])
        C.add_n(xs, out, pro[0], pro[1])
        ctx.k = len(xs)
        return out

    @staticmethod
    def backward(ctx, g):
        return (None,) + (g,) * ctx.k


def to_fm(x):
    return _ToFM.apply(x)


def from_fm(fm, c):
    return _FromFM.apply(fm, c)


def up2_add(low, skip, park_skip=False):
    """``low``/``skip``: tensors or ``ops.bn.Deferred`` (normalise+ReLU applied while loading).
    ``park_skip``: the caller guarantees that exactly one other reader of ``skip`` exists, one of our
    convs, whose backward runs after this op's: dL/dskip is parked for it instead of returned."""
    from .bn import Deferred, split_inputs
    # a skip already materialised (its other reader took the normalise pass) is read as that tensor: one
    # read either way, and a parked gradient is keyed by the tensor the other reader saw
    skip = skip.z if isinstance(skip, Deferred) and skip.z is not None else skip
    (lt, st), coefs, mask = split_inputs([low, skip])
    return _Up2Add.apply((coefs, mask), bool(park_skip), lt, st)


def add_n(*xs):
    """Elementwise sum of tensors / ``ops.bn.Deferred`` BN outputs (always a plain tensor)."""
    from .bn import materialize, split_inputs
    if len(xs) == 1:
        return materialize(xs[0])
    ts, coefs, mask = split_inputs(xs)
    return _AddN.apply((coefs, mask), *ts)


_BN_RELU6 = os.environ.get('MSP_BN_RELU6', '1') != '0'


class _ReLU6(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        C = require()
        x = x.contiguous()
        y = torch.empty_like(x)
        C.relu6(x, y)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        C = require()
        (y,) = ctx.saved_tensors
        dx = torch.empty_like(y)
        C.relu6_bwd(g.contiguous(), y, dx)
        return dx


class _BNReLU6(torch.autograd.Function):
    """relu6(materialize(d)) for a deferred BN output without ReLU in ONE pass (``bn_act_apply_relu6``: the
    affine and the clamp before the single bf16 rounding -- bitwise the two-pass result); backward: the
    ReLU6 mask of the output, passed to the deferred alias like ``ops.bn._Materialize``."""

    @staticmethod
    def forward(ctx, t, stats):
        C = require()
        t = t.contiguous()
        Cp = t.shape[-1]
        y = torch.empty_like(t)
        C.bn_act_apply_relu6(t, stats, y, t.numel() // Cp, Cp)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        C = require()
        (y,) = ctx.saved_tensors
        dx = torch.empty_like(y)
        C.relu6_bwd(g.contiguous(), y, dx)
        return dx, None


def relu6(x):
    """``nn.ReLU6`` (MobileNetV2) on an NHWC bf16 map; a ``ops.bn.Deferred`` input (BN without ReLU, not yet
    materialised) takes the one-pass BN + ReLU6 apply (env MSP_BN_RELU6=0: materialise, then ReLU6)."""
    from .bn import Deferred, materialize, need_stats
    if _BN_RELU6 and isinstance(x, Deferred) and x.z is None and not x.relu:
        need_stats([x])
        return _BNReLU6.apply(x.t, x.stats)
    return _ReLU6.apply(materialize(x))
