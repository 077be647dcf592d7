"""Fused loss kernels (``csrc/loss.hip``) as autograd Functions over NCHW fp32 logits.

* :func:`cross_entropy` == ``nn.CrossEntropyLoss(weight, ignore_index, reduction='mean')``
  (reference ``core/loss.py:30-31``): one kernel computes the loss partials and d(loss)/d(logits);
  backward is a scalar rescale, no second pass over the logits.
* :func:`ohem_cross_entropy` == reference ``OhemCELoss`` (``core/loss.py:6-20``): the per-pixel
  losses come from the same fused kernel; the selection (threshold, exact top-k fallback by radix
  select) runs in device kernels with no host sync, so OHEM steps are graph-captured too.
* :func:`kd_kl_div` == ``F.kl_div(log_softmax(s/T), softmax(t/T)) * T**2`` with the default
  elementwise-mean reduction (reference ``core/loss.py:42-46``).
* :func:`kd_mse` == ``F.mse_loss(s, t)`` (reference ``core/loss.py:47-48``), one fused pass.
* :func:`bce_dice` == ``bw * BCEWithLogits + dw * (1 - mean_n soft-Dice_n)`` for binary heads
  (``num_class == 1``): a per-sample reduction kernel in forward, the gradient
  kernel in backward (it needs the sample's Dice sums), upstream gradient read on the device.
"""
from __future__ import annotations

import math

import torch

from ._ext import require


class _CE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, weight, ignore_index):
        C = require()
        logits = logits.contiguous().float()
        target = target.contiguous().long()
        n, c, h, w = logits.shape
        grad = torch.empty_like(logits)
        part = torch.empty(C.ce_blocks(n * h * w), 2, dtype=torch.float32, device=logits.device)
        C.ce_fwd_bwd(logits, target, weight, grad, None, part, ignore_index)
        tot = part.sum(0)
        ctx.save_for_backward(grad, tot)
        return tot[0] / tot[1]

    @staticmethod
    def backward(ctx, g):
        grad, tot = ctx.saved_tensors
        return grad * (g / tot[1]), None, None, None


def cross_entropy(logits, target, weight=None, ignore_index=255):
    if weight is not None:
        weight = weight.to(device=logits.device, dtype=torch.float32).contiguous()
    return _CE.apply(logits, target, weight, ignore_index)


class _OHEM(torch.autograd.Function):
    """Per-pixel CE from the fused kernel; hard-pixel selection (threshold, else exact top-k) entirely on
    the device (``loss.hip`` ohem_*): no host synchronisation, so the step stays graph-capturable.

    Two documented differences from the reference ``OhemCELoss`` (``core/loss.py:6-20``):
      * no valid pixel at all (n_min = 0) and none above the threshold: the loss is 0 here, the
        reference's ``torch.mean`` of an empty tensor is NaN;
      * pixels tied at the k-th largest loss in the top-k fallback each get the fractional weight
        (n_min - #greater) / #tied, where ``torch.topk`` gives the full 1/n_min to an arbitrary subset of
        them: the loss VALUE is identical, the per-pixel gradients differ on the tied pixels only.
        Tests that compare gradients bit-for-bit use tie-free inputs."""

    @staticmethod
    def forward(ctx, logits, target, thresh, ignore_index):
        C = require()
        logits = logits.contiguous().float()
        target = target.contiguous().long()
        n, c, h, w = logits.shape
        dev = logits.device
        grad = torch.empty_like(logits)
        P = n * h * w
        pix = torch.empty(P, dtype=torch.float32, device=dev)
        nb = C.ce_blocks(P)
        part = torch.empty(nb, 2, dtype=torch.float32, device=dev)
        C.ce_fwd_bwd(logits, target, None, grad, pix, part, ignore_index)
        bpart = torch.empty(nb, 3, dtype=torch.float32, device=dev)
        state = torch.empty(C.ohem_state_words(), dtype=torch.int32, device=dev)
        hist = torch.empty(256, dtype=torch.int32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        C.ohem_select(pix, target, thresh, ignore_index, bpart, state, hist, loss)
        ctx.save_for_backward(grad, pix, state)
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        grad, pix, state = ctx.saved_tensors
        out = grad.clone()
        require().ohem_backward(out, pix, state, g.reshape(1).float().contiguous())
        return out, None, None, None


def ohem_cross_entropy(logits, target, thresh=0.7, ignore_index=255):
    return _OHEM.apply(logits, target, -math.log(thresh), ignore_index)


class _KDKL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, t, T):
        C = require()
        s = s.contiguous().float()
        t = t.detach().contiguous().float()
        grad = torch.empty_like(s)
        n, c, h, w = s.shape
        part = torch.empty(C.ce_blocks(n * h * w), dtype=torch.float32, device=s.device)
        C.kd_kl_fwd_bwd(s, t, grad, part, T)
        ctx.save_for_backward(grad)
        return part.sum() * (T * T) / s.numel()

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g, None, None


def kd_kl_div(student, teacher, T=4.0):
    return _KDKL.apply(student, teacher, float(T))


class _MSE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, t):
        C = require()
        s = s.contiguous().float()
        t = t.detach().contiguous().float()
        grad = torch.empty_like(s)
        part = torch.empty(C.ce_blocks(s.numel()), dtype=torch.float32, device=s.device)
        C.mse_fwd_bwd(s, t, grad, part)
        ctx.save_for_backward(grad)
        return part.sum() / s.numel()

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g, None


def kd_mse(student, teacher):
    return _MSE.apply(student, teacher)


class _BCEDice(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, bw, dw, smooth):
        C = require()
        x = logits.contiguous().float()
        t = target.contiguous().float().view_as(x)
        n = x.shape[0]
        hw = x.numel() // n
        part = torch.empty(n, C.bce_dice_splits(hw), 4, dtype=torch.float32, device=x.device)
        C.bce_dice_stats(x, t, part)
        sums = part.sum(1)                                    # [N, 4]: BCE, p*t, p, t
        den = sums[:, 2] + sums[:, 3] + smooth
        num = 2 * sums[:, 1] + smooth
        loss = bw * sums[:, 0].sum() / x.numel() + dw * (1 - (num / den).mean())
        ctx.save_for_backward(x, t, torch.stack([den, num], 1).contiguous())
        ctx.bw, ctx.dw = bw, dw
        return loss

    @staticmethod
    def backward(ctx, g):
        C = require()
        x, t, coef = ctx.saved_tensors
        grad = torch.empty_like(x)
        C.bce_dice_grad(x, t, coef, g.detach().float().reshape(1).contiguous(), grad, ctx.bw, ctx.dw)
        return grad, None, None, None, None


def bce_dice(logits, target, bce_weight=1.0, dice_weight=1.0, smooth=1.0):
    return _BCEDice.apply(logits, target, float(bce_weight), float(dice_weight), float(smooth))
