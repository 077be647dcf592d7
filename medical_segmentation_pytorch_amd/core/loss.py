"""Losses -- reference ``core/loss.py:6-49``.

On a ROCm device with the HIP extension the CE / OHEM / KD-KL losses run the fused single-pass
kernels of ``csrc/loss.hip`` (loss + gradient in one pass); elsewhere plain PyTorch with identical
semantics.  Added (north star): ``'bce_dice'`` for ``num_class == 1``.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import _ext


def _fused_ok(t):
    return t.is_cuda and t.dim() == 4 and _ext.available()


class CrossEntropyLoss(nn.Module):
    def __init__(self, ignore_index=255, reduction='mean', weight=None):
        super().__init__()
        self.ignore_index, self.reduction = ignore_index, reduction
        self.register_buffer('weight', weight if weight is None else weight.float())

    def forward(self, logits, labels):
        if self.reduction == 'mean' and _fused_ok(logits):
            from ..ops.losses import cross_entropy
            return cross_entropy(logits.float(), labels, self.weight, self.ignore_index)
        return F.cross_entropy(logits.float(), labels, weight=self.weight, ignore_index=self.ignore_index,
                               reduction=self.reduction)


class OhemCELoss(nn.Module):
    """Online hard example mining CE (reference core/loss.py:6-20), device-agnostic threshold."""

    def __init__(self, thresh, ignore_index=255):
        super().__init__()
        self.thresh = -math.log(thresh)
        self.ignore_index = ignore_index

    def forward(self, logits, labels):
        if _fused_ok(logits):
            from ..ops.losses import ohem_cross_entropy
            return ohem_cross_entropy(logits.float(), labels, math.exp(-self.thresh), self.ignore_index)
        n_min = labels[labels != self.ignore_index].numel() // 16
        loss = F.cross_entropy(logits.float(), labels, ignore_index=self.ignore_index, reduction='none').view(-1)
        loss_hard = loss[loss > self.thresh]
        if loss_hard.numel() < n_min:
            loss_hard, _ = loss.topk(n_min)
        return torch.mean(loss_hard)


class BceDiceLoss(nn.Module):
    """Binary (num_class == 1) loss: BCE-with-logits + soft Dice on the sigmoid."""

    def __init__(self, bce_weight=1.0, dice_weight=1.0, smooth=1.0):
        super().__init__()
        self.bw, self.dw, self.smooth = bce_weight, dice_weight, smooth

    def forward(self, logits, labels):
        logits = logits.float()
        target = labels.float().view_as(logits) if labels.dim() == logits.dim() else labels.float().unsqueeze(1)
        if _fused_ok(logits):
            from ..ops.losses import bce_dice
            return bce_dice(logits, target, self.bw, self.dw, self.smooth)
        bce = F.binary_cross_entropy_with_logits(logits, target)
        p = torch.sigmoid(logits)
        inter = (p * target).flatten(1).sum(1)
        den = p.flatten(1).sum(1) + target.flatten(1).sum(1)
        dice = 1 - ((2 * inter + self.smooth) / (den + self.smooth)).mean()
        return self.bw * bce + self.dw * dice


def get_loss_fn(config, device):
    weights = None if config.class_weights is None else torch.tensor(config.class_weights, dtype=torch.float32,
                                                                      device=device)
    if config.loss_type == 'ce':
        return CrossEntropyLoss(ignore_index=config.ignore_index, reduction=config.reduction, weight=weights)
    if config.loss_type == 'ohem':
        return OhemCELoss(thresh=config.ohem_thrs, ignore_index=config.ignore_index)
    if config.loss_type in ('bce_dice', 'bce', 'dice'):
        bw = 0.0 if config.loss_type == 'dice' else 1.0
        dw = 0.0 if config.loss_type == 'bce' else 1.0
        return BceDiceLoss(bw, dw)
    raise NotImplementedError(f'Unsupport loss type: {config.loss_type}')


def kd_loss_fn(config, outputs, outputsT):
    if config.kd_loss_type == 'kl_div':
        if _fused_ok(outputs):
            from ..ops.losses import kd_kl_div
            return kd_kl_div(outputs.float(), outputsT.detach().float(), config.kd_temperature)
        T = config.kd_temperature
        return F.kl_div(F.log_softmax(outputs / T, dim=1), F.softmax(outputsT.detach() / T, dim=1),
                        reduction='mean') * T ** 2
    if config.kd_loss_type == 'mse':
        if _fused_ok(outputs):
            from ..ops.losses import kd_mse
            return kd_mse(outputs.float(), outputsT.detach().float())
        return F.mse_loss(outputs, outputsT.detach())
    raise NotImplementedError(f'Unsupport kd loss type: {config.kd_loss_type}')
