"""Segmentation metrics -- reference ``utils/metrics.py:4-13`` (torchmetrics 1.2.0 ``JaccardIndex``
(task='multiclass', ignore_index, average='none') and ``Dice`` (average='macro')), SURVEY App. C.

Both accumulate ONE ``[C, C]`` int64 confusion matrix (``confmat[target][pred]`` with the per-pixel
argmax prediction): on MI355X it is filled by the ``confmat_update`` HIP kernel (LDS histogram),
on CPU by ``torch.bincount``.  ``compute()`` all-reduces the matrix across ranks (one RCCL
all-reduce of C*C int64, instead of torchmetrics' per-state all_gathers) and derives:
  * IoU per class  = TP / (TP + FP + FN)
  * Dice (macro)   = mean over classes present of 2TP / (2TP + FP + FN)   (includes background)
Dice here ignores no index (the reference constructs ``Dice`` without ``ignore_index``), IoU drops
``ignore_index`` pixels; for {0,1} polyp masks both see the same pixels.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn


def confmat_torch(preds, target, num_classes, ignore_index=None):
    if preds.dim() == target.dim() + 1:
        pred = preds.argmax(1)
    else:
        pred = preds
    t = target.reshape(-1).long()
    p = pred.reshape(-1).long()
    valid = (t >= 0) & (t < num_classes)
    if ignore_index is not None:
        valid &= t != ignore_index
    idx = t[valid] * num_classes + p[valid]
    return torch.bincount(idx, minlength=num_classes * num_classes).view(num_classes, num_classes)


class _ConfmatMetric(nn.Module):
    def __init__(self, num_classes, ignore_index=None, sync=True, group=None):
        super().__init__()
        self.group = group
        self.num_classes = num_classes
        self.ignore_index = ignore_index
        self.sync = sync
        self.register_buffer('confmat', torch.zeros(num_classes, num_classes, dtype=torch.long))

    @torch.no_grad()
    def update(self, preds, target):
        target = target.to(self.confmat.device)
        preds = preds.to(self.confmat.device)
        if preds.is_cuda and preds.dim() == 4 and preds.dtype == torch.float32 and self.num_classes ** 2 <= 1024:
            from ..ops import _ext
            if _ext.available():
                ig = self.ignore_index if self.ignore_index is not None else -1
                _ext.require().confmat_update(preds.contiguous(), target.contiguous().long(), self.confmat, ig)
                return
        self.confmat += confmat_torch(preds, target, self.num_classes, self.ignore_index)

    def _synced(self):
        cm = self.confmat.clone()
        if self.sync and dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(cm, group=self.group)
        return cm

    def reset(self):
        self.confmat.zero_()


class JaccardIndex(_ConfmatMetric):
    def __init__(self, task='multiclass', num_classes=2, ignore_index=None, average='none', sync=True):
        assert task == 'multiclass'
        super().__init__(num_classes, ignore_index, sync)
        self.average = average

    def compute(self):
        cm = self._synced().double()
        tp = cm.diag()
        fp = cm.sum(0) - tp
        fn = cm.sum(1) - tp
        iou = tp / (tp + fp + fn).clamp_min(1e-12)
        iou = torch.where(tp + fp + fn > 0, iou, torch.zeros_like(iou))
        if self.average == 'macro':
            return iou.mean().float()
        return iou.float()


class Dice(_ConfmatMetric):
    def __init__(self, num_classes=2, average='macro', ignore_index=None, sync=True):
        super().__init__(num_classes, ignore_index, sync)
        self.average = average

    def compute(self):
        cm = self._synced().double()
        tp = cm.diag()
        fp = cm.sum(0) - tp
        fn = cm.sum(1) - tp
        den = 2 * tp + fp + fn
        present = den > 0
        dice = torch.where(present, 2 * tp / den.clamp_min(1e-12), torch.zeros_like(tp))
        if self.average == 'macro':
            return (dice[present].mean() if present.any() else dice.sum() * 0).float()
        return dice.float()


def foreground_dice(preds, target, fg=1):
    """Per-image foreground Dice averaged over images (the DUCK-Net paper's convention)."""
    pred = preds.argmax(1) if preds.dim() == target.dim() + 1 else preds
    p = (pred == fg).flatten(1).float()
    t = (target == fg).flatten(1).float()
    inter = (p * t).sum(1)
    den = p.sum(1) + t.sum(1)
    return torch.where(den > 0, 2 * inter / den.clamp_min(1e-12), torch.ones_like(den)).mean()


def get_seg_metrics(config, metric_name):
    nc = max(config.num_class, 2)          # num_class == 1 (sigmoid) is scored as background/foreground
    group = getattr(config, 'dist_group', None)
    if metric_name == 'iou':
        m = JaccardIndex(task='multiclass', num_classes=nc, ignore_index=config.ignore_index, average='none')
    elif metric_name == 'dice':
        m = Dice(num_classes=nc, average='macro')
    else:
        raise ValueError(f'Unsupported metric: {metric_name}.\n')
    m.group = group
    return m

