"""Inference glue on the HIP kernels (``csrc/metrics.hip``): bilinear resize of fp32 NCHW tensors
(validation's ``val_img_stride`` resize and the logits resize back, reference
``core/seg_trainer.py:103-116``) and argmax -> colormap for ``predict`` (``core/seg_trainer.py:162``).
On CPU (or without the extension) both fall back to the equivalent torch ops."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext


def _native(t):
    return t.is_cuda and _ext.available()


def resize_bilinear(x, size, align_corners=False):
    """``F.interpolate(x, size, mode='bilinear', align_corners=align_corners)``."""
    oh, ow = int(size[0]), int(size[1])
    if not _native(x):
        return F.interpolate(x, (oh, ow), mode='bilinear', align_corners=align_corners)
    x = x.contiguous().float()
    y = torch.empty(x.shape[0], x.shape[1], oh, ow, dtype=torch.float32, device=x.device)
    _ext.require().bilinear_resize(x, y, bool(align_corners))
    return y


def colorize(logits, lut):
    """logits [N, C, H, W] -> uint8 [N, H, W, 3]: ``lut[argmax]`` (C == 1: ``lut[logit > 0]``)."""
    if not _native(logits):
        idx = (logits[:, 0] > 0).long() if logits.shape[1] == 1 else logits.argmax(1)
        return lut[idx]
    n, c, h, w = logits.shape
    out = torch.empty(n, h, w, 3, dtype=torch.uint8, device=logits.device)
    _ext.require().colorize(logits.contiguous().float(), lut.to(torch.uint8).contiguous(), out)
    return out
