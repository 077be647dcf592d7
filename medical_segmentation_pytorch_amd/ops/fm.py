"""Feature-map conventions of the fused engine.

Activations are NHWC bf16 tensors ``[N, H, W, Cp]`` with ``Cp = cpad(C)`` (a multiple of 8, so one
16-byte vector = 8 channels of one pixel).  Padded channels always hold zeros.
"""
from __future__ import annotations

import torch


def cpad(c: int) -> int:
    return (int(c) + 7) // 8 * 8


def round_up(x: int, m: int) -> int:
    return (int(x) + m - 1) // m * m


def new_fm(n, h, w, c, device, zero=False):
    shape = (n, h, w, cpad(c))
    if zero:
        return torch.zeros(shape, dtype=torch.bfloat16, device=device)
    return torch.empty(shape, dtype=torch.bfloat16, device=device)


def to_fm_reference(x_nchw: torch.Tensor) -> torch.Tensor:
    """Plain-torch NCHW -> padded NHWC bf16 (what the ``nchw_to_nhwc`` kernel computes)."""
    n, c, h, w = x_nchw.shape
    out = torch.zeros(n, h, w, cpad(c), dtype=torch.bfloat16, device=x_nchw.device)
    out[..., :c] = x_nchw.permute(0, 2, 3, 1).to(torch.bfloat16)
    return out


def from_fm_reference(fm: torch.Tensor, c: int) -> torch.Tensor:
    return fm[..., :c].permute(0, 3, 1, 2).float().contiguous()
