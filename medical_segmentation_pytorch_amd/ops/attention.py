"""MAnet position attention (PAB) products on the HIP kernels of ``csrc/attention.hip``.

Reference: the smp MAnet decoder of the reference hub (``models/__init__.py:8-10``):
``sp = softmax((center @ top^T).view(b, -1)).view(b, hw, hw) @ bottom`` -- the softmax runs over each image's
WHOLE flattened hw x hw map.  Here the two products and the three of the backward are one batched MFMA
kernel (bf16 operands, fp32 accumulation) and the whole-map softmax / its backward are one block per image
(fp32 statistics, bf16 probabilities: the reference's autocast matmul operands are half precision too).
"""
from __future__ import annotations

import torch

from ._ext import require


def _gemm(C, a, b, out, batch, M, N, K, lda, ldb, ldc, ta, tb):
    C.batched_gemm(a, b, out, batch, M, N, K, lda, ldb, ldc, a.stride(0), b.stride(0), out.stride(0), ta, tb)


class _PabAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, center, top, bottom):
        C = require()
        center, top, bottom = center.contiguous(), top.contiguous(), bottom.contiguous()
        b, hw, p = center.shape
        c = bottom.shape[2]
        dev = center.device
        s = torch.empty(b, hw, hw, dtype=torch.float32, device=dev)
        _gemm(C, center, top, s, b, hw, hw, p, p, p, hw, False, True)            # center . top^T
        prob = torch.empty(b, hw, hw, dtype=torch.bfloat16, device=dev)
        C.softmax_all(s, prob, b, hw * hw)
        out = torch.empty(b, hw, c, dtype=torch.bfloat16, device=dev)
        _gemm(C, prob, bottom, out, b, hw, c, hw, hw, c, c, False, False)        # P . bottom
        ctx.save_for_backward(center, top, bottom, prob)
        return out

    @staticmethod
    def backward(ctx, dout):
        C = require()
        center, top, bottom, prob = ctx.saved_tensors
        dout = dout.to(torch.bfloat16).contiguous()
        b, hw, p = center.shape
        c = bottom.shape[2]
        dev = center.device
        dprob = torch.empty(b, hw, hw, dtype=torch.float32, device=dev)
        _gemm(C, dout, bottom, dprob, b, hw, hw, c, c, c, hw, False, True)      # dout . bottom^T
        dbottom = torch.empty(b, hw, c, dtype=torch.bfloat16, device=dev)
        _gemm(C, prob, dout, dbottom, b, hw, c, hw, hw, c, c, True, False)      # P^T . dout
        ds = torch.empty(b, hw, hw, dtype=torch.bfloat16, device=dev)
        C.softmax_all_bwd(prob, dprob, ds, b, hw * hw)
        dcenter = torch.empty(b, hw, p, dtype=torch.bfloat16, device=dev)
        _gemm(C, ds, top, dcenter, b, hw, p, hw, hw, p, p, False, False)        # dS . top
        dtop = torch.empty(b, hw, p, dtype=torch.bfloat16, device=dev)
        _gemm(C, ds, center, dtop, b, hw, p, hw, hw, p, p, True, False)         # dS^T . center
        return dcenter, dtop, dbottom


def pab_attention(center: torch.Tensor, top: torch.Tensor, bottom: torch.Tensor) -> torch.Tensor:
    """[b, hw, P] x [b, hw, P] x [b, hw, C] (bf16) -> softmax_wholemap(center . top^T) . bottom, [b, hw, C] bf16."""
    return _PabAttention.apply(center, top, bottom)
