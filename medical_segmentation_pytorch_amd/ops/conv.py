"""Convolution on the MI355X implicit-GEMM kernels (``csrc/conv.hip``) as an autograd Function.

A :class:`ConvPlan` describes one launch: the tap table (kernel size, stride, padding, dilation),
the channel grouping of its inputs/outputs, and the list of weight *branches* it multiplies.  One
branch = one ``nn.Conv2d`` weight.  Several branches that read the same input and share the tap
grid (the DUCK block's five 3x3 first convs and three 1x1 residual shortcuts,
reference ``models/ducknet.py:144-149``) are packed into ONE GEMM whose output rows are the
branches' channels -- each branch's output lands in its own NHWC tensor (``Go`` output groups).
A 1x1 branch occupies only the centre tap of a 3x3 plan.  Inputs may be a list of tensors that
are logically channel-concatenated (``Gi`` input groups: UNet's ``torch.cat``).

Weight gradients are written into caller-provided fp32 *sinks* (views into the engine's flat grad
arena) when given, otherwise returned to autograd as usual.

Reference parity: ``nn.Conv2d`` / ``nn.ConvTranspose2d`` as used in ``models/modules.py:73-108``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from ._ext import require
from .fm import cpad, round_up


@dataclass
class Branch:
    weight: torch.Tensor            # Conv2d: [co_l, Gi*ci_l, kh_b, kw_b]; ConvTranspose2d: [ci_l, co_l, kh, kw]
    out_group: int = 0
    t_base: int = 0
    T: int = 0
    sink: Optional[torch.Tensor] = None


@dataclass
class ConvPlan:
    kh: int
    kw: int
    ci_l: int                        # logical channels per input group
    co_l: int                        # logical channels per output group
    branches: List[Branch]
    stride: int = 1
    padding: tuple = (0, 0)
    dilation: tuple = (1, 1)
    Gi: int = 1
    Go: int = 1
    transposed: bool = False
    output_padding: int = 0
    bias: Optional[torch.Tensor] = None
    bias_sink: Optional[torch.Tensor] = None
    ready_hook: Optional[object] = None     # called with the plan's params once their grads are final
    prepacked: bool = False                 # packed weights kept up to date by a PackProgram
    wp: Optional[torch.Tensor] = field(default=None, repr=False)
    wd: Optional[torch.Tensor] = field(default=None, repr=False)

    def __post_init__(self):
        self.T = self.kh * self.kw
        self.Cgi = cpad(self.ci_l)
        self.Cgo = cpad(self.co_l)
        self.Cip = self.Gi * self.Cgi
        self.rows = self.Go * self.Cgo
        self.Kp = round_up(self.T * self.Cip, 32)
        ph, pw = self.padding
        dh, dw = self.dilation
        self.taps_fwd = [(r * dh - ph, s * dw - pw) for r in range(self.kh) for s in range(self.kw)]
        self.taps_bwd = [(ph - r * dh, pw - s * dw) for r in range(self.kh) for s in range(self.kw)]
        for b in self.branches:
            if b.T == 0:
                b.T = self.T
        if self.transposed:
            assert self.Gi == 1 and self.Go == 1 and len(self.branches) == 1

    # -- geometry -------------------------------------------------------------------------------
    def out_hw(self, ih, iw):
        ph, pw = self.padding
        dh, dw = self.dilation
        s = self.stride
        if self.transposed:
            op = self.output_padding
            return ((ih - 1) * s - 2 * ph + dh * (self.kh - 1) + op + 1,
                    (iw - 1) * s - 2 * pw + dw * (self.kw - 1) + op + 1)
        return ((ih + 2 * ph - dh * (self.kh - 1) - 1) // s + 1,
                (iw + 2 * pw - dw * (self.kw - 1) - 1) // s + 1)

    def fwd_dims(self, n, ih, iw, oh, ow):
        return [n, ih, iw, self.Gi, self.Cgi, oh, ow, self.Go, self.Cgo, self.co_l, self.T, self.Kp, self.stride]

    def uses_halo(self, n, ih, iw):
        """Whether the forward of this plan on an [n, ih, iw] input runs the halo-tiled kernel."""
        cache = self.__dict__.setdefault('_halo_cache', {})
        key = (n, ih, iw)
        if key not in cache:
            oh, ow = self.out_hw(ih, iw)
            taps = self.taps_bwd if self.transposed else self.taps_fwd
            cache[key] = bool(require().conv_uses_halo(self.fwd_dims(n, ih, iw, oh, ow), [t[0] for t in taps],
                                                       [t[1] for t in taps], self.transposed and self.stride > 1))
        return cache[key]

    def uses_gemm(self, n, ih, iw):
        """Whether the forward of this plan runs the LDS-DMA GEMM kernel (no deferred-BN input prologue there)."""
        cache = self.__dict__.setdefault('_gemm_cache', {})
        key = (n, ih, iw)
        if key not in cache:
            oh, ow = self.out_hw(ih, iw)
            taps = self.taps_bwd if self.transposed else self.taps_fwd
            cache[key] = bool(require().conv_uses_gemm(self.fwd_dims(n, ih, iw, oh, ow), [t[0] for t in taps],
                                                       [t[1] for t in taps], self.transposed and self.stride > 1))
        return cache[key]

    def stat_blocks(self, n, ih, iw):
        oh, ow = self.out_hw(ih, iw)
        taps = self.taps_bwd if self.transposed else self.taps_fwd
        return require().conv_stat_blocks(self.fwd_dims(n, ih, iw, oh, ow), [t[0] for t in taps],
                                          [t[1] for t in taps], self.transposed and self.stride > 1)

    # -- weight packing ---------------------------------------------------------------------------
    # A job = (src flat view, dst flat view, nrow, nch, T, Cpk, Kp, t_base, c_base, s_row, s_ch):
    #   dst[row*Kp + (t_base + t)*Cpk + c_base + c] = bf16(src[row*s_row + c*s_ch + t])
    def fwd_jobs(self, wp):
        flat = wp.view(-1)
        if self.transposed:
            w = self.branches[0].weight.detach()             # [ci, co, kh, kw]
            return [(w.reshape(-1), flat, self.co_l, self.ci_l, self.T, self.Cip, self.Kp, 0, 0,
                     self.T, self.co_l * self.T)]
        jobs = []
        cin_tot = self.Gi * self.ci_l
        for b in self.branches:
            w = b.weight.detach().reshape(-1)
            dst = flat[b.out_group * self.Cgo * self.Kp:]
            for gi in range(self.Gi):
                jobs.append((w[gi * self.ci_l * b.T:], dst, self.co_l, self.ci_l, b.T, self.Cip, self.Kp,
                             b.t_base, gi * self.Cgi, cin_tot * b.T, b.T))
        return jobs

    def dgrad_jobs(self, wd):
        """Weights of the data-gradient conv: rows = input channels, k = (tap, output channel)."""
        flat = wd.view(-1)
        Kp_d = self.Kp_d
        if self.transposed:
            w = self.branches[0].weight.detach()             # [ci, co, kh, kw]
            return [(w.reshape(-1), flat, self.ci_l, self.co_l, self.T, self.rows, Kp_d, 0, 0,
                     self.co_l * self.T, self.T)]
        jobs = []
        cin_tot = self.Gi * self.ci_l
        for b in self.branches:
            w = b.weight.detach().reshape(-1)
            for gi in range(self.Gi):
                jobs.append((w[gi * self.ci_l * b.T:], flat[gi * self.Cgi * Kp_d:], self.ci_l, self.co_l, b.T,
                             self.rows, Kp_d, b.t_base, b.out_group * self.Cgo, b.T, cin_tot * b.T))
        return jobs

    @property
    def Kp_d(self):
        return round_up(self.T * self.rows, 32)

    def alloc_fwd(self, device):
        return torch.zeros(require().conv_rows_alloc(self.rows), self.Kp, dtype=torch.bfloat16, device=device)

    def alloc_dgrad(self, device):
        return torch.zeros(require().conv_rows_alloc(self.Gi * self.Cgi), self.Kp_d, dtype=torch.bfloat16,
                           device=device)

    def pack_fwd(self, device):
        if self.prepacked:
            return self.wp
        C = require()
        wp = self.alloc_fwd(device)
        for job in self.fwd_jobs(wp):
            C.pack_weight(*job)
        return wp

    def pack_dgrad(self, device):
        if self.prepacked:
            return self.wd, self.Kp_d
        C = require()
        wd = self.alloc_dgrad(device)
        for job in self.dgrad_jobs(wd):
            C.pack_weight(*job)
        return wd, self.Kp_d


class PackProgram:
    """All weight-packing jobs of a set of plans in ONE launch (``pack_batch``); the packed buffers
    become persistent (zero padding written once) and the plans stop packing per call."""

    def __init__(self, plans, device):
        C = require()
        rows, prefix, nblk = [], [], 0
        per = C.pack_per_block()
        self.keep = []
        for p in plans:
            p.wp = p.alloc_fwd(device)
            p.wd = p.alloc_dgrad(device)
            for src, dst, nrow, nch, T, Cpk, Kp, tb, cb, sr, sc in p.fwd_jobs(p.wp) + p.dgrad_jobs(p.wd):
                n = nrow * nch * T
                rows.append([src.data_ptr(), dst.data_ptr(), nrow, nch, T, Cpk, Kp, tb, cb, sr, sc, n])
                prefix.append(nblk)
                nblk += (n + per - 1) // per
                self.keep.append(src)
        self.jobs = torch.tensor(rows, dtype=torch.int64).to(device)
        self.prefix = torch.tensor(prefix, dtype=torch.int32).to(device)
        self.blocks = nblk
        self.plans = list(plans)
        for p in plans:
            p.prepacked = True

    def run(self):
        require().pack_batch(self.jobs, self.prefix, self.blocks)


def _taps(tl):
    return [t[0] for t in tl], [t[1] for t in tl]


# env MSP_FUSED_BWD=0: the narrow stride-1 convs run the separate data- and weight-gradient kernels (A/B)
FUSED_BWD = os.environ.get('MSP_FUSED_BWD', '1') != '0'
# A deferred BN data-gradient is NOT rebuilt by the separate halo data- and weight-gradient kernels (each
# re-reads y; measured net-neutral in round 4 and -1.6 % in round 5: profiles/r04/kernels_deferdy_*,
# profiles/r05/defer_dy_separate_ab_bs320.txt): outside the fused backward it is resolved (the apply pass).
# A module constant (no env knob): tests/test_gpu_deferred_dy.py sets it to keep that kernel path covered.
DEFER_SEPARATE = False


def _fused_bwd(ctx, plan, gys, xs, shape, need_dx, dev, dxt=None, pro=None, bn_handle=None):
    """Data- and weight-gradient of a narrow stride-1 single-group conv in ONE kernel (csrc/conv_bwd.hip):
    dY (rebuilt from a deferred BN data-gradient when one arrives) and x (through the forward's deferred-BN
    prologue) are staged once per tile; the BN epilogue of the data-gradient (BwdStatsHandle) runs in it too.
    ``dxt``: add the data-gradient into this tensor (sibling launches over one input, :class:`_MultiConvFn`);
    ``pro`` / ``bn_handle`` default to ``ctx``'s.  Returns (dxs, wgrads) or None when the shape is not eligible."""
    if not (FUSED_BWD and need_dx and not plan.transposed and plan.stride == 1 and plan.Gi == 1 and plan.Go <= 2
            and plan.bias is None and plan.Cgi <= 48 and plan.Cgo <= 48 and 2 <= plan.T <= 9
            and all(b.weight.requires_grad for b in plan.branches)):
        return None
    t1 = -1
    if plan.Go == 2:   # the ResidualBlock pair: group 0 over the full tap grid, group 1 (the 1x1) at one tap
        b0, b1 = sorted(plan.branches, key=lambda b: b.out_group)
        if len(plan.branches) != 2 or b0.t_base != 0 or b0.T != plan.T or b1.T != 1:
            return None
        t1 = b1.t_base
    C = require()
    n, ih, iw, oh, ow = shape
    dims = plan.fwd_dims(n, ih, iw, oh, ow)
    tdy, tdx = _taps(plan.taps_fwd)
    nblk = C.conv_bwd_fused_blocks(dims, tdy, tdx)
    if nblk <= 0:
        return None
    from .bn import claim_deferred, peek_deferred
    d = peek_deferred(gys[0])
    d2 = peek_deferred(gys[1]) if plan.Go == 2 else None
    coefs, rmask = ctx.pro if pro is None else pro
    xc = coefs[0] if coefs else None
    wd, Kp_d = plan.pack_dgrad(dev)
    accumulate = dxt is not None
    if not accumulate:
        dxt = torch.empty(n, ih, iw, plan.Cgi, dtype=torch.bfloat16, device=dev)
    h = ctx.bn_handle if pro is None else bn_handle
    bne = h is not None and h.y is not None
    part = torch.empty(nblk, 2, plan.Cgi, dtype=torch.float32, device=dev) if bne else None
    dwp = torch.empty(nblk * plan.rows * plan.T * plan.Cip, dtype=torch.float32, device=dev)
    C.conv_bwd_fused(d.dz if d is not None else gys[0],
                     d.y if d is not None else None, d.stats if d is not None else None,
                     d.coef if d is not None else None, bool(d.relu) if d is not None else False,
                     xs[0], xc, bool(rmask & 1), wd, Kp_d, dxt,
                     h.y if bne else None, h.stats if bne else None, bool(h.relu) if bne else False, part,
                     dwp, dims, tdy, tdx,
                     dz2=(d2.dz if d2 is not None else gys[1]) if plan.Go == 2 else None,
                     gy2=d2.y if d2 is not None else None, gs2=d2.stats if d2 is not None else None,
                     gk2=d2.coef if d2 is not None else None, grelu2=bool(d2.relu) if d2 is not None else False,
                     t1=t1, accumulate=accumulate)
    if bne:
        h.part = part
    for dd in (d, d2):
        if dd is not None:
            claim_deferred(dd)
    need = [b.weight.requires_grad for b in plan.branches]
    return [dxt], _unpack_slabs(plan, dwp, nblk, need)


def _bwd_operands(grads, plan, dims_d, taps_d, dims_w, taps_w, dgrad=True):
    """Deferred BN data-gradients among this launch's incoming gradient groups (``ops.bn.DeferredGrad``).

    Returns (gys, bwd) where ``gys`` are the tensors the kernels read (dz for a deferred group) and
    ``bwd`` = (gy, gs, gk, grelu, claims) for the kernels' BN-backward staging prologue -- or None, when
    no group is deferred or a launch of this plan cannot rebuild dY (only the non-chunked stride-1 halo
    data-gradient and the halo weight-gradient can): then every deferred group is resolved (written)
    and the launches see plain gradients, exactly as before."""
    from .bn import peek_deferred, resolve
    ds = [peek_deferred(g) for g in grads]
    if not any(d is not None for d in ds):
        return list(grads), None
    C = require()
    # Without a data-gradient launch (the first conv: its input is the image) the weight-gradient is dY's
    # only reader: rebuilding dY there reads (dz, y) once instead of the apply pass's read dz, y + write dy
    # + the weight-gradient's read dy -- 2 passes instead of 4, a win even where the halo kernels' re-read
    # of y made deferral neutral (DEFER_SEPARATE).
    ok = (DEFER_SEPARATE or not dgrad) and not plan.transposed and plan.stride == 1 and plan.bias is None
    if ok and dgrad:
        ok = bool(C.conv_uses_halo(dims_d, taps_d[0], taps_d[1], False, True))
    if ok:
        ok = bool(C.conv_wgrad_uses_halo(dims_w, taps_w[0], taps_w[1], False))
    if not ok:
        return [resolve(g) for g in grads], None
    gys, gy, gs, gk, grelu = [], [], [], [], 0
    for i, (g, d) in enumerate(zip(grads, ds)):
        if d is None:
            gys.append(g)
            gy.append(None); gs.append(None); gk.append(None)
        else:
            gys.append(d.dz)
            gy.append(d.y); gs.append(d.stats); gk.append(d.coef)
            grelu |= int(bool(d.relu)) << i
    return gys, (gy, gs, gk, grelu, [d for d in ds if d is not None])


# Identity-branch data-gradients waiting for the conv that shares their input (``ops.pool.res_tail``): a
# ResNet identity block's input x feeds conv1 and the block tail.  The tail's backward parks dL/dx of the
# identity path here (keyed by x's storage) instead of returning it; conv1's backward then accumulates its
# data-gradient into it in the GEMM / halo epilogue (``accumulate=True``) and returns the sum -- no
# autograd bf16 add of the two contributions.
_GRAD_ACC = {}


def park_input_grad(x, g):
    """``g`` is (part of) dL/dx: the next conv backward whose input is ``x`` returns its dgrad + g."""
    key = x.data_ptr()
    assert key not in _GRAD_ACC, 'one parked identity gradient per tensor'
    _GRAD_ACC[key] = (g, tuple(x.shape))


def check_parked_grads():
    """Step boundary: every parked identity gradient has been claimed (else a gradient was lost)."""
    if _GRAD_ACC:
        n = len(_GRAD_ACC)
        _GRAD_ACC.clear()
        raise RuntimeError(f'{n} parked identity gradient(s) never claimed by their conv')


def _claim_parked(xs, nx):
    if not _GRAD_ACC or nx != 1:
        return None
    ent = _GRAD_ACC.get(xs[0].data_ptr())
    if ent is None or ent[1] != tuple(xs[0].shape):
        return None
    del _GRAD_ACC[xs[0].data_ptr()]
    return ent[0]


class _ConvFn(torch.autograd.Function):
    # pro = (coefs, relu mask): deferred-BN prologue of the input groups (ops.bn.Deferred); the same
    # prologue runs again in the weight-gradient staging, so z never exists in HBM
    @staticmethod
    def forward(ctx, plan: ConvPlan, want_stats: bool, nx: int, bn_handle, pro, *args):
        C = require()
        ctx.set_materialize_grads(False)   # the stats output never gets a zero-filled gradient
        xs = [a.contiguous() for a in args[:nx]]
        coefs, rmask = pro
        n, ih, iw, _ = xs[0].shape
        oh, ow = plan.out_hw(ih, iw)
        dev = xs[0].device
        wp = plan.pack_fwd(dev)
        ys = [torch.empty(n, oh, ow, plan.Cgo, dtype=torch.bfloat16, device=dev) for _ in range(plan.Go)]
        dims = plan.fwd_dims(n, ih, iw, oh, ow)
        if plan.transposed:
            dy, dx = _taps(plan.taps_bwd)
            trans = plan.stride > 1
        else:
            dy, dx = _taps(plan.taps_fwd)
            trans = False
        part = None
        if want_stats:
            nblk = C.conv_stat_blocks(dims, dy, dx, trans)
            part = torch.empty(nblk, 2, plan.rows, dtype=torch.float32, device=dev)
        bias = plan.bias.detach().float().contiguous() if plan.bias is not None else None
        C.conv_fwd(xs, wp, ys, bias, part, dims, dy, dx, trans, coefs, rmask)
        ctx.plan = plan
        ctx.nx = nx
        ctx.pro = pro
        ctx.bn_handle = bn_handle if (bn_handle is not None and plan.stride == 1 and not plan.transposed
                                      and plan.Gi == 1) else None
        ctx.shape = (n, ih, iw, oh, ow)
        ctx.save_for_backward(*xs)
        if part is None:
            part = torch.empty(0, device=dev)
        ctx.mark_non_differentiable(part)
        return (*ys, part)

    @staticmethod
    def backward(ctx, *grads):
        from .bn import need_grads
        C = require()
        need_grads(grads)
        plan: ConvPlan = ctx.plan
        xs = list(ctx.saved_tensors)
        n, ih, iw, oh, ow = ctx.shape
        dev = xs[0].device
        gys = []
        for g in grads[:plan.Go]:
            gys.append(torch.zeros(n, oh, ow, plan.Cgo, dtype=torch.bfloat16, device=dev) if g is None
                       else g.contiguous())
        need_dx = any(ctx.needs_input_grad[5:5 + ctx.nx])
        Kp_d = plan.Kp_d
        dims_d = [n, oh, ow, plan.Go, plan.Cgo, ih, iw, plan.Gi, plan.Cgi, plan.ci_l, plan.T, Kp_d, plan.stride]
        if plan.transposed:
            dy, dx = _taps(plan.taps_fwd)
            trans = False
        else:
            dy, dx = _taps(plan.taps_bwd)
            trans = plan.stride > 1
        fused = _fused_bwd(ctx, plan, gys, xs, (n, ih, iw, oh, ow), need_dx, dev)
        if fused is not None:
            dxs, wgrads = fused
            parked = _claim_parked(xs, ctx.nx) if need_dx else None
            if parked is not None and dxs[0] is not None:
                dxs[0].add_(parked)
            ctx.bn_handle = None
            if plan.ready_hook is not None:
                plan.ready_hook([b.weight for b in plan.branches])
            return tuple([None, None, None, None, None] + dxs + wgrads)
        # deferred BN data-gradients: rebuilt in the staging of both launches below, or resolved here
        gys, bwd = _bwd_operands(gys, plan, dims_d, (dy, dx), plan.fwd_dims(n, ih, iw, oh, ow),
                                 _taps(plan.taps_fwd), dgrad=need_dx)
        bk = {} if bwd is None else dict(gy=bwd[0], gs=bwd[1], gk=bwd[2], grelu=bwd[3])
        dxs = [None] * ctx.nx
        parked = _claim_parked(xs, ctx.nx) if need_dx else None
        # (the parked tensor may also be this conv's own output gradient: then the sum goes to a fresh tensor)
        in_place = parked is not None and all(g.data_ptr() != parked.data_ptr() for g in gys)
        if need_dx:
            wd, Kp_d = plan.pack_dgrad(dev)
            dxs = [torch.empty(n, ih, iw, plan.Cgi, dtype=torch.bfloat16, device=dev) for _ in range(plan.Gi)]
            h = ctx.bn_handle
            if in_place and plan.Gi == 1 and (h is None or h.y is None):
                # dL/dx = this dgrad + the parked gradient of x's other reader, summed in the epilogue (a
                # strided data-gradient too: every phase launch adds into its own output pixels)
                C.conv_fwd(gys, wd, [parked], None, None, dims_d, dy, dx, trans, accumulate=True, **bk)
                dxs, parked = [parked], None
            elif h is not None and h.y is not None and not trans:
                # dL/dx is the BN output's gradient: emit the BN backward partials in the epilogue
                nblk = C.conv_stat_blocks(dims_d, dy, dx, False, bwd is not None, True)
                part = torch.empty(nblk, 2, plan.Gi * plan.Cgi, dtype=torch.float32, device=dev)
                C.conv_fwd_bn(gys, wd, dxs, part, dims_d, dy, dx, h.y, h.stats, h.relu, **bk)
                h.part = part
            else:
                C.conv_fwd(gys, wd, dxs, None, None, dims_d, dy, dx, trans, **bk)
            if parked is not None:   # (a launch without the accumulate epilogue: one bf16 add)
                dxs[0].add_(parked)
            ctx.bn_handle = None
        wgrads = _conv_wgrad(plan, gys, xs, (n, ih, iw, oh, ow), dev, ctx.pro, bk)
        if bwd is not None:
            from .bn import claim_deferred
            for d in bwd[4]:
                claim_deferred(d)
        bgrad = None
        if plan.bias is not None:
            bg = gys[0].view(-1, plan.Cgo)[:, :plan.co_l].float().sum(0)
            if plan.bias_sink is not None:
                plan.bias_sink.add_(bg)
            else:
                bgrad = bg
        if plan.ready_hook is not None:
            plan.ready_hook([b.weight for b in plan.branches] + ([plan.bias] if plan.bias is not None else []))
        # inputs of forward: plan, want_stats, nx, bn_handle, pro, *xs, *weights, bias
        out = [None, None, None, None, None] + dxs + wgrads
        if plan.bias is not None:
            out.append(bgrad)
        return tuple(out)


class InBnAug:
    """The first DUCK block's in_bn gradient shortcut (see :func:`ops.bn.aug_in_bn`).  The block's first convs
    read ``[z, m, 0..]`` (z = relu(bn(x)), m its ReLU mask, C channels each) and need no data-gradient: the image
    needs none, and in_bn's parameters get theirs from the weight-gradient slabs.  With G_z / G_m the slab
    channels of z / m (correlations of dY with z / m) and W the bf16 weights the forward used,
        dbeta = sum W * G_m = sum_pixels dz * m,
        sum W * G_z = sum_pixels dz * z = gamma * dgamma + beta * dbeta,
    so dgamma = (sum W * G_z - beta * dbeta) / gamma.  Exact up to fp32 summation order: the usual path's dz
    is rounded to bf16 before its BN backward sums, this one sums fp32 correlations."""

    def __init__(self, st, C):
        self.st, self.C = st, C
        self.s_z = self.s_m = None

    def add(self, w, g):
        """w: a branch's weights [co, C, T_b] (fp32 view); g: its slab channels [co, 2C, T_b] fp32."""
        wb = w.detach().to(torch.bfloat16).float()
        sz = (wb * g[:, :self.C]).sum(dim=(0, 2))
        sm = (wb * g[:, self.C:2 * self.C]).sum(dim=(0, 2))
        self.s_z = sz if self.s_z is None else self.s_z + sz
        self.s_m = sm if self.s_m is None else self.s_m + sm

    def finish(self):
        st = self.st
        gam, bet = st.weight.detach().float(), st.bias.detach().float()
        dbeta = self.s_m
        dgamma = torch.where(gam.abs() > 1e-12, (self.s_z - bet * dbeta) / gam, torch.zeros_like(gam))
        st.weight_sink.add_(dgamma)
        st.bias_sink.add_(dbeta)
        self.s_z = self.s_m = None
        if st.ready_hook is not None:
            st.ready_hook([st.weight, st.bias])


def _conv_wgrad(plan: ConvPlan, gys, xs, shape, dev, pro=([], 0), bk=None, aug=None):
    """``bk``: the BN-backward prologue kwargs of the dY groups (see :func:`_bwd_operands`); ``aug``: an
    :class:`InBnAug` collecting the z / mask channels of the slabs."""
    C = require()
    bk = bk or {}
    coefs, rmask = pro
    n, ih, iw, oh, ow = shape
    res = []
    need = [b.weight.requires_grad for b in plan.branches]
    if not any(need):
        return [None] * len(plan.branches)
    if plan.transposed:
        b = plan.branches[0]
        # dW[ci][co][t] = sum_i X[i][ci] * dY[i*S + r*d - p][co]: the X tensor plays the "output" role
        Kp_w = round_up(plan.T * plan.Cgo, 32)
        dims = [n, oh, ow, 1, plan.Cgo, ih, iw, 1, plan.Cgi, plan.ci_l, plan.T, Kp_w, plan.stride]
        dy, dx = _taps(plan.taps_fwd)
        assert not coefs, 'transposed convs take materialised inputs'
        nrep = C.conv_wgrad_replicas(dims, dy, dx, False)   # split-K slabs, summed in order by unpack
        one = plan.Cgi * plan.T * plan.Cgo
        dwp = torch.empty(nrep * one, dtype=torch.float32, device=dev)
        C.conv_wgrad(xs, gys, dwp, dims, dy, dx, False)
        dst = b.sink if b.sink is not None else torch.zeros_like(b.weight, dtype=torch.float32)
        C.unpack_wgrad(dwp, dst.view(-1), plan.ci_l, plan.co_l, plan.T, plan.Cgo, plan.T * plan.Cgo, 0, 0,
                       plan.co_l * plan.T, plan.T, True, nrep, one)
        return [None if b.sink is not None else dst]
    dims = plan.fwd_dims(n, ih, iw, oh, ow)
    dy, dx = _taps(plan.taps_fwd)
    KT = plan.T * plan.Cip
    nrep = C.conv_wgrad_replicas(dims, dy, dx, False, bool(bk), bool(coefs))   # split-K dW slabs, summed in fixed order
    dwp = torch.empty(nrep * plan.rows * KT, dtype=torch.float32, device=dev)
    C.conv_wgrad(gys, xs, dwp, dims, dy, dx, False, coefs, rmask, **bk)
    if aug is not None:   # channels [0, 2C) of every branch's slab rows (z, then the ReLU mask)
        c2 = 2 * aug.C
        for b in plan.branches:
            g = torch.empty(plan.co_l, c2, b.T, dtype=torch.float32, device=dev)
            C.unpack_wgrad(dwp[b.out_group * plan.Cgo * KT:], g.view(-1), plan.co_l, c2, b.T, plan.Cip, KT,
                           b.t_base, 0, c2 * b.T, b.T, False, nrep, plan.rows * KT)
            aug.add(b.weight.view(plan.co_l, aug.C, b.T), g)
    return _unpack_slabs(plan, dwp, nrep, need)


def _unpack_slabs(plan: ConvPlan, dwp, nrep, need):
    """dW of every branch from ``nrep`` split-K slabs [nrep][rows][T*Cip] (fixed-order sum, into the branch's
    arena sink or a fresh fp32 tensor returned to autograd)."""
    C = require()
    KT = plan.T * plan.Cip
    res = []
    cin_tot = plan.Gi * plan.ci_l
    for b, nd in zip(plan.branches, need):
        if not nd:
            res.append(None)
            continue
        dst = b.sink if b.sink is not None else torch.zeros_like(b.weight, dtype=torch.float32)
        src = dwp[b.out_group * plan.Cgo * KT:]
        flat = dst.view(-1)
        for gi in range(plan.Gi):
            C.unpack_wgrad(src, flat[gi * plan.ci_l * b.T:], plan.co_l, plan.ci_l, b.T, plan.Cip, KT, b.t_base,
                           gi * plan.Cgi, cin_tot * b.T, b.T, True, nrep, plan.rows * KT)
        res.append(None if b.sink is not None else dst)
    return res


class _MultiConvFn(torch.autograd.Function):
    """Sibling launches over ONE input tensor (the DUCK first convs split per width,
    ``runtime.fused_model.duck_split``) as one autograd node: the backward writes the input gradient
    once -- the first plan's data-gradient stores it, every later plan's ACCUMULATES in its epilogue
    (``conv_fwd(accumulate=True)``: bitwise a separate bf16 add, minus its three tensor passes) --
    then runs each plan's weight gradient.  Narrow plans (the 'P' split: singles and 3x3 + 1x1 pairs) take
    the fused data+weight-gradient kernel instead, its accumulate epilogue adding into the same tensor
    (:func:`_fused_bwd`).  Stride-1, single input group, no bias."""

    @staticmethod
    def forward(ctx, plans, want_stats, pro, mode, x, *weights):
        C = require()
        ctx.set_materialize_grads(False)
        ctx.aug, ctx.fused_ok = mode   # (InBnAug | None, narrow plans may take the fused data+weight-gradient kernel)
        x = x.contiguous()
        coefs, rmask = pro
        n, ih, iw, _ = x.shape
        dev = x.device
        outs, parts = [], []
        for plan in plans:
            oh, ow = plan.out_hw(ih, iw)
            ys = [torch.empty(n, oh, ow, plan.Cgo, dtype=torch.bfloat16, device=dev) for _ in range(plan.Go)]
            dims = plan.fwd_dims(n, ih, iw, oh, ow)
            dy, dx = _taps(plan.taps_fwd)
            part = None
            if want_stats:
                part = torch.empty(C.conv_stat_blocks(dims, dy, dx), 2, plan.rows, dtype=torch.float32, device=dev)
            C.conv_fwd([x], plan.pack_fwd(dev), ys, None, part, dims, dy, dx, False, coefs, rmask)
            outs += ys
            parts.append(part if part is not None else torch.empty(0, device=dev))
        ctx.plans, ctx.pro, ctx.shape = plans, pro, (n, ih, iw)
        ctx.save_for_backward(x)
        ctx.mark_non_differentiable(*parts)
        return (*outs, *parts)

    @staticmethod
    def backward(ctx, *grads):
        from .bn import need_grads
        C = require()
        need_grads(grads)
        (x,) = ctx.saved_tensors
        n, ih, iw = ctx.shape
        dev = x.device
        dxt, o, per_plan = None, 0, []
        fused_w = {}   # plan index -> weight gradients from the fused backward kernel (dgrad + wgrad in one)
        for pi, plan in enumerate(ctx.plans):
            oh, ow = plan.out_hw(ih, iw)
            gys = [torch.zeros(n, oh, ow, plan.Cgo, dtype=torch.bfloat16, device=dev) if g is None else g.contiguous()
                   for g in grads[o:o + plan.Go]]
            o += plan.Go
            if ctx.aug is None and ctx.fused_ok and ctx.needs_input_grad[4]:
                # narrow plans: one fused launch (deferred dY rebuilt in staging), its dgrad added into dxt
                fused = _fused_bwd(ctx, plan, gys, [x], (n, ih, iw, oh, ow), True, dev, dxt=dxt, pro=ctx.pro)
                if fused is not None:
                    dxt = fused[0][0]
                    fused_w[pi] = fused[1]
                    per_plan.append(None)
                    continue
            dims_d = [n, oh, ow, plan.Go, plan.Cgo, ih, iw, plan.Gi, plan.Cgi, plan.ci_l, plan.T, plan.Kp_d, plan.stride]
            dy, dx = _taps(plan.taps_bwd)
            gys, bwd = _bwd_operands(gys, plan, dims_d, (dy, dx), plan.fwd_dims(n, ih, iw, oh, ow),
                                     _taps(plan.taps_fwd), dgrad=ctx.needs_input_grad[4])
            bk = {} if bwd is None else dict(gy=bwd[0], gs=bwd[1], gk=bwd[2], grelu=bwd[3])
            per_plan.append((gys, bk, bwd))
            if ctx.needs_input_grad[4]:
                wd, Kp_d = plan.pack_dgrad(dev)
                first = dxt is None
                if first:
                    dxt = torch.empty(n, ih, iw, plan.Cgi, dtype=torch.bfloat16, device=dev)
                C.conv_fwd(gys, wd, [dxt], None, None, dims_d, dy, dx, False, accumulate=not first, **bk)
        wgrads = []
        for pi, (plan, pp) in enumerate(zip(ctx.plans, per_plan)):
            if pp is None:
                wgrads += fused_w[pi]
                if plan.ready_hook is not None:
                    plan.ready_hook([b.weight for b in plan.branches])
                continue
            gys, bk, bwd = pp
            oh, ow = plan.out_hw(ih, iw)
            wgrads += _conv_wgrad(plan, gys, [x], (n, ih, iw, oh, ow), dev, ctx.pro, bk, aug=ctx.aug)
            if bwd is not None:
                from .bn import claim_deferred
                for d in bwd[4]:
                    claim_deferred(d)
            if plan.ready_hook is not None:
                plan.ready_hook([b.weight for b in plan.branches])
        if ctx.aug is not None:
            ctx.aug.finish()
        ctx.plans = ctx.aug = None
        return (None, None, None, None, dxt) + tuple(wgrads)


def conv_multi(plans, x, want_stats=False, aug=None, fused_bwd=True):
    """Several stride-1 single-group plans on the same input ``x`` (tensor or Deferred) as one node;
    returns [(outputs, stat partials)] per plan.  ``aug``: ``x`` is :func:`ops.bn.aug_in_bn`'s tensor and
    ``aug`` the :class:`InBnAug` that turns the weight-gradient slabs into in_bn's gradients.  ``fused_bwd``
    False: every plan's backward on the separate data- / weight-gradient kernels (the in_bn-shortcut block with
    the shortcut off, which must match the shortcut's weight gradients bitwise)."""
    from .bn import Deferred, materialize, split_inputs
    for p in plans:
        assert p.stride == 1 and p.Gi == 1 and not p.transposed and p.bias is None
    if isinstance(x, Deferred) and x.z is None:
        n, ih, iw, _ = x.shape
        if any(not p.uses_halo(n, ih, iw) for p in plans) and plans[0].Cgi >= 64:
            x = materialize(x)   # the gather kernel's per-k-step prologue costs more than one pass (see conv)
    x = x.z if isinstance(x, Deferred) and x.z is not None else x
    (t,), coefs, mask = split_inputs([x])
    weights = [b.weight for p in plans for b in p.branches]
    out = _MultiConvFn.apply(plans, want_stats, (coefs, mask), (aug, fused_bwd), t, *weights)
    res, o = [], 0
    ngo = sum(p.Go for p in plans)
    for i, p in enumerate(plans):
        res.append((list(out[o:o + p.Go]), out[ngo + i] if want_stats else None))
        o += p.Go
    return res


def conv(plan: ConvPlan, xs, want_stats=False, bn_handle=None):
    """Run ``plan`` on input groups ``xs`` (tensors or ``ops.bn.Deferred`` BN outputs, whose
    normalise+ReLU runs as this conv's load prologue); returns (list of Go output tensors, stat
    partials).  ``bn_handle``: the input is a BN output read by this conv only
    (see ``ops.bn.BwdStatsHandle``)."""
    from .bn import Deferred, materialize, split_inputs
    if not isinstance(xs, (list, tuple)):
        xs = [xs]
    assert len(xs) == plan.Gi
    if plan.transposed:
        xs = [materialize(x) for x in xs]
    elif any(isinstance(x, Deferred) for x in xs):
        # The implicit-GEMM (non-halo) kernel re-reads every input pixel once per tap from L2, so its
        # prologue costs T times the affine work per pixel; from 64 channels up one normalise pass
        # (shared by all consumers through Deferred.z) is cheaper -- measured: L3-L5 fused-8 forward
        # +0.6 ms each with the per-k-step prologue vs ~0.05 ms for the pass.
        n, ih, iw, _ = xs[0].shape
        if plan.uses_gemm(n, ih, iw) or (not plan.uses_halo(n, ih, iw) and plan.Cgi >= 64):
            xs = [materialize(x) for x in xs]
    xs = [x.z if isinstance(x, Deferred) and x.z is not None else x for x in xs]
    ts, coefs, mask = split_inputs(xs)
    weights = [b.weight for b in plan.branches]
    extra = [plan.bias] if plan.bias is not None else []
    out = _ConvFn.apply(plan, want_stats, len(ts), bn_handle, (coefs, mask), *ts, *weights, *extra)
    return list(out[:plan.Go]), (out[plan.Go] if want_stats else None)


# ------------------------------------------------------------------------------------------------
# Pure-PyTorch reference of the same plan (NHWC padded bf16 in/out), used by CPU tests and as the
# numerics oracle for the GPU kernel tests.
def conv_reference(plan: ConvPlan, xs, dtype=torch.float32):
    import torch.nn.functional as F
    if isinstance(xs, torch.Tensor):
        xs = [xs]
    x = torch.cat([t[..., :plan.ci_l] for t in xs], dim=-1).permute(0, 3, 1, 2).to(dtype)
    outs = []
    if plan.transposed:
        w = plan.branches[0].weight.to(dtype)
        b = plan.bias.to(dtype) if plan.bias is not None else None
        y = F.conv_transpose2d(x, w, b, plan.stride, plan.padding, plan.output_padding, 1, plan.dilation)
        outs.append(y)
    else:
        by_group = {}
        for br in plan.branches:
            w = br.weight.to(dtype)
            if br.T != plan.T:   # 1x1 branch at the centre tap of a larger grid
                full = torch.zeros(w.shape[0], w.shape[1], plan.kh, plan.kw, dtype=dtype, device=w.device)
                r, s = divmod(br.t_base, plan.kw)
                full[:, :, r, s] = w[:, :, 0, 0]
                w = full
            b = plan.bias.to(dtype) if plan.bias is not None else None
            y = F.conv2d(x, w, b, plan.stride, plan.padding, plan.dilation)
            by_group[br.out_group] = y
        outs = [by_group[g] for g in range(plan.Go)]
    res = []
    for y in outs:
        n, c, h, w_ = y.shape
        o = torch.zeros(n, h, w_, plan.Cgo, dtype=torch.bfloat16, device=y.device)
        o[..., :c] = y.permute(0, 2, 3, 1).to(torch.bfloat16)
        res.append(o)
    return res
