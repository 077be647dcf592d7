"""BatchNorm(+ReLU) over NHWC bf16 feature maps on the HIP kernels (``csrc/bn.hip``).

``bn_act(xs, bn)`` computes ``act(BN(sum(xs)))`` in training or eval mode with exactly the
``nn.BatchNorm2d`` semantics of the reference (batch statistics with biased variance for the
normalisation, running statistics updated with momentum and the unbiased variance; eval uses the
running statistics).  With a process group it is ``nn.SyncBatchNorm``: the per-channel
(sum, sum-of-squares) and, in backward, (sum dy, sum dy*xmu) are all-reduced across ranks -- ONE
RCCL all-reduce of 2*C floats per BN and direction (reference ``utils/parallel.py:37-38`` does an
all-gather of (mean, invstd, count) per BN via torch's SyncBatchNorm).

Multi-input ``xs`` fuses the residual / branch sums that feed a BN (DUCK's 6-way branch sum,
``models/ducknet.py:151``; ResidualBlock ``upper + lower``, ``ducknet.py:107``) into the statistics
pass.  When the producing conv already emitted per-block channel partials (conv stats epilogue),
the statistics pass is skipped entirely.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ._ext import require


@dataclass
class BNState:
    C: int
    weight: Optional[torch.Tensor]
    bias: Optional[torch.Tensor]
    running_mean: Optional[torch.Tensor]
    running_var: Optional[torch.Tensor]
    momentum: float = 0.1
    eps: float = 1e-5
    weight_sink: Optional[torch.Tensor] = None
    bias_sink: Optional[torch.Tensor] = None
    group: object = None            # torch.distributed process group for SyncBN (None = local BN)
    num_batches_tracked: Optional[torch.Tensor] = None
    count_nbt: bool = True          # False when the engine bumps all counters in one launch
    ready_hook: Optional[object] = None

    @staticmethod
    def from_module(bn: torch.nn.modules.batchnorm._BatchNorm, group=None, sinks=None):
        sinks = sinks or {}
        return BNState(bn.num_features, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                       bn.momentum if bn.momentum is not None else 0.1, bn.eps,
                       sinks.get(id(bn.weight)) if bn.weight is not None else None,
                       sinks.get(id(bn.bias)) if bn.bias is not None else None, group,
                       bn.num_batches_tracked)


class Deferred:
    """A BatchNorm(+ReLU) output that is never materialised: ``z = act(stats[0] * t + stats[1])``
    per channel.  ``t`` is an autograd alias of the BN's input ``y`` whose gradient is dL/dz; every
    consumer kernel applies the affine+ReLU while it loads ``t`` (the "BN prologue": conv halo/igemm
    staging, weight-gradient staging, branch sums), so no ``bn_act_apply`` pass ever writes ``z``.
    :func:`materialize` turns it into a plain tensor for consumers without a prologue."""
    __slots__ = ('t', 'stats', 'relu', 'z', 'bh')

    def __init__(self, t, stats, relu, bh=None):
        self.t, self.stats, self.relu = t, stats, relu
        self.z = None   # materialised copy, made at most once (shared by every consumer that needs it)
        self.bh = bh    # BwdStatsHandle of this BN when a summing BN may emit its backward partials (bn_act partner)

    @property
    def shape(self):
        return self.t.shape

    @property
    def device(self):
        return self.t.device


def aug_in_bn(d: 'Deferred', C: int):
    """The first DUCK block's in_bn over the image, augmented: a plain 8-channel tensor
    ``[relu(bn(x)) (C channels), relu mask (C channels), 0 ...]`` built from the Deferred's scale / shift in one
    pass (``bn_aug_mask``).  It is NOT connected to autograd: the convs that read it (their weights for
    channels >= C are zero, so their outputs are exactly those on z) skip their data-gradient, and in_bn's
    gamma / beta gradients come from their weight-gradient slabs instead (``ops.conv.InBnAug``)."""
    need_stats([d])
    out = torch.empty_like(d.t)
    require().bn_aug_mask(d.t.detach().contiguous(), d.stats, out, C)
    return out


def split_inputs(xs):
    """(tensors, prologue coefficient list or [], relu bitmask) of a list of Tensor | Deferred."""
    ts, cs, mask = [], [], 0
    need_stats(xs)
    for i, x in enumerate(xs):
        if isinstance(x, Deferred):
            ts.append(x.t.contiguous())
            cs.append(x.stats)
            mask |= int(bool(x.relu)) << i
        else:
            ts.append(x.contiguous())
            cs.append(None)
    if all(c is None for c in cs):
        cs = []
    return ts, cs, mask


class _Materialize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, stats, relu):
        C = require()
        t = t.contiguous()
        Cp = t.shape[-1]
        z = torch.empty_like(t)
        C.bn_act_apply(t, stats, z, t.numel() // Cp, Cp, relu)
        return z

    @staticmethod
    def backward(ctx, dz):   # z and the alias t are the same logical tensor
        return dz, None, None


def materialize(x):
    """Plain NHWC tensor of ``x`` (Deferred -> one bn_act_apply pass; tensors pass through)."""
    if isinstance(x, Deferred):
        if x.z is None:
            need_stats([x])
            x.z = _Materialize.apply(x.t, x.stats, x.relu)
        return x.z
    return x


class BwdStatsHandle:
    """Links a training-mode BN output ``z`` that exactly ONE stride-1 conv reads (nothing else) to
    that conv: the conv's data-gradient launch -- whose output is dL/dz -- also emits the BN backward's
    channel partials (``conv_fwd_bn``), and the BN backward then skips its own partial-sum pass over
    (dz, y).  Only the executor, which knows every consumer of ``z``, creates handles."""
    __slots__ = ('y', 'stats', 'relu', 'part')

    def __init__(self):
        self.y = self.stats = self.part = None
        self.relu = False


class DeferredGrad:
    """A BatchNorm(+ReLU) data-gradient that was never written: dy = bwd(dz, y) per channel (``coef`` =
    the finalized backward coefficients, ``stats`` the forward scale/shift for the ReLU test).  The BN
    backward returns an uninitialised ``token`` tensor of dy's shape in its place; the conv that produced
    y (the only reader of y, guaranteed by the executor) either rebuilds dy while staging its data- and
    weight-gradient loads (the halo kernels' BN-backward prologue: the mirror of :class:`Deferred`), or
    :func:`resolve` writes the token (one ``bn_act_bwd_apply`` pass) and it is a plain gradient again."""
    __slots__ = ('dz', 'y', 'stats', 'coef', 'relu', 'token', 'claims', 'done')

    def __init__(self, dz, y, stats, coef, relu, token, claims):
        self.dz, self.y, self.stats, self.coef, self.relu, self.token = dz, y, stats, coef, relu, token
        self.claims, self.done = claims, False


_DEFERRED = {}   # token data_ptr -> DeferredGrad (alive between a BN backward and its producers' backward)
# env MSP_DEFER_DY=0 turns the deferral off (A/B).  A deferred gradient pays only where ONE kernel rebuilds dY
# for both the data- and the weight-gradient (ops.conv._fused_bwd, csrc/conv_bwd.hip); everywhere else the
# consumer resolves it (the same apply pass as the materialised path).  Rebuilding it in the SEPARATE halo
# data- and weight-gradient kernels measured net-neutral (profiles/r04/kernels_deferdy_{on,off}_bs320.txt:
# bn_act_bwd_apply 73.6 -> 38.1 ms/step, but each kernel re-reads y: +41 ms/step).
DEFER_DY = os.environ.get('MSP_DEFER_DY', '1') != '0'
_DY_CONSUMERS = {'_ConvFnBackward', '_MultiConvFnBackward'}


def _register_deferred(dz, y, stats, coef, relu, claims):
    token = torch.empty_like(y)
    _DEFERRED[token.data_ptr()] = DeferredGrad(dz, y, stats, coef, relu, token, claims)
    return token


def peek_deferred(g):
    """The unresolved :class:`DeferredGrad` whose token is ``g`` (None for a plain gradient)."""
    if g is None or not _DEFERRED:
        return None
    d = _DEFERRED.get(g.data_ptr())
    if d is None or d.done or d.token.shape != g.shape:
        return None
    return d


def claim_deferred(d):
    """A producer consumed ``d`` through its staging prologue (one of the BN's ``claims`` readers)."""
    d.claims -= 1
    if d.claims <= 0:
        _DEFERRED.pop(d.token.data_ptr(), None)


def resolve(g):
    """Make ``g`` a plain gradient: write a deferred token (one apply pass) the first time it is asked."""
    d = peek_deferred(g)
    if d is not None:
        C = require()
        Cp = d.y.shape[-1]
        C.bn_act_bwd_apply(d.dz, d.y, d.stats, d.coef, d.token, d.y.numel() // Cp, Cp, d.relu)
        d.done = True
        d.claims -= 1
        if d.claims <= 0:
            _DEFERRED.pop(d.token.data_ptr(), None)
    return g


def clear_deferred():
    """Step boundary: drop every token.  All of them must have been claimed or resolved by the end of
    backward; a token still unresolved means its gradient reached a node that neither rebuilt nor wrote
    it (e.g. an autograd accumulation with another gradient): that gradient was garbage, so raise (the
    mirror of ``ops.conv.check_parked_grads``)."""
    lost = sum(1 for d in _DEFERRED.values() if not d.done)
    _DEFERRED.clear()
    if lost:
        raise RuntimeError(f'{lost} deferred BN data-gradient(s) were never claimed by their producing conv nor '
                           'resolved: a deferred BN output had a consumer outside the fused backward')


def _dy_deferrable(ts):
    """Every input is produced by a conv node that knows deferred data-gradients (it claims or resolves)."""
    return all(t.grad_fn is not None and type(t.grad_fn).__name__ in _DY_CONSUMERS for t in ts)


class _Pending:
    """SyncBN statistic exchanges waiting to leave as ONE collective.

    Forward: a training BN under SyncBN reduces its local (sum, sum^2) to one fp64 row and parks
    it here with its finalize; backward: the same for (sum dy, sum dy*xmu) with finalize + apply.
    The queue is flushed -- ONE all-reduce over the concatenated rows, then every parked job -- by the
    first consumer that needs a parked result (``need_stats`` / ``need_grads``: the consumer's
    kernels read the BN coefficients or the data-gradient).  The fused executor launches sibling
    branches level by level (``runtime.fused_model._lockstep``), so every BN of a level is parked
    before any consumer runs, in both directions: per-BN collectives become per-level ones
    (reference SyncBatchNorm: one all-gather per BN forward and one all-reduce per BN backward,
    ``/root/reference/utils/parallel.py:37-38``)."""

    def __init__(self):
        self.rows, self.jobs, self.keys, self.group = [], [], set(), None

    def add(self, row, group, job, key):
        if self.rows and group is not self.group:
            self.flush()
        self.group = group
        self.rows.append(row)
        self.jobs.append(job)
        self.keys.add(key)

    def flush(self):
        if not self.rows:
            return
        rows, jobs, group = self.rows, self.jobs, self.group
        self.rows, self.jobs, self.keys, self.group = [], [], set(), None
        buf = torch.cat([r.reshape(-1) for r in rows]) if len(rows) > 1 else rows[0].reshape(-1)
        _exchange(buf, group)
        o = 0
        for r, job in zip(rows, jobs):
            job(buf[o:o + r.numel()].view(1, -1))
            o += r.numel()


_FWD, _BWD = _Pending(), _Pending()
EXCHANGES = [0]   # SyncBN collectives issued by this process (tests count them)
# Comm instrumentation (bench.py's multi-GPU evidence pass): 'enabled' False knocks the SyncBN exchanges
# out (local statistics -- a timing probe only); 'instrument' True keeps each exchange's RCCL work so its
# duration (TORCH_NCCL_ENABLE_TIMING=1) can be read after the step.
COMM = {'enabled': True, 'instrument': False, 'works': []}


class _EventSpan:
    """Duration of one IPC exchange kernel (the ``Work._get_duration`` shape of an RCCL work)."""
    __slots__ = ('a', 'b')

    def __init__(self, a, b):
        self.a, self.b = a, b

    def _get_duration(self):
        return self.a.elapsed_time(self.b)


def _exchange(buf, group):
    """One SyncBN statistic all-reduce (SUM, in place): the IPC peer-memory kernel when the group has
    one (``runtime.comm``), RCCL otherwise."""
    EXCHANGES[0] += 1
    if not COMM['enabled']:
        return
    from ..runtime import comm as ipc
    c = ipc.lookup(group)
    if c is not None and c.fits(buf):
        if COMM['instrument']:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            c.all_reduce(buf)
            b.record()
            COMM['works'].append((buf.numel() * buf.element_size(), _EventSpan(a, b)))
        else:
            c.all_reduce(buf)
        return
    if COMM['instrument']:
        w = dist.all_reduce(buf, group=group, async_op=True)
        w.wait()
        COMM['works'].append((buf.numel() * buf.element_size(), w))
    else:
        dist.all_reduce(buf, group=group)


def need_stats(xs):
    """Flush the forward queue if any Deferred in ``xs`` has coefficients still parked in it."""
    if _FWD.keys and any(isinstance(x, Deferred) and x.stats.data_ptr() in _FWD.keys for x in xs):
        _FWD.flush()


def need_stats_all():
    """Flush every parked forward exchange (before a collective issued outside the queue)."""
    _FWD.flush()


def need_grads(gs):
    """Flush the backward queue if any incoming gradient in ``gs`` is a parked BN data-gradient."""
    if _BWD.keys and any(g is not None and g.data_ptr() in _BWD.keys for g in gs):
        _BWD.flush()


def flush_pending():
    """Issue every parked exchange (step boundaries; idempotent)."""
    _FWD.flush()
    _BWD.flush()
    clear_deferred()
    from .conv import check_parked_grads
    check_parked_grads()


def _world(group):
    if group is None or not dist.is_available() or not dist.is_initialized():
        return 1
    return dist.get_world_size(group)


_COUNTERS = {}


def _counters(dev):
    """Per-device arrival counters of the fused reduce+finalize kernels (zeroed once; every call
    re-arms the counters it used, and kernels on a stream run in order)."""
    t = _COUNTERS.get(dev)
    if t is None:
        t = _COUNTERS[dev] = torch.zeros(256, dtype=torch.int32, device=dev)
    return t


def _channel_sums(C, part, nblk, width, col_off, Cp, group, dev, reduce=True):
    """fp64 [S, 2*Cp] split sums (finalize kernels sum the S rows); SyncBN: collapsed to one row and
    all-reduced across the group (one RCCL call of 2*Cp doubles; ``reduce=False``: the local row,
    for the caller to park in a :class:`_Pending` queue)."""
    S = C.bn_reduce_splits(nblk)
    tmp = torch.empty(S, 2 * Cp, dtype=torch.float64, device=dev)
    C.bn_reduce_partials(part, nblk, width, col_off, Cp, tmp)
    if _world(group) > 1:
        out = torch.empty(1, 2 * Cp, dtype=torch.float64, device=dev)
        C.bn_collapse(tmp, Cp, out)
        if reduce:
            _exchange(out, group)
        return out
    return tmp


def _apply_dy(C, dz, y, stats, coef, dy, P, Cp, relu, pt):
    """dy = the BN backward apply pass; with a partner (the handle of a deferred BN whose output is a summand of
    this BN's input) the same pass emits that BN's backward partials into ``pt.part`` -- on every rank count alike
    (a parked SyncBN apply included), so single- and multi-rank steps take the same arithmetic."""
    if pt is not None and pt.y is not None and pt.part is None and pt.y.shape == y.shape:
        part2 = torch.empty(C.bn_partial_blocks(P, Cp), 2, Cp, dtype=torch.float32, device=y.device)
        C.bn_act_bwd_apply_part(dz, y, stats, coef, dy, pt.y, pt.stats, bool(pt.relu), part2, P, Cp, relu)
        pt.part = part2
    else:
        C.bn_act_bwd_apply(dz, y, stats, coef, dy, P, Cp, relu)


class _BNAct(torch.autograd.Function):
    # inputs: st, relu, training, part_info, handle, deferred, pro, gamma, beta, *xs  (gamma/beta are
    # inputs so that their grads reach autograd when the engine gives no grad sink).  pro = (coefs,
    # relu mask): inputs that are themselves Deferred BN outputs (their prologue runs in sum_stats).
    # mode = (deferred, defer_bwd).  deferred: return the alias of y (the caller wraps it in a Deferred)
    # instead of materialising z.  defer_bwd: under SyncBN, park the backward exchange (the caller
    # guarantees every input is read only by this BN, so the returned data-gradient reaches one of
    # our backward functions -- which flush -- and never an autograd accumulation).
    @staticmethod
    def forward(ctx, st: BNState, relu: bool, training: bool, part_info, handle, mode, pro, gamma, beta, *xs):
        C = require()
        ctx.set_materialize_grads(False)   # no zero-filled grad for the non-differentiable stats output
        deferred, defer_bwd = mode[0], mode[1]
        xs = [x.contiguous() for x in xs]
        coefs, rmask = pro
        y0 = xs[0]
        Cp = y0.shape[-1]
        P = y0.numel() // Cp
        dev = y0.device
        stats = torch.empty(4, Cp, dtype=torch.float32, device=dev)
        g_ = gamma.detach() if gamma is not None else None
        b_ = beta.detach() if beta is not None else None
        summed = len(xs) > 1 or bool(coefs)   # y must be written: a sum, or a transformed input
        y = torch.empty_like(y0) if summed else y0
        if training:
            if part_info is not None and not summed:
                part, width, col_off = part_info
                nblk = part.shape[0]
            else:
                nblk = C.bn_partial_blocks(P, Cp)
                part = torch.empty(nblk, 2, Cp, dtype=torch.float32, device=dev)
                C.sum_stats(xs, y if summed else None, part, P, Cp, coefs, rmask)
                width, col_off = Cp, 0
            world = _world(st.group)
            count = float(P * world)
            if world == 1:   # one launch: column reduction + finalize (last-arriving block)
                tmp = torch.empty(C.bn_reduce_splits(nblk), 2 * Cp, dtype=torch.float64, device=dev)
                C.bn_reduce_finalize(part, nblk, width, col_off, st.C, Cp, tmp, _counters(dev), count, g_, b_,
                                     st.running_mean, st.running_var, st.momentum, st.eps, stats)
            else:            # SyncBN: collapse, park (one all-reduce per level), finalize on flush
                row = _channel_sums(C, part, nblk, width, col_off, Cp, st.group, dev, reduce=False)

                def job(sums, st=st, Cp=Cp, count=count, g_=g_, b_=b_, stats=stats):
                    C.bn_finalize(sums, st.C, Cp, count, g_, b_, st.running_mean, st.running_var, st.momentum,
                                  st.eps, True, stats)
                _FWD.add(row, st.group, job, stats.data_ptr())
                if not deferred:   # z is normalised right here
                    _FWD.flush()
            if st.count_nbt and st.num_batches_tracked is not None:
                st.num_batches_tracked.add_(1)
        else:
            if summed:
                C.add_n(xs, y, coefs, rmask)
            sums = torch.zeros(1, 2 * Cp, dtype=torch.float64, device=dev)
            C.bn_finalize(sums, st.C, Cp, 1.0, g_, b_, st.running_mean, st.running_var, st.momentum,
                          st.eps, False, stats)
            count = float(P)
        ctx.st, ctx.relu, ctx.k, ctx.count, ctx.training = st, relu, len(xs), count, training
        ctx.defer_bwd = defer_bwd
        ctx.defer_dy = bool(mode[2]) if len(mode) > 2 else False
        # partner: the handle of a deferred BN whose output is one of this BN's summands -- this BN's dy is that
        # BN's incoming gradient, so the apply pass below emits its backward partials too (bn_act_bwd_apply_part)
        ctx.partner = mode[3] if len(mode) > 3 and training else None
        ctx.handle = handle if training else None
        if ctx.handle is not None:
            handle.y, handle.stats, handle.relu, handle.part = y, stats, relu, None
        ctx.save_for_backward(y, stats)
        ctx.mark_non_differentiable(stats)
        if deferred:
            return y, stats
        z = torch.empty_like(y)
        C.bn_act_apply(y, stats, z, P, Cp, relu)
        return z, stats

    @staticmethod
    def backward(ctx, dz, _dstats=None):
        C = require()
        need_grads([dz])
        y, stats = ctx.saved_tensors
        st: BNState = ctx.st
        dz = torch.zeros_like(y) if dz is None else dz.contiguous()
        Cp = y.shape[-1]
        P = y.numel() // Cp
        dev = y.device
        h = ctx.handle
        if h is not None and h.part is not None:   # partials came with dz from the consumer's dgrad
            part, h.part = h.part, None
            nblk = part.shape[0]
        else:
            nblk = C.bn_partial_blocks(P, Cp)
            part = torch.empty(nblk, 2, Cp, dtype=torch.float32, device=dev)
            C.bn_act_bwd_partial(dz, y, stats, part, P, Cp, ctx.relu)
        world = _world(st.group) if ctx.training else 1
        fused = ctx.training and world == 1
        # park the exchange only when nothing reads this backward's outputs before the flush: dy goes to
        # our own backward functions (defer_bwd) and dgamma/dbeta to arena sinks, not to autograd
        park = (ctx.training and world > 1 and ctx.defer_bwd and (st.weight is None or st.weight_sink is not None)
                and (st.bias is None or st.bias_sink is not None))
        sums = None if fused else _channel_sums(C, part, nblk, Cp, 0, Cp, st.group if ctx.training else None, dev,
                                                reduce=not park)
        need_g = ctx.needs_input_grad[7] and st.weight_sink is None
        need_b = ctx.needs_input_grad[8] and st.bias_sink is None
        dgamma = torch.zeros(Cp, dtype=torch.float32, device=dev) if need_g else None
        dbeta = torch.zeros(Cp, dtype=torch.float32, device=dev) if need_b else None
        g_t = st.weight_sink if st.weight_sink is not None else dgamma
        b_t = st.bias_sink if st.bias_sink is not None else dbeta
        coef = torch.empty(3, Cp, dtype=torch.float32, device=dev)
        defer_dy = ctx.defer_dy and any(ctx.needs_input_grad[9:])
        if park:
            relu, count, hook = ctx.relu, ctx.count, st.ready_hook
            dy = _register_deferred(dz, y, stats, coef, relu, ctx.k) if defer_dy else torch.empty_like(y)

            pt = ctx.partner

            def job(sums, st=st, Cp=Cp, P=P):
                C.bn_bwd_finalize(sums, st.C, Cp, count, stats, g_t, b_t, coef, 1.0 / world)
                if not defer_dy:
                    _apply_dy(C, dz, y, stats, coef, dy, P, Cp, relu, pt)
                if hook is not None:
                    hook([t for t in (st.weight, st.bias) if t is not None])
            _BWD.add(sums, st.group, job, dy.data_ptr())
            ctx.partner = None
            if h is not None:
                h.y = h.stats = h.part = None
                ctx.handle = None
            return (None,) * 9 + (dy,) * ctx.k
        if fused:            # one launch: column reduction + backward finalize (last-arriving block)
            tmp = torch.empty(C.bn_reduce_splits(nblk), 2 * Cp, dtype=torch.float64, device=dev)
            C.bn_reduce_bwd_finalize(part, nblk, st.C, Cp, tmp, _counters(dev), ctx.count, stats, g_t, b_t, coef, 1.0)
        elif ctx.training:
            # global (SyncBN) sums -> dgamma/dbeta scaled by 1/world: the bucketed all-reduce-average
            # then yields the mean of the per-rank local parameter gradients (torch SyncBatchNorm).
            C.bn_bwd_finalize(sums, st.C, Cp, ctx.count, stats, g_t, b_t, coef, 1.0 / world)
        else:
            # eval-mode BN is a per-channel affine map: dx = dzr * scale
            coef[0] = stats[0]
            coef[1:] = 0
            tot = sums.sum(0).float().view(2, Cp)
            if g_t is not None:
                g_t[:st.C] += (tot[1] * stats[3])[:st.C]
            if b_t is not None:
                b_t[:st.C] += tot[0][:st.C]
        # no input needs a data-gradient (the first DUCK's in_bn over the image): only dgamma/dbeta
        need_dy = any(ctx.needs_input_grad[9:])
        dy = None
        if need_dy and defer_dy:   # the producing conv rebuilds dy in its staging (or resolves it)
            dy = _register_deferred(dz, y, stats, coef, ctx.relu, ctx.k)
        elif need_dy:
            dy = torch.empty_like(y)
            _apply_dy(C, dz, y, stats, coef, dy, P, Cp, ctx.relu, ctx.partner)
        ctx.partner = None
        if h is not None:   # break the output -> node -> ctx -> handle -> output cycle now
            h.y = h.stats = h.part = None
            ctx.handle = None
        if st.ready_hook is not None:
            st.ready_hook([t for t in (st.weight, st.bias) if t is not None])
        return (None, None, None, None, None, None, None,
                dgamma[:st.C] if dgamma is not None else None,
                dbeta[:st.C] if dbeta is not None else None) + (dy,) * ctx.k


# backward nodes whose data-gradient input may be a parked (not yet written) SyncBN dy: each calls
# need_grads() before reading it (the parked-exchange invariant of _BNAct.backward)
# (or that hands the gradient on unread to such nodes: _AddN, _Materialize)
_FLUSHING_NODES = {'_ConvFnBackward', '_MultiConvFnBackward', '_BNActBackward', '_DuckTailBackward',
                   '_Up2AddBackward', '_AddNBackward', '_MaterializeBackward', '_MaxPoolBackward',
                   '_Up2CatBackward', '_AddActBackward'}


def _check_deferrable(ts):
    """Cheap guard of the ``defer_bwd`` invariant under multi-rank SyncBN: every input must come from one
    of our autograd Functions (which flush the parked exchanges before reading a gradient) -- an input
    produced by a stock torch op would let autograd read the parked dy before it is written."""
    for t in ts:
        gf = t.grad_fn
        if gf is not None and type(gf).__name__ not in _FLUSHING_NODES:
            raise RuntimeError(f'bn_act(defer_bwd=True): input produced by {type(gf).__name__}, which does not '
                               'flush parked SyncBN exchanges; call with defer_bwd=False')


def bn_act(xs, st: BNState, relu=True, training=True, part_info=None, handle=None, deferred=False,
           defer_bwd=False, partner=None, bh=None):
    """act(BN(sum(xs))) for NHWC bf16 feature maps (``xs``: tensors and/or :class:`Deferred` BN
    outputs).  ``part_info = (part, width, col_off)`` reuses conv-epilogue channel partials (single
    plain input only); ``handle``: see :class:`BwdStatsHandle`.  ``deferred=True`` returns a
    :class:`Deferred` (no normalise pass) -- only for callers whose consumers all take prologues.
    ``defer_bwd=True``: every input is read by this BN only (SyncBN backward exchange may be parked,
    see :class:`_Pending`).  ``partner``: the :class:`BwdStatsHandle` of a Deferred input's BN (its backward partials
    come from this BN's apply pass); ``bh``: this BN's own such handle (kept on the returned Deferred)."""
    if isinstance(xs, (torch.Tensor, Deferred)):
        xs = [xs]
    ts, coefs, mask = split_inputs(xs)
    if defer_bwd and training and _world(st.group) > 1:
        _check_deferrable(ts)
    # the data-gradient stays deferred (DeferredGrad) when every input is a conv output read by this BN only
    defer_dy = DEFER_DY and defer_bwd and training and not coefs and _dy_deferrable(ts)
    if bh is not None:
        assert handle is None, 'one backward-partials handle per BN'
        handle = bh
    out, stats = _BNAct.apply(st, relu, training, part_info, handle, (deferred, defer_bwd, defer_dy, partner),
                              (coefs, mask), st.weight, st.bias, *ts)
    return Deferred(out, stats, relu, bh) if deferred else out


# ------------------------------------------------------------------------------------------------
def bn_act_reference(xs, st: BNState, relu=True, training=True):
    """Pure-torch oracle on the same NHWC layout (fp32 math, bf16 output)."""
    import torch.nn.functional as F
    if isinstance(xs, torch.Tensor):
        xs = [xs]
    y = xs[0].float()
    for x in xs[1:]:
        y = y + x.float()
    if len(xs) > 1:
        y = y.to(torch.bfloat16).float()
    Cp = y.shape[-1]
    yc = y[..., :st.C].reshape(-1, st.C).t().reshape(1, st.C, -1)
    out = F.batch_norm(yc, st.running_mean, st.running_var, st.weight, st.bias, training, st.momentum, st.eps)
    if relu:
        out = torch.relu(out)
    out = out.reshape(st.C, -1).t().reshape(*y.shape[:-1], st.C)
    z = torch.zeros(*y.shape[:-1], Cp, dtype=torch.bfloat16, device=y.device)
    z[..., :st.C] = out.to(torch.bfloat16)
    return z


# ------------------------------------------------------------------------------------------------
class BNSpec:
    """A training-mode BN(+ReLU) the caller has NOT applied yet: ``act(BN(sum(xs)))`` (``xs``: tensors
    and/or :class:`Deferred`; ``part_info`` as in :func:`bn_act`).  The DUCK tail takes the six
    branch-last BNs in this form so that their backward runs fused with out_bn's (:func:`duck_tail`)."""
    __slots__ = ('xs', 'st', 'relu', 'part_info')

    def __init__(self, xs, st, relu, part_info=None):
        self.xs, self.st, self.relu, self.part_info = list(xs), st, relu, part_info

    def apply(self, training, deferred=True):
        """The plain path: this BN as its own autograd node (eval mode, or the tail fusion off)."""
        return bn_act(self.xs, self.st, self.relu, training, self.part_info, deferred=deferred, defer_bwd=True)


def _stats_local(C, xs, coefs, rmask, part_info, P, Cp, dev):
    """(y, part, nblk, width, col_off) of a training BN's input sum (y written only for sums / prologues)."""
    summed = len(xs) > 1 or bool(coefs)
    y = torch.empty_like(xs[0]) if summed else xs[0]
    if part_info is not None and not summed:
        part, width, col_off = part_info
        return y, part, part.shape[0], width, col_off
    nblk = C.bn_partial_blocks(P, Cp)
    part = torch.empty(nblk, 2, Cp, dtype=torch.float32, device=dev)
    C.sum_stats(xs, y if summed else None, part, P, Cp, coefs, rmask)
    return y, part, nblk, Cp, 0


def _finalize_many(C, jobs, group, dev):
    """Forward finalize of several BNs: jobs = [(st, part, nblk, width, col_off, Cp, count, stats)].  One
    launch each on a single rank; under SyncBN ONE all-reduce of every BN's (sum, sum^2) row."""
    world = _world(group)
    if world == 1:
        for st, part, nblk, width, col_off, Cp, count, stats in jobs:
            tmp = torch.empty(C.bn_reduce_splits(nblk), 2 * Cp, dtype=torch.float64, device=dev)
            g_ = st.weight.detach() if st.weight is not None else None
            b_ = st.bias.detach() if st.bias is not None else None
            C.bn_reduce_finalize(part, nblk, width, col_off, st.C, Cp, tmp, _counters(dev), count, g_, b_,
                                 st.running_mean, st.running_var, st.momentum, st.eps, stats)
        return
    need_stats_all()
    rows = [_channel_sums(C, part, nblk, width, col_off, Cp, group, dev, reduce=False)
            for st, part, nblk, width, col_off, Cp, count, stats in jobs]
    buf = torch.cat([r.reshape(-1) for r in rows])
    _exchange(buf, group)
    o = 0
    for (st, part, nblk, width, col_off, Cp, count, stats), r in zip(jobs, rows):
        g_ = st.weight.detach() if st.weight is not None else None
        b_ = st.bias.detach() if st.bias is not None else None
        C.bn_finalize(buf[o:o + r.numel()].view(1, -1), st.C, Cp, count, g_, b_, st.running_mean, st.running_var,
                      st.momentum, st.eps, True, stats)
        o += r.numel()


# env MSP_TAIL_SPLIT=0: the partial pass as one six-branch launch (A/B)
_TAIL_SPLIT = os.environ.get('MSP_TAIL_SPLIT', '1') != '0'


class _DuckTail(torch.autograd.Function):
    """out_bn(act(sum_i act_i(BN_i(sum(xs_i))))) -- the DUCK block tail (reference ducknet.py:151-154) --
    with the six branch-last BNs and out_bn as ONE autograd node.  Forward: the branch BNs' statistics
    (one SyncBN collective for all six), then out_bn's sum + statistics pass over their deferred outputs.
    Backward: out_bn's partial pass, then ``bn_tail_partial`` (every branch BN's channel partials, with
    out_bn's data-gradient recomputed in registers -- it is never written), the branch finalizes (one
    collective under SyncBN), and ``bn_tail_apply`` (every branch data-gradient in one pass)."""

    @staticmethod
    def forward(ctx, specs, out_st, out_relu, pros, nx, *args):
        C = require()
        ctx.set_materialize_grads(False)
        k = len(specs)
        flat = [a.contiguous() for a in args[:sum(nx)]]
        y0 = flat[0]
        Cp = y0.shape[-1]
        P = y0.numel() // Cp
        dev = y0.device
        group = out_st.group
        world = _world(group)
        count = float(P * world)
        ys, stats, jobs, o = [], [], [], 0
        for sp, n, (coefs, rmask) in zip(specs, nx, pros):
            xs = flat[o:o + n]
            o += n
            y, part, nblk, width, col_off = _stats_local(C, xs, coefs, rmask, sp.part_info, P, Cp, dev)
            st_t = torch.empty(4, Cp, dtype=torch.float32, device=dev)
            jobs.append((sp.st, part, nblk, width, col_off, Cp, count, st_t))
            ys.append(y)
            stats.append(st_t)
        _finalize_many(C, jobs, group, dev)
        # out_bn over the branches' deferred outputs
        relu_mask = sum(int(bool(sp.relu)) << i for i, sp in enumerate(specs))
        y_sum = torch.empty_like(y0)
        nblk = C.bn_partial_blocks(P, Cp)
        part = torch.empty(nblk, 2, Cp, dtype=torch.float32, device=dev)
        C.sum_stats(ys, y_sum, part, P, Cp, stats, relu_mask)
        o_stats = torch.empty(4, Cp, dtype=torch.float32, device=dev)
        _finalize_many(C, [(out_st, part, nblk, Cp, 0, Cp, count, o_stats)], group, dev)
        for sp in list(specs) + [out_st]:
            st = sp if isinstance(sp, BNState) else sp.st
            if st.count_nbt and st.num_batches_tracked is not None:
                st.num_batches_tracked.add_(1)
        ctx.specs, ctx.out_st, ctx.out_relu, ctx.nx, ctx.k, ctx.count = specs, out_st, out_relu, nx, k, count
        ctx.relu_mask = relu_mask
        # branches whose BN input is one conv output read by this BN only (no prologue): their data-gradient can
        # stay deferred -- the producing conv rebuilds it from out_bn's data-gradient g (see backward)
        ctx.defer_ok, o = [], 0
        for n, (cs, _) in zip(nx, pros):
            ctx.defer_ok.append(DEFER_DY and n == 1 and not cs and _dy_deferrable(flat[o:o + n]))
            o += n
        ctx.save_for_backward(y_sum, o_stats, *ys, *stats)
        ctx.mark_non_differentiable(o_stats)
        return y_sum, o_stats

    @staticmethod
    def backward(ctx, dz, _dstats=None):
        C = require()
        need_grads([dz])
        k = ctx.k
        saved = ctx.saved_tensors
        y_sum, o_stats = saved[0], saved[1]
        ys, stats = list(saved[2:2 + k]), list(saved[2 + k:2 + 2 * k])
        Cp = y_sum.shape[-1]
        P = y_sum.numel() // Cp
        dev = y_sum.device
        out_st: BNState = ctx.out_st
        group = out_st.group
        world = _world(group)
        dz = torch.zeros_like(y_sum) if dz is None else dz.contiguous()
        sts = [sp.st for sp in ctx.specs] + [out_st]
        # parameter-gradient targets: arena sinks, else fresh buffers returned to autograd
        gb = []
        for st in sts:
            g_t = st.weight_sink if st.weight_sink is not None else (
                torch.zeros(Cp, dtype=torch.float32, device=dev) if st.weight is not None else None)
            b_t = st.bias_sink if st.bias_sink is not None else (
                torch.zeros(Cp, dtype=torch.float32, device=dev) if st.bias is not None else None)
            gb.append((g_t, b_t))

        def finalize(rows_parts, which):
            """backward finalize of BNs ``which`` from their partials (one collective under SyncBN)."""
            coefs = [torch.empty(3, Cp, dtype=torch.float32, device=dev) for _ in which]
            if world == 1:
                for (part, nblk), i, cf in zip(rows_parts, which, coefs):
                    tmp = torch.empty(C.bn_reduce_splits(nblk), 2 * Cp, dtype=torch.float64, device=dev)
                    st_i = o_stats if i == k else stats[i]
                    C.bn_reduce_bwd_finalize(part, nblk, sts[i].C, Cp, tmp, _counters(dev), ctx.count, st_i,
                                             gb[i][0], gb[i][1], cf, 1.0)
                return coefs
            rows = [_channel_sums(C, part, nblk, Cp, 0, Cp, group, dev, reduce=False) for part, nblk in rows_parts]
            buf = torch.cat([r.reshape(-1) for r in rows])
            _exchange(buf, group)
            o = 0
            for r, i, cf in zip(rows, which, coefs):
                st_i = o_stats if i == k else stats[i]
                C.bn_bwd_finalize(buf[o:o + r.numel()].view(1, -1), sts[i].C, Cp, ctx.count, st_i, gb[i][0], gb[i][1],
                                  cf, 1.0 / world)
                o += r.numel()
            return coefs

        nblk = C.bn_partial_blocks(P, Cp)
        part = torch.empty(nblk, 2, Cp, dtype=torch.float32, device=dev)
        C.bn_act_bwd_partial(dz, y_sum, o_stats, part, P, Cp, ctx.out_relu)
        (o_coef,) = finalize([(part, nblk)], [k])
        tb = C.bn_tail_blocks(P, Cp)
        tpart = torch.empty(k, tb, 2, Cp, dtype=torch.float32, device=dev)
        # branch partials in launches of <= 3 branches (half the accumulator registers -> twice the occupancy
        # of one six-branch launch, for one extra read of dz and ys; env MSP_TAIL_SPLIT=0: one launch)
        step = 3 if _TAIL_SPLIT else k
        for b0 in range(0, k, step):
            b1 = min(k, b0 + step)
            C.bn_tail_partial(dz, y_sum, o_stats, o_coef, ctx.out_relu, ys[b0:b1], stats[b0:b1],
                              ctx.relu_mask >> b0, tpart[b0:b1], P, Cp)
        coefs = finalize([(tpart[i], tb) for i in range(k)], list(range(k)))
        # Narrow blocks (<= 48 channels: every branch-last conv runs the fused backward, which rebuilds dY while
        # staging): the branches that allow it get a deferred data-gradient over g = out_bn's data-gradient (written
        # once by this pass) instead of their own dy -- per such branch the pass skips a y_i read and a dy_i write and
        # the consumer reads (g, y_i) instead of dy_i.
        defer = [i for i in range(k) if ctx.defer_ok[i]] if Cp <= 48 else []
        g = torch.empty_like(y_sum) if defer else None
        dys = [y_sum.new_empty(0) if i in defer else torch.empty_like(y_sum) for i in range(k)]
        # the apply pass as ONE k-branch launch (3-branch launches measured no faster, round 5)
        C.bn_tail_apply(dz, y_sum, o_stats, o_coef, ctx.out_relu, ys, stats, coefs, ctx.relu_mask, dys, P, Cp, g=g)
        for i in defer:
            dys[i] = _register_deferred(g, ys[i], stats[i], coefs[i], bool((ctx.relu_mask >> i) & 1), ctx.nx[i])
        for st in sts:
            if st.ready_hook is not None:
                st.ready_hook([t for t in (st.weight, st.bias) if t is not None])
        grads = []
        for dy, n in zip(dys, ctx.nx):
            grads += [dy] * n
        pgrads = []
        base = 5 + len(grads)   # forward inputs: specs, out_st, out_relu, pros, nx, *flat, (gamma, beta) per BN
        for j, (st, (g_t, b_t)) in enumerate(zip(sts, gb)):
            need_g = ctx.needs_input_grad[base + 2 * j] and st.weight_sink is None
            need_b = ctx.needs_input_grad[base + 2 * j + 1] and st.bias_sink is None
            pgrads.append(g_t[:st.C] if need_g else None)
            pgrads.append(b_t[:st.C] if need_b else None)
        ctx.specs = None   # drop the input references held since forward
        return (None, None, None, None, None) + tuple(grads) + tuple(pgrads)


def duck_tail(specs, out_st: BNState, out_relu=True):
    """Training-mode DUCK tail over ``specs`` (:class:`BNSpec`, the branch-last BNs): returns out_bn's
    output as a :class:`Deferred`.  Falls back to separate BN nodes where the fused passes do not apply."""
    C = require()
    widths = {(x.t if isinstance(x, Deferred) else x).shape[-1] for sp in specs for x in sp.xs}
    if len(specs) > C.kTailMax or len(widths) != 1 or widths.pop() > C.kTailMaxCp:
        outs = [sp.apply(True) for sp in specs]
        return bn_act(outs, out_st, out_relu, True, deferred=True, defer_bwd=True)
    flat, nx, pros = [], [], []
    for sp in specs:
        ts, cs, mask = split_inputs(sp.xs)
        flat += ts
        nx.append(len(ts))
        pros.append((cs, mask))
    params = []
    for st in [sp.st for sp in specs] + [out_st]:
        params += [st.weight, st.bias]
    out, stats = _DuckTail.apply(specs, out_st, out_relu, pros, nx, *flat, *params)
    return Deferred(out, stats, out_relu)
