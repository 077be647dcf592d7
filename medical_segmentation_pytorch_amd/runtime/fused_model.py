"""Fused MI355X executor for the model families: walks the reference-shaped ``nn.Module`` tree and
drives the HIP kernels with the modules' own parameters (so ``state_dict`` / checkpoints are the
reference's), keeping every activation NHWC bf16 on the device.

What is fused relative to the module graph (reference ``models/ducknet.py``, ``models/unet.py``):
  * every ConvBNAct = 1 implicit-GEMM conv launch whose epilogue emits the BN channel partials
    + one reduce/finalize launch; the normalize+ReLU never runs as a pass of its own: the BN output
    stays *deferred* (``ops.bn.Deferred``) and every consumer -- the next conv's halo/igemm staging,
    its weight-gradient staging, the branch sums feeding the next BN, the decoder up2+add -- applies
    scale/shift/ReLU while loading the pre-BN tensor (SURVEY §7.2 "BN-apply+ReLU prologue");
  * DUCK (``ducknet.py:113-154``): the five 3x3 first convs and the three 1x1 residual shortcuts
    that all read ``in_bn(x)`` are ONE GEMM with 8 output groups (Cout = 8*C), so the input is read
    once and the data-gradient of all eight is a single launch that sums them for free;
  * ResidualBlock (``ducknet.py:90-110``): the 1x1 shortcut rides in the first 3x3 conv's launch,
    and ``bn(upper + lower)`` sums inside the BN statistics pass;
  * DUCK's 6-way branch sum + ``out_bn`` is one statistics pass over six inputs;
  * decoder ``interpolate(nearest) + skip`` is one kernel; UNet's ``torch.cat`` is never built (the
    conv reads both tensors as channel groups).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..ops.bn import BNSpec, BNState, BwdStatsHandle, Deferred, aug_in_bn, bn_act, duck_tail, flush_pending, materialize
from ..ops.conv import Branch, ConvPlan, InBnAug, PackProgram, conv, conv_multi
from ..ops.elementwise import add_n, from_fm, relu6, to_fm, up2_add
from ..ops.gconv import gconv
from ..ops.pool import maxpool, res_tail, up2_cat
from .fused_decoders import SmpDecoders, fused_decoder_kind


# env MSP_BN_EPILOGUE=0 disables the dgrad-epilogue BN partials (A/B switch)
_BN_EPILOGUE = os.environ.get('MSP_BN_EPILOGUE', '1') != '0'
# env MSP_DEFER_BN=0 materialises every BN output (bn_act_apply pass) instead of deferring it (A/B switch)
_DEFER_BN = os.environ.get('MSP_DEFER_BN', '1') != '0'
# env MSP_DUCK_TAIL=0 runs the DUCK tail's seven BNs as separate autograd nodes (A/B switch; see ops.bn.duck_tail)
_DUCK_TAIL = os.environ.get('MSP_DUCK_TAIL', '1') != '0'
# env MSP_DUCK_MULTI=0 launches the separated branch's 1x7 on its own (its dgrad then adds through autograd)
_MULTI = os.environ.get('MSP_DUCK_MULTI', '1') != '0'
# The first DUCK block (in_bn over the image): its convs read [z, relu mask] and skip their data-gradient;
# in_bn's gamma / beta gradients come from the weight-gradient slabs (ops.conv.InBnAug).  A module constant
# the GPU test toggles to compare against the data-gradient path.
_AUG_INBN = True
# DUCKNet skips: the decoder's share of dL/dskip is parked for the downsample conv (ops.elementwise.up2_add)
_PARK_SKIP = True
# ResidualBlock bn(upper + lower): its backward apply pass also emits the lower BN's backward partials (no partial
# pass of its own; bitwise the same gradients).  A module constant the GPU test toggles.
_RES_PARTNER = True
# env MSP_LOCKSTEP=1/0 forces level-synchronous branch order on/off (default: on under multi-rank SyncBN)
_LOCKSTEP = {'1': True, '0': False}.get(os.environ.get('MSP_LOCKSTEP', ''))
# env MSP_FUSED_DECODERS=0 keeps every non-Unet smp decoder on the hybrid (eager decoder) path (A/B)
_FUSED_DECODERS = os.environ.get('MSP_FUSED_DECODERS', '1') != '0'


# How the DUCK block's 8 first convs (0-4: the 3x3 first convs of wide/mid/res1/res2/res3, 5-7: the
# three 1x1 residual shortcuts, reference ducknet.py:144-149) split into launches, per block width.
# One 8-group launch reads xb once and sums the 8 data-gradients in one kernel, but it carries the
# 1x1 convs at the centre tap of a 3x3 GEMM (8/9 of their MFMA work is on zero weights) and, from
# 576 output rows up, loses the halo kernel.  env MSP_DUCK_SPLIT ("8", "5+3", "3+2+3", ...) forces
# one split for every width (A/B measurements).  Measured per level at bs128, fwd+dgrad+wgrad ms
# (tools/conv_bench.py, profiles/r02/conv_bench_duck_splits_bs128.log): 17 ch @352: 8 = 10.1 vs 5+3 =
# 10.6 (the input is the largest tensor: reading it once wins); 34 @176: 8.4 vs 7.0; 68 @88: 8.4 vs 5.5;
# 136 @44: 7.0 vs 5.1 vs 3+2+3 = 4.9; 272 @22: 7.1 vs 5.8 vs 4.9.
# Round 6: where the fused narrow-conv kernel takes every piece (input and output <= 48 / 40 channels), split 'P':
# wide and mid as single 3x3 plans and each residual 3x3 with its own 1x1 shortcut as a Go = 2 pair -- every
# launch then runs the fused forward mode and the fused data+weight-gradient backward (deferred dY rebuilt in
# staging, the data-gradients summed by the accumulate epilogue): no apply passes, no chunked halo dgrad.
_PAIRS = [[0], [1], [2, 5], [3, 6], [4, 7]]


def _default_split(cout, cin=None, pairs_ok=True):
    c = (cout + 7) // 8 * 8
    if pairs_ok and cin is not None and (cin + 7) // 8 * 8 <= 48 and c <= 40:
        return 'P'
    return '8' if c <= 24 else ('5+3' if c <= 72 else '3+2+3')


def duck_split(cout, cin=None, pairs_ok=True):
    """Launches of a DUCK block's first convs (``cout`` output channels each, reading ``cin``): consecutive
    runs of the order 0..7, or 'P' (see _PAIRS); ``pairs_ok`` False: the block needs one plan over all 8
    (the first DUCK's in_bn shortcut)."""
    spec = (os.environ.get('MSP_DUCK_SPLIT') or os.environ.get(f'MSP_DUCK_SPLIT_{cout}')   # per-width override
            or _default_split(cout, cin, pairs_ok))
    if spec == 'P':
        return [list(g) for g in _PAIRS]
    sizes = [int(n) for n in spec.split('+')]
    assert sum(sizes) == 8 and min(sizes) > 0, f'bad DUCK split {spec}'
    starts = [sum(sizes[:i]) for i in range(len(sizes))]
    return [list(range(a, a + n)) for a, n in zip(starts, sizes)]


def _is_relu(act_mod):
    inner = getattr(act_mod, 'activation', act_mod)
    if isinstance(inner, nn.ReLU):
        return True
    if isinstance(inner, nn.Identity):
        return False
    raise NotImplementedError(f'fused engine supports ReLU/Identity activations, got {inner}')


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


class FusedExecutor(SmpDecoders):
    """Holds per-module plans/BN states; ``forward(model, images)`` returns NCHW fp32 logits."""

    def __init__(self, model: nn.Module, group=None, sinks=None, count_nbt=True, ready_hook=None):
        self.model = model
        self.group = group
        self.sinks = sinks or {}
        self.count_nbt = count_nbt
        self.ready_hook = ready_hook
        self._plans = {}
        self._bns = {}
        self.pack_program = None
        # BN outputs read by exactly one stride-1 conv: id(z) -> (z, BwdStatsHandle); the consuming conv
        # pops its input's handle (see ops.bn.BwdStatsHandle).  Reset every forward.
        self._handles = {}

    # Caches are keyed by id(module); the entry keeps the module itself and a hit must be the SAME
    # object (an id can be reused by a new module once the old one is freed).
    def _cached(self, cache, key, owner):
        e = cache.get(key)
        return e[1] if e is not None and e[0] is owner else None

    def build_pack_program(self, device):
        """After one forward created every plan: pack all weights in one launch per step.  The
        persistent packed buffers start zeroed, so the program runs once right away: every later
        forward -- eager or captured -- sees the current weights even before its own repack()."""
        self.pack_program = PackProgram([e[1] for e in self._plans.values()], device)
        self.pack_program.run()
        return self.pack_program

    def repack(self):
        if self.pack_program is not None:
            self.pack_program.run()

    # -- caches -------------------------------------------------------------------------------------
    def bn(self, m):
        st = self._cached(self._bns, id(m), m)
        if st is None:
            st = BNState.from_module(m, self.group, self.sinks)
            st.count_nbt = self.count_nbt
            st.ready_hook = self.ready_hook
            self._bns[id(m)] = (m, st)
        return st

    def _branch(self, conv_mod, out_group=0, t_base=0):
        kh, kw = _pair(conv_mod.kernel_size)
        return Branch(conv_mod.weight, out_group, t_base, kh * kw, self.sinks.get(id(conv_mod.weight)))

    def plan_conv(self, c: nn.Conv2d, gi=1):
        key = ('c', id(c), gi)
        p = self._cached(self._plans, key, c)
        if p is None:
            kh, kw = _pair(c.kernel_size)
            assert c.groups == 1, 'grouped convs take grouped_conv_bn'
            p = ConvPlan(kh, kw, c.in_channels // gi, c.out_channels, [self._branch(c)], stride=_pair(c.stride)[0],
                         padding=_pair(c.padding), dilation=_pair(c.dilation), Gi=gi, bias=c.bias,
                         bias_sink=self.sinks.get(id(c.bias)) if c.bias is not None else None,
                         ready_hook=self.ready_hook)
            self._plans[key] = (c, p)
        return p

    def plan_deconv(self, c: nn.ConvTranspose2d):
        key = ('t', id(c))
        p = self._cached(self._plans, key, c)
        if p is None:
            kh, kw = _pair(c.kernel_size)
            p = ConvPlan(kh, kw, c.in_channels, c.out_channels,
                         [Branch(c.weight, 0, 0, kh * kw, self.sinks.get(id(c.weight)))],
                         stride=_pair(c.stride)[0], padding=_pair(c.padding), dilation=_pair(c.dilation),
                         transposed=True, output_padding=_pair(c.output_padding)[0], bias=c.bias,
                         bias_sink=self.sinks.get(id(c.bias)) if c.bias is not None else None,
                         ready_hook=self.ready_hook)
            self._plans[key] = (c, p)
        return p

    def plan_fused3x3(self, key, convs3, convs1):
        """One 3x3/d1/p1 GEMM over sibling convs reading the same input: 3x3 convs first, then 1x1
        convs at the centre tap.  Output group order = convs3 + convs1."""
        p = self._cached(self._plans, key, convs3[0])
        if p is None:
            c0 = convs3[0]
            branches = [self._branch(c, g, 0) for g, c in enumerate(convs3)]
            branches += [self._branch(c, len(convs3) + g, 4) for g, c in enumerate(convs1)]
            for c in convs3:
                assert _pair(c.kernel_size) == (3, 3) and _pair(c.dilation) == (1, 1) and _pair(c.stride) == (1, 1)
            for c in convs1:
                assert _pair(c.kernel_size) == (1, 1) and c.bias is None
            p = ConvPlan(3, 3, c0.in_channels, c0.out_channels, branches, stride=1, padding=(1, 1),
                         dilation=(1, 1), Go=len(branches), ready_hook=self.ready_hook)
            self._plans[key] = (convs3[0], p)
        return p

    def plan_fused1x1(self, key, convs1):
        """One 1x1 GEMM over sibling 1x1 convs reading the same input (output group order = convs1)."""
        p = self._cached(self._plans, key, convs1[0])
        if p is None:
            c0 = convs1[0]
            for c in convs1:
                assert _pair(c.kernel_size) == (1, 1) and _pair(c.stride) == (1, 1) and c.bias is None
            p = ConvPlan(1, 1, c0.in_channels, c0.out_channels, [self._branch(c, g, 0) for g, c in enumerate(convs1)],
                         stride=1, padding=(0, 0), dilation=(1, 1), Go=len(convs1), ready_hook=self.ready_hook)
            self._plans[key] = (convs1[0], p)
        return p

    # -- single-consumer BN outputs ------------------------------------------------------------------
    def _bn_out(self, xs, st, relu, training, part_info=None, single=False, bh=False, partner=None):
        """Deferred bn_act; ``single``: the caller guarantees the output feeds exactly one stride-1 conv.
        ``bh``: the output is a summand of exactly one summing BN, which gets its handle as ``partner`` (that BN's
        apply pass emits this BN's backward partials: ops.bn.bn_act)."""
        h = BwdStatsHandle() if (single and training and _BN_EPILOGUE) else None
        own = BwdStatsHandle() if (bh and h is None and training and _BN_EPILOGUE and _DEFER_BN) else None
        # every caller's inputs are conv outputs / BN outputs read by this BN only -> defer_bwd
        z = bn_act(xs, st, relu, training, part_info, handle=h, deferred=_DEFER_BN, defer_bwd=True,
                   partner=partner if training else None, bh=own)
        key = z.t if isinstance(z, Deferred) else z
        if h is not None:
            self._handles[id(key)] = (key, h)
        return z

    def _conv(self, plan, xs, training):
        key = xs[0].t if isinstance(xs[0], Deferred) else xs[0]
        h = self._handles.pop(id(key), (None, None))[1] if len(xs) == 1 else None
        return conv(plan, xs, want_stats=training, bn_handle=h)

    # -- blocks -------------------------------------------------------------------------------------
    def cba(self, m, xs, training, single=False):
        """ConvBNAct: Sequential(conv, BN, act)."""
        if not isinstance(xs, (list, tuple)):
            xs = [xs]
        plan = self.plan_conv(m[0], gi=len(xs))
        (y,), part = self._conv(plan, xs, training)
        return self._bn_out([y], self.bn(m[1]), _is_relu(m[2]), training,
                            (part, plan.rows, 0) if training else None, single)

    def bn_from_group(self, bn_mod, act, ys, part, plan, g, training, single=False):
        return self._bn_out([ys[g]], self.bn(bn_mod), _is_relu(act), training,
                            (part, plan.rows, g * plan.Cgo) if training else None, single)

    def residual(self, m, x, training, single_out=False):
        return self._lockstep([self._g_residual(m, x, training, single_out)])[0]

    # -- level-synchronous branch scheduling ----------------------------------------------------------
    # A branch is a generator that yields at the end of each PHASE, alternating "conv" (launch this
    # level's conv, possibly none) and "bn" (this level's BN).  _lockstep advances sibling branches one
    # phase at a time, so all convs of a level launch before all of its BNs.  Under SyncBN that parks
    # the level's statistic exchanges together (ops.bn._Pending: ONE collective per level instead of one
    # per BN); and since autograd runs ready nodes in reverse creation order, the backward reaches every
    # BN of a level before any conv of it, which batches the backward exchanges the same way.
    def _g_cba(self, m, x, training, single=False, raw=False, bh=False):
        """``raw``: return the BN as a :class:`BNSpec` (applied later by the DUCK tail); ``bh``: see _bn_out."""
        xs = x if isinstance(x, (list, tuple)) else [x]
        plan = self.plan_conv(m[0], gi=len(xs))
        (y,), part = self._conv(plan, xs, training)
        yield
        if raw:
            z = BNSpec([y], self.bn(m[1]), _is_relu(m[2]), (part, plan.rows, 0))
        else:
            z = self._bn_out([y], self.bn(m[1]), _is_relu(m[2]), training,
                             (part, plan.rows, 0) if training else None, single, bh=bh)
        yield
        return z

    @staticmethod
    def _g_bn(fn):
        yield                # no conv at this level
        z = fn()
        yield
        return z

    def _g_residual_tail(self, m, upper_y, low_fn, training, single_out=False, raw=False):
        """ResidualBlock whose fused 3x3+1x1 launch already ran: (low BN) -> cba -> bn(upper + lower)."""
        low = yield from self._g_bn(low_fn)
        # (not raw: the block's bn(upper + lower) backward emits the lower BN's backward partials in its apply pass)
        low = yield from self._g_cba(m.lower_branch[1], low, training, bh=_RES_PARTNER and not raw)
        if raw:
            return (yield from self._g_bn(lambda: BNSpec([upper_y, low], self.bn(m.bn[0]), _is_relu(m.bn[1]))))
        partner = low.bh if isinstance(low, Deferred) else None
        return (yield from self._g_bn(lambda: self._bn_out([upper_y, low], self.bn(m.bn[0]), _is_relu(m.bn[1]),
                                                            training, single=single_out, partner=partner)))

    def _g_residual(self, m, x, training, single_out=False, raw=False):
        plan = self.plan_fused3x3(('res', id(m)), [m.lower_branch[0][0]], [m.upper_branch])
        ys, part = self._conv(plan, [x], training)
        low_fn = lambda: self.bn_from_group(m.lower_branch[0][1], m.lower_branch[0][2], ys, part, plan, 0,  # noqa: E731
                                            training, single=True)
        return (yield from self._g_residual_tail(m, ys[1], low_fn, training, single_out, raw))

    def _g_chain(self, first, blocks, training, raw=False):
        """``first`` (a branch generator) followed by residual ``blocks``, each feeding the next only;
        ``raw``: the last block's BN comes back as a :class:`BNSpec`."""
        o = yield from first
        for k, blk in enumerate(blocks):
            o = yield from self._g_residual(blk, o, training, single_out=k + 1 < len(blocks),
                                            raw=raw and k + 1 == len(blocks))
        return o

    def _g_parallel(self, gens):
        res = [None] * len(gens)
        if not self._level_sync():   # nothing to batch: plain depth-first order
            for i, g in enumerate(gens):
                while True:
                    try:
                        next(g)
                    except StopIteration as e:
                        res[i] = e.value
                        break
            return res
        live = list(range(len(gens)))
        while live:
            nxt = []
            for i in live:
                try:
                    next(gens[i])
                    nxt.append(i)
                except StopIteration as e:
                    res[i] = e.value
            live = nxt
            if live:
                yield
        return res

    def _level_sync(self):
        """Level-synchronous order only where it batches something: SyncBN over > 1 rank (env
        MSP_LOCKSTEP=1 forces it, =0 disables it)."""
        if _LOCKSTEP is not None:
            return _LOCKSTEP
        g = self.group
        return g is not None and torch.distributed.is_initialized() and torch.distributed.get_world_size(g) > 1

    def _lockstep(self, gens):
        g = self._g_parallel(gens)
        while True:
            try:
                next(g)
            except StopIteration as e:
                return e.value

    def _g_duck(self, m, xs, training):
        """DUCK block over in_bn(sum(xs)): the encoder's ``x_i + x`` merge rides in in_bn's statistics
        pass (both summands are deferred BN outputs).  in_bn's inputs may have other readers, so its
        backward exchange is never parked."""
        xb = yield from self._g_bn(lambda: bn_act(xs, self.bn(m.in_bn[0]), _is_relu(m.in_bn[1]), training,
                                                  deferred=_DEFER_BN))
        b1, b2, b3, b4, b5, b6 = m.branches()
        r4, r5 = b4[0], b5[0]
        convs3 = [b1[0][0], b2[0][0], b3.lower_branch[0][0], r4.lower_branch[0][0], r5.lower_branch[0][0]]
        convs1 = [b3.upper_branch, r4.upper_branch, r5.upper_branch]
        allc = convs3 + convs1
        # the 8 convs reading xb as one or more multi-output launches (duck_split); src[g] = (outputs,
        # partials, plan, index) of conv g
        src = [None] * 8
        # the separated branch's 1x7 reads xb too: it joins the same node (its data-gradient accumulates
        # into dL/dxb as well -- no autograd add pass for xb's gradient at all)
        sep_plan = self.plan_conv(b6[0][0])
        multi = _MULTI and sep_plan.stride == 1 and sep_plan.bias is None
        aug, aug_ok = None, False
        if multi and training and len(xs) == 1 and isinstance(xs[0], torch.Tensor) and \
                not xs[0].requires_grad and isinstance(xb, Deferred) and xb.relu:
            # in_bn over an input that needs no gradient (the image): the InBnAug shortcut
            st = self.bn(m.in_bn[0])
            nf = m.in_bn[0].num_features
            aug_ok = (xb.t.shape[-1] == 8 and 2 * nf <= 8 and st.weight_sink is not None and st.bias_sink is not None
                      and all(c.in_channels == nf for c in allc + [b6[0][0]]))
            if aug_ok and _AUG_INBN:
                aug = InBnAug(st, nf)
                xb = aug_in_bn(xb, nf)
        plans, orders = [], []
        # (the shortcut-eligible block keeps its one 8-group plan with the shortcut off too: the data-gradient path
        # then differs from the shortcut only in in_bn's gradients -- tests/test_gpu_models.py)
        split = duck_split(allc[0].out_channels, allc[0].in_channels, pairs_ok=multi and not aug_ok)
        for li, idx in enumerate(split):
            i3, i1 = [i for i in idx if i < 5], [i for i in idx if i >= 5]
            plans.append(self.plan_fused3x3(('duck', id(m), li, len(split)), [allc[i] for i in i3],
                                            [allc[i] for i in i1])
                         if i3 else self.plan_fused1x1(('duck', id(m), li, len(split)), [allc[i] for i in i1]))
            orders.append(i3 + i1)   # plan output groups: 3x3 convs first, then the 1x1s
        if multi:
            outs = conv_multi(plans + [sep_plan], xb, want_stats=training, aug=aug, fused_bwd=not aug_ok)
            sep_y, sep_part = outs[-1][0][0], outs[-1][1]
            outs = outs[:-1]
        else:
            outs = ([conv(plans[0], [xb], want_stats=training)] if len(plans) == 1
                    else conv_multi(plans, xb, want_stats=training))
        for plan, order, (ys_l, part_l) in zip(plans, orders, outs):
            for j, i in enumerate(order):
                src[i] = (ys_l, part_l, plan, j)
        ys = [src[i][0][src[i][3]] for i in range(8)]

        # every first-conv BN output feeds one conv only (single=True); branch outputs feed the 6-way sum
        def bnz(seq, g):
            ys_l, part_l, plan_l, j = src[g]
            return lambda: self.bn_from_group(seq[1], seq[2], ys_l, part_l, plan_l, j, training, single=True)

        # training: each branch's LAST BN comes back unapplied (BNSpec) and runs inside the fused tail
        raw = training and _DUCK_TAIL and _DEFER_BN

        def wide():      # d1 -> d2 -> d3
            o = yield from self._g_bn(bnz(b1[0], 0))
            o = yield from self._g_cba(b1[1], o, training, single=True)
            return (yield from self._g_cba(b1[2], o, training, raw=raw))

        def mid():       # d1 -> d2
            o = yield from self._g_bn(bnz(b2[0], 1))
            return (yield from self._g_cba(b2[1], o, training, raw=raw))

        def sep():       # 1x7 -> 7x1
            if multi:    # the 1x7 already ran in the shared launch node
                o = yield from self._g_bn(lambda: self._bn_out(
                    [sep_y], self.bn(b6[0][1]), _is_relu(b6[0][2]), training,
                    (sep_part, sep_plan.rows, 0) if training else None, single=True))
            else:
                o = yield from self._g_cba(b6[0], xb, training, single=True)
            return (yield from self._g_cba(b6[1], o, training, raw=raw))

        rest4, rest5 = list(b4)[1:], list(b5)[1:]
        # residual x1 / x2 / x3: the first block's two convs come from the fused launch; inside a chain a
        # block's output feeds only the next block's fused conv
        branches = [wide(), mid(),
                    self._g_residual_tail(b3, ys[5], bnz(b3.lower_branch[0], 2), training, raw=raw),
                    self._g_chain(self._g_residual_tail(r4, ys[6], bnz(r4.lower_branch[0], 3), training,
                                                        single_out=bool(rest4), raw=raw and not rest4),
                                  rest4, training, raw=raw),
                    self._g_chain(self._g_residual_tail(r5, ys[7], bnz(r5.lower_branch[0], 4), training,
                                                        single_out=bool(rest5), raw=raw and not rest5),
                                  rest5, training, raw=raw),
                    sep()]
        outs = yield from self._g_parallel(branches)
        if raw:   # six branch-last BNs + out_bn: one fused backward (ops.bn.duck_tail)
            return (yield from self._g_bn(lambda: duck_tail(outs, self.bn(m.out_bn[0]), _is_relu(m.out_bn[1]))))
        return (yield from self._g_bn(lambda: bn_act(outs, self.bn(m.out_bn[0]), _is_relu(m.out_bn[1]), training,
                                                     deferred=_DEFER_BN, defer_bwd=True)))

    def duck(self, m, xs, training, extra=()):
        """DUCK block; ``extra``: independent branch generators scheduled level-synchronously with it
        (their results follow the block's output in the returned list when given)."""
        res = self._lockstep([self._g_duck(m, xs, training)] + list(extra))
        return res if extra else res[0]

    def head(self, conv_mod, x, num_class):
        plan = self.plan_conv(conv_mod)
        (y,), _ = conv(plan, [x], want_stats=False)
        return from_fm(y, num_class)

    # -- models -------------------------------------------------------------------------------------
    def ducknet(self, model, images, training):
        x = to_fm(images)
        stages = model.down_stages()
        s1 = stages[0]
        skip, shortcut = self.duck(s1.duck, [x], training, extra=[self._g_cba(s1.conv2, x, training)])
        down = self.cba(s1.conv1, skip, training)
        skips = [skip]
        for st in stages[1:]:
            # x_i + x inside in_bn's stats pass; the next shortcut conv runs level-synchronously with it
            skip, shortcut = self.duck(st.duck, [down, shortcut], training,
                                       extra=[self._g_cba(st.conv2, shortcut, training)])
            down = self.cba(st.conv1, skip, training)
            skips.append(skip)
        x = add_n(down, shortcut)
        mids = list(model.mid_stage)
        for k, blk in enumerate(mids):
            x = self.residual(blk, x, training, single_out=k + 1 < len(mids))
        for st, skip in zip(model.up_stages(), reversed(skips)):
            # the skip's other reader is the encoder's downsample conv, whose backward runs after every
            # decoder node (it needs the mid blocks' gradient): it adds dL/dskip in its epilogue
            x = up2_add(x, skip, park_skip=training and _PARK_SKIP)
            x = self.duck(st.duck, [x], training)
        return self.head(model.seg_head, x, model.num_class)

    def unet(self, model, images, training):
        x = to_fm(images)
        skips = []
        for i in range(1, 5):
            st = getattr(model, f'down_stage{i}')
            f = self.cba(st.conv[0], x, training, single=True)
            f = materialize(self.cba(st.conv[1], f, training))   # maxpool has no BN prologue
            skips.append(f)
            p = st.pool
            x = maxpool(f, p.kernel_size, p.stride, p.padding)
        x = self.cba(model.mid_stage[0], x, training, single=True)
        x = self.cba(model.mid_stage[1], x, training)
        for i in range(4, 0, -1):
            st = getattr(model, f'up_stage{i}')
            dc = st.up.up_conv
            plan = self.plan_deconv(dc[0])
            (u,), part = conv(plan, [x], want_stats=training)
            u = self._bn_out([u], self.bn(dc[1]), _is_relu(dc[2]), training, (part, plan.rows, 0) if training else None)
            x = self.cba(st.conv[0], [u, skips[i - 1]], training, single=True)
            x = self.cba(st.conv[1], x, training)
        return self.head(model.seg_head, x, model.num_class)

    # -- smp Unet with a ResNet encoder (reference models/__init__.py:23-25; KD teacher :42-62) ---------
    def conv_bn(self, conv_mod, bn_mod, x, training, relu, single=False):
        if conv_mod.groups != 1:
            return self.grouped_conv_bn(conv_mod, bn_mod, x, training, relu)
        plan = self.plan_conv(conv_mod)
        (y,), part = self._conv(plan, [x], training)
        return self._bn_out([y], self.bn(bn_mod), relu, training, (part, plan.rows, 0) if training else None,
                            single)

    def grouped_conv_bn(self, conv_mod, bn_mod, x, training, relu):
        """Grouped 3x3 conv (ResNeXt ``conv2``, ``groups=32``) on the HIP grouped-conv kernels
        (``ops.gconv``, csrc/gconv.hip: direct VALU convolutions -- a group's reduction is only 36-288 long);
        until round 4 it ran on MIOpen's channels-last kernels.  Its BN takes the statistics pass (no conv
        epilogue) and never parks its backward exchange: the data-gradient goes to this op's own backward."""
        z = materialize(x)
        assert z.shape[-1] == conv_mod.in_channels, 'grouped conv input must be unpadded (C % 8 == 0)'
        y = gconv(z, conv_mod)   # (smp-Unet ResNeXt50 bs64: 1196 img/s vs 361 on MIOpen, profiles/r04/)
        return bn_act([y], self.bn(bn_mod), relu, training, deferred=_DEFER_BN)

    def resnet_block(self, blk, x, training):
        """torchvision BasicBlock / Bottleneck: ``relu(bn_last(conv_last(...)) + identity)``."""
        if blk.downsample is not None:
            idt = self.conv_bn(blk.downsample[0], blk.downsample[1], x, training, relu=False)
        else:
            idt = x
        o = self.conv_bn(blk.conv1, blk.bn1, x, training, relu=True, single=True)
        if hasattr(blk, 'conv3'):
            o = self.conv_bn(blk.conv2, blk.bn2, o, training, relu=True, single=True)
            o = self.conv_bn(blk.conv3, blk.bn3, o, training, relu=False)
        else:
            o = self.conv_bn(blk.conv2, blk.bn2, o, training, relu=False)
        # one pass from the deferred BN outputs; an identity block parks the identity gradient for conv1
        return res_tail(o, idt, park_identity=blk.downsample is None)

    def resnet_encoder(self, enc, images, training):
        """smp ResNet encoder stages 1..depth as NHWC bf16 feature maps (dilated output-stride-8/16
        variants included: their stride-1 dilated convs are ordinary fused convs)."""
        x = to_fm(images)
        f1 = materialize(self.conv_bn(enc.conv1, enc.bn1, x, training, relu=True))
        feats = [f1]
        if enc._depth >= 2:
            mp = enc.maxpool
            x = maxpool(f1, _pair(mp.kernel_size)[0], _pair(mp.stride)[0], _pair(mp.padding)[0])
        for layer in (enc.layer1, enc.layer2, enc.layer3, enc.layer4)[:max(enc._depth - 1, 0)]:
            for blk in layer:
                x = self.resnet_block(blk, x, training)
            feats.append(x)
        return feats

    def smp_hybrid(self, model, images, training):
        """smp decoders over a ResNet encoder with the decoder run eagerly (only with MSP_FUSED_DECODERS=0:
        every decoder of the hub -- Unet++, Linknet, FPN, DeepLabV3(+), PSPNet, PAN, MAnet -- has a fused
        implementation in ``runtime.fused_decoders``): the encoder -- the bulk of the FLOPs -- runs on the
        fused kernels, the decoder and head eagerly under bf16 autocast on the NCHW features (reference
        ``models/__init__.py:8-10,23-25``)."""
        enc = model.encoder
        feats = self.resnet_encoder(enc, images, training)
        chans = list(enc.out_channels[1:])
        # ResNet feature widths are multiples of 8 (no channel padding): the NHWC bf16 map IS a
        # channels-last NCHW tensor, so the decoder gets MIOpen's NHWC kernels.  The view is widened
        # to fp32 (one cast, layout kept) so that the decoder's fan-out gradients (ASPP's five
        # branches, FPN's lateral + top-down reads) accumulate in fp32 as with fp32 features; the
        # bf16 view alone cost DeepLabV3 ~0.05 of mean grad cosine vs the fp32 model.
        nchw = [images] + [f.permute(0, 3, 1, 2).float() if f.shape[-1] == c else from_fm(f, c)
                           for f, c in zip(feats, chans)]
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=images.is_cuda):
            out = model.segmentation_head(model.decoder(*nchw))
        return out.float()

    # -- smp Unet with a MobileNetV2 encoder (reference models/backbone.py:39-57, models/__init__.py:23-25) ----
    def conv_bn_relu6(self, conv_mod, bn_mod, x, training, act=True):
        """conv -> BN (-> ReLU6): convs on the implicit-GEMM / halo kernels, depthwise ones on the grouped
        kernels (csrc/gconv.hip, stride 1 or 2); ReLU6 is its own pass (``ops.elementwise.relu6``) on the
        materialised BN output.  Without ``act`` the BN output stays deferred (the block's add loads it)."""
        if conv_mod.groups != 1:
            y = gconv(materialize(x), conv_mod)
            z = bn_act([y], self.bn(bn_mod), False, training, deferred=_DEFER_BN)
        else:
            plan = self.plan_conv(conv_mod)
            (y,), part = self._conv(plan, [x], training)
            z = self._bn_out([y], self.bn(bn_mod), False, training, (part, plan.rows, 0) if training else None)
        return relu6(z) if act else z

    def inverted_residual(self, blk, x, training):
        """torchvision InvertedResidual: [1x1 expand-BN-ReLU6] -> 3x3 depthwise-BN-ReLU6 -> 1x1 project-BN
        (+ x when stride 1 and in == out: one add pass that applies the project BN while loading)."""
        layers = list(blk.conv)
        h = x
        k = 0
        if len(layers) == 8:   # expand
            h = self.conv_bn_relu6(layers[0], layers[1], h, training)
            k = 3
        h = self.conv_bn_relu6(layers[k], layers[k + 1], h, training)
        o = self.conv_bn_relu6(layers[k + 3], layers[k + 4], h, training, act=False)
        return add_n(x, o) if blk.use_res else materialize(o)

    def mobilenet_encoder(self, enc, images, training):
        x = to_fm(images)
        feats = []
        for stage in enc.get_stages()[1:enc._depth + 1]:
            for m in stage:
                if isinstance(m, nn.Sequential):   # stem conv / last 1x1: conv-BN-ReLU6
                    x = self.conv_bn_relu6(m[0], m[1], x, training)
                else:
                    x = self.inverted_residual(m, x, training)
            feats.append(x)
        return feats

    def mobilenet_unet(self, model, images, training):
        feats = self.mobilenet_encoder(model.encoder, images, training)
        return self.unet_decode(model, feats, training)

    def resnet_unet(self, model, images, training):
        return self.unet_decode(model, self.resnet_encoder(model.encoder, images, training), training)

    def unet_decode(self, model, feats, training):
        """smp UnetDecoder + head over the encoder's stage features (nearest up2 + skip concat, 2 x cba)."""
        enc, dec = model.encoder, model.decoder
        chans = list(enc.out_channels[1:])
        skips, skip_ch = feats[:-1][::-1], chans[:-1][::-1]
        x, cx = feats[-1], chans[-1]
        for i, blk in enumerate(dec.blocks):
            skip = skips[i] if i < len(skips) else None
            cs = skip_ch[i] if skip is not None else 0
            x = up2_cat(materialize(x), skip, cx, cs)
            x = self.cba(blk.conv1, x, training, single=True)
            x = self.cba(blk.conv2, x, training)
            cx = blk.conv2[0].out_channels
        return self.head(model.segmentation_head[0], x, model.segmentation_head[0].out_channels)

    def forward(self, images, training=None):
        self._handles.clear()
        try:
            return self._forward(images, training)
        finally:
            self._handles.clear()
            flush_pending()

    def _forward(self, images, training=None):
        model = self.model
        training = model.training if training is None else training
        name = type(model).__name__
        if name == 'DuckNet':
            return self.ducknet(model, images, training)
        if name == 'UNet':
            return self.unet(model, images, training)
        if _is_resnet_unet(model):
            return self.resnet_unet(model, images, training)
        if _is_mobilenet_unet(model):
            return self.mobilenet_unet(model, images, training)
        if _is_resnet_smp(model):
            kind = fused_decoder_kind(model)   # Unet++ / Linknet / FPN / DeepLabV3(+) / PSPNet: fully fused
            if kind is not None and _FUSED_DECODERS:
                return getattr(self, kind)(model, images, training)
            return self.smp_hybrid(model, images, training)
        raise NotImplementedError(f'no fused executor for {name}')

    __call__ = forward


def _is_resnet_smp(model) -> bool:
    """smp model over a non-grouped ResNet encoder (any decoder; dilated encoders included)."""
    from ..models.smp import ResNetEncoder, SegmentationModel
    if not isinstance(model, SegmentationModel):
        return False
    enc = getattr(model, 'encoder', None)
    if not isinstance(enc, ResNetEncoder) or enc._depth < 1:
        return False
    # grouped convs (ResNeXt) run on MIOpen inside the fused graph: channel widths must be unpadded
    return all(m.in_channels % 8 == 0 and m.out_channels % 8 == 0
               for m in enc.modules() if isinstance(m, nn.Conv2d) and m.groups != 1)


def _is_resnet_unet(model) -> bool:
    """smp ``Unet`` over a (non-grouped, stride-32) ResNet encoder with BatchNorm decoder blocks."""
    from ..models.smp import UnetDecoder
    if not _is_resnet_smp(model):
        return False
    enc, dec = model.encoder, model.decoder
    if not isinstance(dec, UnetDecoder) or enc._depth != 5:
        return False
    if any(_pair(m.dilation) != (1, 1) for m in enc.modules() if isinstance(m, nn.Conv2d)):
        return False
    head = model.segmentation_head
    if not isinstance(head[1], nn.Identity):
        return False
    return all(isinstance(b.conv1[1], nn.BatchNorm2d) for b in dec.blocks)


def eager_parts(model):
    """Attribute names of the sub-modules the fused executor runs eagerly (hybrid smp models)."""
    if type(model).__name__ in ('DuckNet', 'UNet') or _is_resnet_unet(model) or not _is_resnet_smp(model):
        return []
    if _FUSED_DECODERS and fused_decoder_kind(model) is not None:
        return []
    return ['decoder', 'segmentation_head']


def _is_mobilenet_unet(model) -> bool:
    """smp ``Unet`` over the MobileNetV2 encoder (stride 32, BatchNorm decoder blocks, no head upsampling)."""
    from ..models.smp import MobileNetV2Encoder, SegmentationModel, UnetDecoder
    if not isinstance(model, SegmentationModel):
        return False
    enc, dec = getattr(model, 'encoder', None), getattr(model, 'decoder', None)
    if not isinstance(enc, MobileNetV2Encoder) or not isinstance(dec, UnetDecoder) or enc._depth != 5:
        return False
    if any(_pair(m.dilation) != (1, 1) for m in enc.modules() if isinstance(m, nn.Conv2d)):
        return False
    if not isinstance(model.segmentation_head[1], nn.Identity):
        return False
    return all(isinstance(b.conv1[1], nn.BatchNorm2d) for b in dec.blocks)


def supports(model) -> bool:
    return type(model).__name__ in ('DuckNet', 'UNet') or _is_resnet_smp(model) or _is_mobilenet_unet(model)
