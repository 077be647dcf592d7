"""MI355X training engine: flat parameter/gradient arenas, single-launch optimizer + EMA, bucketed
RCCL gradient all-reduce overlapped with backward, and hipGraph capture of the whole static step.

Reference semantics reproduced (``core/seg_trainer.py:24-95``): zero_grad -> forward -> loss ->
backward (DDP bucketed all-reduce, averaging) -> optimizer.step -> scheduler.step (per iteration)
-> EMA update.  Layout decisions:

* every parameter of the model is a view into ONE fp32 arena, every gradient a view into ONE fp32
  grad arena: ``zero_grad`` is one memset, the optimizer one kernel (``csrc/optim.hip``), the EMA
  one kernel, and the DDP buckets are plain slices of the grad arena (no flatten/unflatten copies);
* the fused ops write weight gradients straight into their arena slice (grad *sinks*), and report
  completion so a bucket's all-reduce is issued the moment its last gradient lands -- RCCL runs on
  its own stream and overlaps the rest of backward (xGMI is point-to-point, so large buckets);
* BatchNorm ``num_batches_tracked`` counters live in one int64 arena (one add per step);
* hyper-parameters (lr, momentum/beta1 from OneCycle, bias corrections, 1/world) are a device
  tensor refreshed by one H2D copy before each (graph) replay.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops._ext import require


class Arena:
    """Re-homes a module's parameters (and grads) into flat contiguous buffers."""

    def __init__(self, model: nn.Module, device, align=64, with_grad=True):
        self.params: List[nn.Parameter] = [p for p in model.parameters() if p.requires_grad or not with_grad]
        offs, n = [], 0
        for p in self.params:
            offs.append(n)
            n += (p.numel() + align - 1) // align * align
        self.numel = n
        self.offsets = offs
        self.data = torch.zeros(n, dtype=torch.float32, device=device)
        self.grad = torch.zeros(n, dtype=torch.float32, device=device) if with_grad else None
        for p, o in zip(self.params, offs):
            view = self.data[o:o + p.numel()].view_as(p)
            view.copy_(p.detach())
            p.data = view
            if with_grad:
                p.grad = self.grad[o:o + p.numel()].view_as(p)
        # float buffers (BN running statistics) -> one flat arena too (single-kernel EMA)
        fb = [(m, k, b) for m in model.modules() for k, b in m._buffers.items()
              if b is not None and b.dtype == torch.float32]
        tot = sum(b.numel() for _, _, b in fb)
        self.bufdata = torch.zeros(max(tot, 1), dtype=torch.float32, device=device)
        o = 0
        for m, k, b in fb:
            view = self.bufdata[o:o + b.numel()].view_as(b)
            view.copy_(b.detach())
            m._buffers[k] = view
            o += b.numel()
        # num_batches_tracked counters
        nbts = [(m, m.num_batches_tracked) for m in model.modules()
                if isinstance(m, nn.modules.batchnorm._BatchNorm) and m.num_batches_tracked is not None]
        self.nbt = torch.zeros(max(len(nbts), 1), dtype=torch.long, device=device)
        for i, (m, t) in enumerate(nbts):
            self.nbt[i] = t.to(device)
            m.num_batches_tracked = self.nbt[i:i + 1].view(())

    def sinks(self) -> Dict[int, torch.Tensor]:
        return {id(p): p.grad for p in self.params}

    def param_index(self):
        return {id(p): i for i, p in enumerate(self.params)}


_STAT_GROUPS = {}


def register_stat_group(group, stat_group):
    """Pair ``group`` with a dedicated communicator for SyncBN statistics (created collectively by the
    caller, e.g. :func:`hpo.distributed.make_trial_groups`)."""
    _STAT_GROUPS[group] = stat_group


def stat_group(group, device=None):
    """Communicator for the SyncBN statistic exchanges of a run on ``group``.

    Each RCCL communicator runs its collectives in order on its own stream, so tiny BN all-reduces
    that share the gradient buckets' communicator queue behind multi-MB bucket all-reduces during
    backward.  For WORLD a duplicate communicator is created here (every rank of the job reaches this
    point together); a sub-group uses the partner registered by ``register_stat_group`` or, failing
    that, itself.  On a single-node GPU job the exchanges themselves then run on the IPC peer-memory
    kernel (:mod:`runtime.comm`), attached here collectively; the RCCL communicator stays the fallback.
    """
    if group is None or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return group
    if group in _STAT_GROUPS:
        sg = _STAT_GROUPS[group]
    elif group is dist.group.WORLD or dist.get_world_size(group) == dist.get_world_size():
        sg = _STAT_GROUPS[group] = dist.new_group(list(range(dist.get_world_size())))
    else:
        sg = group
    if device is None and torch.cuda.is_available():
        device = torch.device('cuda', torch.cuda.current_device())
    from . import comm
    comm.attach(sg, device)
    return sg


class _Bucket:
    """One all-reduce unit: ``members`` (arena parameter indices, in the order their gradients land).
    ``span`` = (lo, hi) when the members tile one contiguous arena slice (the all-reduce runs in place);
    otherwise the bucket is *packed*: its gradients are gathered into a staging slice (one multi-tensor
    copy), all-reduced there and scattered back in ``finish``."""

    def __init__(self, arena, members):
        self.members = list(members)
        self.set = set(self.members)
        self.numel = sum(arena.params[i].numel() for i in self.members)
        lo = min(arena.offsets[i] for i in self.members)
        hi = max(arena.offsets[i] + arena.params[i].numel() for i in self.members)
        inside = {i for i, o in enumerate(arena.offsets) if lo <= o < hi}
        self.span = (lo, hi) if inside == self.set else None
        self.stage = None   # (lo, hi) in the staging buffer of a packed bucket


class GradBucketer:
    """DDP-equivalent gradient averaging over RCCL: a bucket is all-reduced as soon as all of its
    parameters reported ready (SUM; the 1/world factor is folded into the optimizer's grad scale).

    Bucket order: the first step's buckets follow reverse registration order (backward produces the
    last layers first -- torch DDP's initial guess) as contiguous slices of the grad arena.  During that
    step every gradient's arrival is recorded (``ready_order``); at its ``finish`` rank 0's observed
    order is broadcast and the buckets are REBUILT in that order (torch DDP's rebuild-after-first-
    iteration), so every bucket's gradients land together and it leaves as early as possible.  A rebuilt
    bucket whose members are not one contiguous arena slice is packed through a staging buffer.

    ``compress='bf16'`` (config ``grad_compress``; torch DDP's ``bf16_compress_hook``): a ready bucket
    is rounded into a persistent bf16 shadow, all-reduced at half the xGMI bytes, and widened back into
    the fp32 arena in :meth:`finish`."""

    def __init__(self, arena: Arena, group=None, bucket_cap_mb=64.0, first_bucket_mb=4.0, compress=None,
                 rebuild=True):
        self.arena = arena
        self.group = group
        self.world = dist.get_world_size(group)
        if compress not in (None, 'bf16'):
            raise ValueError(f'grad_compress must be None or "bf16", got {compress!r}')
        self.compress = compress
        self.cap_mb, self.first_mb = bucket_cap_mb, first_bucket_mb
        self.shadow = torch.empty(arena.numel, dtype=torch.bfloat16, device=arena.grad.device) \
            if compress == 'bf16' else None
        self.stage = None
        self.pidx = arena.param_index()
        self._assign(list(range(len(arena.params)))[::-1])
        self.rebuild_pending = rebuild
        self.rebuilt = False
        # evidence knobs (bench.py's multi-GPU pass): enabled=False skips the all-reduces (timing probe);
        # instrument=True records, per bucket, an event at issue time and the RCCL work (its on-stream
        # duration needs TORCH_NCCL_ENABLE_TIMING=1), read back by collect() after the step
        self.enabled = True
        # gradient accumulation: False on every micro-step but an optimizer step's last (torch DDP no_sync):
        # the gradients keep accumulating in the arena and only the last micro-step's backward buckets them
        self.sync = True
        self.instrument = False
        self.records = []
        self.ready_order = []   # parameter indices in the order their gradients landed (first step)
        self.reset()

    def _assign(self, order):
        """Cut ``order`` into buckets (first one small: it leaves early; then ``cap_mb`` each)."""
        a = self.arena
        groups, cur, cur_bytes, cap = [], [], 0, self.first_mb * 2 ** 20
        for i in order:
            cur.append(i)
            cur_bytes += a.params[i].numel() * 4
            if cur_bytes >= cap:
                groups.append(cur)
                cur, cur_bytes, cap = [], 0, self.cap_mb * 2 ** 20
        if cur:
            groups.append(cur)
        self.buckets = [_Bucket(a, g) for g in groups]
        self.owner = {i: b for b, bk in enumerate(self.buckets) for i in bk.members}
        n, dev = 0, a.grad.device
        for bk in self.buckets:
            if bk.span is None:
                bk.stage = (n, n + bk.numel)
                n += bk.numel
        dtype = torch.bfloat16 if self.compress == 'bf16' else torch.float32
        self.stage = torch.empty(n, dtype=dtype, device=dev) if n else None
        for bk in self.buckets:
            if bk.span is None:
                lo = bk.stage[0]
                bk.grads = [a.params[i].grad.view(-1) for i in bk.members]
                bk.views = []
                for g in bk.grads:
                    bk.views.append(self.stage[lo:lo + g.numel()])
                    lo += g.numel()

    def rebuild(self):
        """Re-bucket along the grad-ready order observed in the first step (identical on every rank:
        rank 0's order is broadcast).  Parameters that never reported come last."""
        n = len(self.arena.params)
        seen = set(self.ready_order)
        order = list(dict.fromkeys(self.ready_order)) + [i for i in range(n - 1, -1, -1) if i not in seen]
        t = torch.tensor(order, dtype=torch.int64, device=self.arena.grad.device)
        if self.world > 1:
            dist.broadcast(t, dist.get_global_rank(self.group, 0) if self.group is not None and
                           self.group is not dist.group.WORLD else 0, group=self.group)
        self._assign(t.cpu().tolist())
        self.rebuilt = True

    def bucket_order(self):
        """Parameter indices in bucket order (bucket 0's members first)."""
        return [i for bk in self.buckets for i in bk.members]

    def reset(self):
        self.pending = [set(bk.set) for bk in self.buckets]
        self.works = []
        self.launched = [False] * len(self.buckets)
        self.launch_order = []

    def ready(self, params):
        if not self.sync:
            return
        for p in params:
            i = self.pidx.get(id(p))
            if i is None:
                continue
            if len(self.ready_order) < len(self.arena.params):
                self.ready_order.append(i)
            b = self.owner[i]
            self.pending[b].discard(i)
            if not self.pending[b] and not self.launched[b]:
                self._launch(b)

    def _launch(self, b, late=False):
        bk = self.buckets[b]
        self.launched[b] = True
        self.launch_order.append((b, late))
        if bk.span is not None:
            lo, hi = bk.span
            buf = self.arena.grad[lo:hi]
            if self.shadow is not None:
                buf = self.shadow[lo:hi]
                buf.copy_(self.arena.grad[lo:hi])
        else:   # packed: gather the members' gradients into the staging slice (one multi-tensor copy)
            torch._foreach_copy_(bk.views, bk.grads)
            buf = self.stage[bk.stage[0]:bk.stage[1]]
        ev = None
        if self.instrument:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        w = dist.all_reduce(buf, group=self.group, async_op=True) if self.enabled else None
        self.works.append((b, w, ev))

    def finish(self):
        from ..ops.bn import flush_pending
        flush_pending()   # parked SyncBN backward jobs report their gamma/beta grads ready
        end = None
        if self.instrument:   # backward's end on the compute stream (every bucket's data is ready by now)
            end = torch.cuda.Event(enable_timing=True)
            end.record()
        for b in range(len(self.buckets)):
            if not self.launched[b]:
                self._launch(b, late=True)
        for b, w, ev in self.works:
            if w is not None:
                w.wait()
            bk = self.buckets[b]
            if bk.span is None:
                torch._foreach_copy_(bk.grads, bk.views)
            elif self.shadow is not None:
                lo, hi = bk.span
                self.arena.grad[lo:hi].copy_(self.shadow[lo:hi])
        if self.instrument:
            self.records.append((list(self.works), end, list(self.launch_order)))
        self.reset()
        if self.rebuild_pending:   # after the first step: re-bucket in the observed grad-ready order
            self.rebuild_pending = False
            self.rebuild()
            self.reset()

    def collect(self):
        """Per-bucket evidence of the instrumented steps (host-syncs; call after the timed region):
        MiB, RCCL on-stream ms, ms between the bucket's issue and backward's end (the compute it could
        hide under), and whether it launched only at finish() (not overlapped at all)."""
        torch.cuda.synchronize()
        out = []
        for works, end, order in self.records:
            late = {b: lt for b, lt in order}
            for b, w, ev in works:
                bk = self.buckets[b]
                dur = None
                if w is not None:
                    try:
                        dur = float(w._get_duration())
                    except Exception:
                        dur = None
                out.append({'bucket': b, 'mib': round(bk.numel * 4 / 2 ** 20, 2), 'packed': bk.span is None,
                            'rccl_ms': dur,
                            'issue_to_bwd_end_ms': round(ev.elapsed_time(end), 3) if ev is not None and end is not None
                            else None, 'late': bool(late.get(b, False))})
        self.records = []
        return out


class StagedScalars:
    """A small device fp32 tensor refreshed from pinned host memory once per step, race-free.

    The host runs ahead of the GPU (hipGraph replays / eager launches are asynchronous), so a single
    pinned staging buffer could be overwritten with step k+1's values before the DMA of step k's
    copy has read it.  The staging buffers form a ring; a slot is rewritten only after the event
    recorded behind its previous copy completed (a stall only if the host is ``depth`` steps ahead).
    ``dev`` keeps its address, so graphs that captured it stay valid."""

    def __init__(self, n, device, depth=8):
        self.dev = torch.zeros(n, dtype=torch.float32, device=device)
        self.cuda = self.dev.is_cuda
        self.ring = [torch.zeros(n, dtype=torch.float32).pin_memory() if self.cuda else torch.zeros(n)
                     for _ in range(depth)]
        self.events = [None] * depth
        self.i = 0

    def host(self):
        """The next writable pinned buffer (waits for its previous copy if still in flight)."""
        ev = self.events[self.i]
        if ev is not None:
            ev.synchronize()
        return self.ring[self.i]

    def push(self):
        """Enqueue the H2D copy of the buffer returned by :meth:`host` on the current stream."""
        buf = self.ring[self.i]
        self.dev.copy_(buf, non_blocking=True)
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()
            self.events[self.i] = ev
        self.i = (self.i + 1) % len(self.ring)


class FlatOptimizer:
    """Adam / AdamW / SGD(momentum, wd) over the arena in one kernel (torch.optim semantics)."""

    def __init__(self, arena: Arena, kind='adam', lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 momentum=0.9):
        self.arena, self.kind = arena, kind
        self.lr, self.betas, self.eps, self.wd, self.momentum = lr, betas, eps, weight_decay, momentum
        dev = arena.data.device
        n = arena.numel
        if kind in ('adam', 'adamw'):
            self.m = torch.zeros(n, device=dev)
            self.v = torch.zeros(n, device=dev)
        else:
            self.buf = torch.zeros(n, device=dev)
        self.step_count = 0
        self.staged = StagedScalars(8, dev)
        self.hyper = self.staged.dev
        self.grad_scale = 1.0

    def prepare(self):
        """Host-side: advance step count, write hyper-parameters, H2D copy (outside any graph)."""
        self.step_count += 1
        h = self.staged.host()
        if self.kind in ('adam', 'adamw'):
            b1, b2 = self.betas
            h[0], h[1], h[2], h[3], h[4] = self.lr, b1, b2, self.eps, self.wd
            h[5] = 1 - b1 ** self.step_count
            h[6] = 1 - b2 ** self.step_count
            h[7] = self.grad_scale
        else:
            h[0], h[1], h[2], h[3] = self.lr, self.momentum, self.wd, self.grad_scale
        self.staged.push()

    def step(self):
        C = require()
        a = self.arena
        if self.kind in ('adam', 'adamw'):
            C.adam_step(a.data, a.grad, self.m, self.v, self.hyper, self.kind == 'adamw')
        else:
            C.sgd_step(a.data, a.grad, self.buf, self.hyper)


class OneCycle:
    """torch.optim.lr_scheduler.OneCycleLR (cos anneal, cycle_momentum) computed on the host, per
    iteration -- the values feed the device hyper tensor (reference utils/scheduler.py:13-19)."""

    def __init__(self, max_lr, total_steps, pct_start=0.3, anneal='cos', div_factor=25.0, final_div_factor=1e4,
                 base_momentum=0.85, max_momentum=0.95):
        self.max_lr, self.total = max_lr, total_steps
        self.initial = max_lr / div_factor
        self.min_lr = self.initial / final_div_factor
        self.anneal = anneal
        self.phase_end = [float(pct_start * total_steps) - 1, float(total_steps - 1)]
        self.bm, self.mm = base_momentum, max_momentum
        self.step_num = 0

    def _f(self, start, end, pct):
        if self.anneal == 'cos':
            return end + (start - end) / 2.0 * (math.cos(math.pi * pct) + 1)
        return (end - start) * pct + start

    def values(self, step=None):
        s = self.step_num if step is None else step
        start = 0
        if s <= self.phase_end[0]:
            pct = (s - start) / max(self.phase_end[0] - start, 1e-12)
            return self._f(self.initial, self.max_lr, pct), self._f(self.mm, self.bm, pct)
        start = self.phase_end[0]
        pct = (s - start) / max(self.phase_end[1] - start, 1e-12)
        return self._f(self.max_lr, self.min_lr, pct), self._f(self.bm, self.mm, pct)

    def step(self):
        self.step_num += 1
