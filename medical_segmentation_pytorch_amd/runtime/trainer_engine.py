"""THE fused MI355X training step: one implementation, driven by ``core.SegTrainer`` (``main.py``),
by ``bench.py`` (which builds a real ``SegTrainer``) and by the programmatic :class:`FusedStep`.

One step = reference ``core/seg_trainer.py:24-95`` semantics: zero_grad, forward, loss (+ KD term),
backward with DDP-style averaged gradients (RCCL buckets overlapped with backward) and SyncBN,
``scaler.step(optimizer)`` + ``scaler.update()``, then -- outside the device step -- the per-iteration
``scheduler.step()`` and the EMA update.  :class:`StepEngine` owns the device part: after ``warmup``
eager iterations (allocator / autograd warm-up, every conv plan created, then the weight pack program
built) the whole device step is captured once into a hipGraph (``torch.cuda.CUDAGraph`` is HIP graphs
on ROCm) and replayed; the only per-step host work left is writing the optimizer's hyper-parameters
(lr / betas from OneCycle, bias corrections) into its staged device tensor.
"""
from __future__ import annotations

import contextlib
import gc
from types import SimpleNamespace

import torch
import torch.distributed as dist

from ..ops._ext import require
from ..ops.bn import flush_pending
from ..ops.losses import cross_entropy, kd_kl_div


class StepEngine:
    """Device part of one fused training iteration (the trainer's and the bench's).

    ``model``: a :class:`utils.parallel.FusedModel`; ``optimizer``: a :class:`utils.optimizer.FusedOptimizer`
    (flat arena, one kernel; its bucketer -- if attached -- all-reduces the gradients during backward);
    ``loss_fn(preds, masks)``; ``scaler``: :class:`utils.optimizer.FusedGradScaler` or None; ``teacher``: a
    frozen eval-mode model (KD) with ``kd_fn(student, teacher)`` and ``kd_coef``.  ``static``: optional
    (images, masks) tensors that ARE the graph inputs (the caller writes every batch into them); otherwise
    each call copies its batch into engine-owned static buffers.

    ``accum_steps`` K > 1: gradient accumulation -- each call is one micro-batch; the first of a group zeroes
    the gradient arena, every one back-propagates ``loss / K`` (the kernels accumulate weight / BN-parameter
    gradients into the arena), and only the K-th runs the bucketed all-reduce (earlier micro-steps keep the
    bucketer quiet: torch DDP ``no_sync``) and the optimizer; ``stepped`` tells the caller whether this call
    stepped (scheduler / EMA follow optimizer steps).  Graph mode captures one graph per micro-step kind
    (first / middle / last) in ONE shared memory pool (replayed strictly in capture order, never
    concurrently).  BN statistics are per micro-batch, as with DDP + no_sync."""

    def __init__(self, model, optimizer, loss_fn, scaler=None, teacher=None, kd_fn=None, kd_coef=1.0,
                 use_graph=True, warmup=1, static=None, accum_steps=1):
        self.model, self.optimizer, self.loss_fn, self.scaler = model, optimizer, loss_fn, scaler
        self.teacher, self.kd_fn, self.kd_coef = teacher, kd_fn, kd_coef
        self.accum = max(1, int(accum_steps))
        # every micro-step kind must have run eagerly once before its capture (lazy state, plan creation)
        self.use_graph, self.warmup = use_graph, max(1, int(warmup), self.accum)
        self.images, self.masks = static if static is not None else (None, None)
        self.graph = None       # the most recently captured graph (accum 1: THE step graph)
        self.graphs = {}        # (first, last) micro-step kind -> captured graph
        self.graph_outs = {}    # (first, last) -> that graph's static (loss, kd) outputs
        self._pool = None
        self.micro = 0          # micro-step index inside the current optimizer step
        self.stepped = False    # whether the latest call ran the optimizer
        self.loss = self.kd = None
        self.last_kd = None    # KD term of the latest step (the graph's static output or a ragged eager step)
        self.calls = 0
        self._nbt_inc = None   # 0/1 per arena BN counter: BNs the executor runs (one add per step)

    @property
    def executor(self):
        return self.model.executor

    def _count_bn(self):
        """num_batches_tracked of every executor-run BN in ONE add over the optimizer arena's counter
        array (the executor is built with count_nbt=False; BNs run eagerly count themselves)."""
        arena = getattr(self.optimizer, 'arena', None)
        if arena is None or self.executor.count_nbt:
            return
        if self._nbt_inc is None:
            import torch.nn as nn
            run = {id(m) for m, _ in self.executor._bns.values()}
            bns = [m for m in self.model.module.modules()
                   if isinstance(m, nn.modules.batchnorm._BatchNorm) and m.num_batches_tracked is not None]
            inc = torch.zeros_like(arena.nbt)
            inc[:len(bns)] = torch.tensor([1 if id(m) in run else 0 for m in bns], dtype=inc.dtype)
            self._nbt_inc = inc
        arena.nbt.add_(self._nbt_inc)

    def body(self, images, masks, first=True, last=True):
        """zero_grad -> repack -> forward -> loss [+ KD] -> backward -> optimizer (+ scaler) -- capturable.
        Gradient accumulation: zero_grad / repack only on a group's ``first`` micro-step, all-reduce + optimizer
        only on its ``last``."""
        opt = self.optimizer
        if first:
            opt.zero_grad()
            self.executor.repack()
        bk = getattr(opt, 'bucketer', None)
        if bk is not None:
            bk.sync = last
        preds = self.model(images)
        loss = self.loss_fn(preds, masks)
        kd = None
        if self.teacher is not None:   # reference core/seg_trainer.py:69-79
            with torch.no_grad():
                t_out = self.teacher(images)
            kd = self.kd_fn(preds, t_out.detach())
            loss = loss + self.kd_coef * kd
            kd = kd.detach()
        sc = self.scaler if self.scaler is not None and self.scaler.is_enabled() else None
        obj = loss if self.accum == 1 else loss * (1.0 / self.accum)   # the mean over the group's micro-batches
        (sc.scale(obj) if sc is not None else obj).backward()
        flush_pending()   # SyncBN exchanges parked by the last BN backwards (normally none)
        if last:
            opt.launch(sc)    # bucket all-reduce wait + one optimizer kernel (fp16: finite check / skip)
            if sc is not None:
                sc.update()
        if self.model.training:
            self._count_bn()
        return loss.detach(), kd   # the autograd graph (and every ctx it holds) dies with this step

    def __call__(self, images=None, masks=None):
        """One device step; returns the (device) loss.  Graph mode: calls 1..warmup run eagerly on a side
        stream, the last of them builds the weight pack program; the next call captures the body and
        replays it; every later call is one replay."""
        self.calls += 1
        first, last = self.micro == 0, self.micro == self.accum - 1
        self.micro = 0 if last else self.micro + 1
        self.stepped = last
        if self.images is None:
            self.images, self.masks = torch.empty_like(images), torch.empty_like(masks)
        if images is not None and images is not self.images:
            if images.shape != self.images.shape or masks.shape != self.masks.shape:
                # ragged batch: not capturable, run eagerly.  Its loss / KD term are returned through
                # last_kd, never stored over self.loss / self.kd: those are the captured graph's static
                # outputs, which every later replay refreshes
                if last:
                    self.optimizer.prepare()
                loss, self.last_kd = self.body(images, masks, first, last)
                return loss
            self.images.copy_(images, non_blocking=True)
            self.masks.copy_(masks, non_blocking=True)
        if last:   # this step's hyper-parameters (lr, bias corrections): host work, outside the graph
            self.optimizer.prepare()
        ex = self.executor
        if not self.use_graph or self.calls <= self.warmup:
            if self.use_graph and self.images.is_cuda:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    self.loss, self.kd = self.body(self.images, self.masks, first, last)
                torch.cuda.current_stream().wait_stream(s)
            else:
                self.loss, self.kd = self.body(self.images, self.masks, first, last)
            if ex.pack_program is None and (not self.use_graph or self.calls == self.warmup):
                ex.build_pack_program(self.images.device)
            self.last_kd = self.kd
            return self.loss
        key = (first, last)
        g = self.graphs.get(key)
        if g is None:
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with no_gc(), torch.cuda.graph(g, pool=self._pool, capture_error_mode=capture_mode()):
                outs = self.body(self.images, self.masks, first, last)
            self._pool = g.pool()
            self.graphs[key] = g
            # each micro-step kind (first / middle / last of an accumulation group) has its own graph and
            # its own static loss / KD outputs: kept alive here (the shared pool cannot reuse them) and
            # selected after every replay, so a replayed 'first' step never reports the 'last' graph's loss
            self.graph_outs[key] = outs
            self.graph = g
        g.replay()
        self.loss, self.kd = self.graph_outs[key]
        self.last_kd = self.kd
        return self.loss


def iteration(engine, scheduler, ema, itrs, images=None, masks=None):
    """One training iteration exactly as ``SegTrainer.train_one_epoch`` runs it: device step, then the
    per-iteration scheduler step and EMA update (reference core/seg_trainer.py:82-87)."""
    loss = engine(images, masks)
    if not engine.stepped:   # gradient accumulation: a micro-step without an optimizer step
        return loss
    # the optimizer step ran inside the engine (launched, not via optimizer.step()): tell the LR
    # scheduler's call-order check so, which it otherwise warns about on the first step
    engine.optimizer._opt_called = True
    scheduler.step()
    ema.update(engine.model, itrs // engine.accum)   # the EMA ramp counts optimizer steps
    return loss


class FusedStep:
    """Programmatic training step (tests, tools) assembled from the SAME components ``SegTrainer`` uses:
    :class:`FusedOptimizer` (+ :class:`GradBucketer` under torch.distributed), :class:`FusedModel`,
    torch ``OneCycleLR``, :class:`ModelEmaV2` on the arena, driven by :class:`StepEngine` +
    :func:`iteration`.  ``images`` / ``masks`` are the static graph inputs; ``feed(images, masks)``
    (optional) writes the next batch into them before each step."""

    def __init__(self, model, images, masks, optimizer='adam', lr=1e-3, weight_decay=0.0, momentum=0.9,
                 total_steps=100000, pct_start=3 / 400, use_ema=False, use_graph=True, distributed=False,
                 syncbn=True, bucket_cap_mb=64.0, ignore_index=255, teacher=None, kd_temperature=4.0,
                 kd_coef=1.0, feed=None, accum_steps=1, bucket_world1=False):
        from ..utils.model_ema import ModelEmaV2
        from ..utils.optimizer import FusedOptimizer
        from ..utils.parallel import FusedModel
        from .engine import GradBucketer, stat_group
        require()
        dev = images.device
        self.model = model
        self.images, self.masks = images, masks
        self.world = dist.get_world_size() if distributed else 1
        group = dist.group.WORLD if distributed else None
        self.opt = FusedOptimizer(model, optimizer, lr=lr, momentum=momentum, weight_decay=weight_decay,
                                  device=dev)
        self.arena = self.opt.arena
        self.bucketer = None
        if distributed and (self.world > 1 or bucket_world1):   # bucket_world1: the RCCL path on one GPU (tests)
            self.bucketer = GradBucketer(self.arena, group, bucket_cap_mb)
            self.opt.attach_bucketer(self.bucketer)
        self.fm = FusedModel(model, group=stat_group(group) if syncbn else None, sinks=self.arena.sinks(),
                             ready_hook=self.bucketer.ready if self.bucketer else None, count_nbt=False)
        self.sched = torch.optim.lr_scheduler.OneCycleLR(self.opt, max_lr=lr, total_steps=total_steps,
                                                         pct_start=pct_start)
        self.ema = ModelEmaV2(SimpleNamespace(use_ema=use_ema, total_itrs=total_steps), model, dev,
                              src_arena=self.arena)
        self.ema_model = self.ema.ema
        t_fm = None
        if teacher is not None:   # KD (reference core/seg_trainer.py:69-79): frozen eval-mode fused teacher
            t_fm = FusedModel(teacher).eval()
        self.engine = StepEngine(self.fm, self.opt, lambda p, m: cross_entropy(p, m, None, ignore_index),
                                 teacher=t_fm, kd_fn=lambda s, t: kd_kl_div(s, t, kd_temperature),
                                 kd_coef=kd_coef, use_graph=use_graph, warmup=1, static=(images, masks),
                                 accum_steps=accum_steps)
        self.feed = feed
        self.itrs = 0

    @property
    def graph(self):
        return self.engine.graph

    @property
    def ex(self):
        return self.fm.executor

    def __call__(self):
        if self.feed is not None:
            self.feed(self.images, self.masks)
        self.itrs += 1
        return iteration(self.engine, self.sched, self.ema, self.itrs)


@contextlib.contextmanager
def no_gc():
    """Cyclic GC off while a step is captured: a collection that frees objects from an earlier graph or
    trainer (their CUDA-graph / event destructors) in the middle of a capture aborts the process (seen
    when the allocations of a captured step crossed a GC threshold).  torch.cuda.graph collects right
    before the capture, so nothing is left pending."""
    enabled = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if enabled:
            gc.enable()


def capture_mode():
    """hipGraph capture error mode: 'thread_local' under torch.distributed -- the process group's
    watchdog thread polls its (uncaptured) work events while a world-size-1 step is being captured, which
    the default 'global' mode turns into a capture error."""
    return 'thread_local' if dist.is_available() and dist.is_initialized() else 'global'


def make_model(model_name, base_channel=17, num_class=2):
    """Bench/test model zoo: 'ducknet' (DUCKNet-<base_channel>), 'unet' (UNet-<base_channel>),
    'smp-<encoder>' (smp Unet over a ResNet encoder, e.g. 'smp-resnet18', 'smp-resnet101'),
    'smp-<decoder>-<encoder>' (any smp decoder, e.g. 'smp-fpn-resnet18', 'smp-deeplabv3plus-resnet50')."""
    from ..models.ducknet import DuckNet
    from ..models.smp import Unet
    from ..models.unet import UNet
    if model_name == 'ducknet':
        return DuckNet(num_class=num_class, n_channel=3, base_channel=base_channel)
    if model_name == 'unet':
        return UNet(num_class=num_class, n_channel=3, base_channel=base_channel)
    if model_name.startswith('smp-'):
        parts = model_name.split('-')
        if len(parts) == 3:   # smp-<decoder>-<encoder>, e.g. smp-fpn-resnet18
            from ..models import smp
            return getattr(smp, smp_arch(parts[1]))(encoder_name=parts[2], encoder_weights=None, in_channels=3,
                                                   classes=num_class)
        return Unet(encoder_name=model_name[4:], encoder_weights=None, in_channels=3, classes=num_class)
    raise ValueError(f'unknown model {model_name!r}')


def smp_arch(name):
    """smp class name of a lower-case decoder key ('fpn' -> 'FPN', 'deeplabv3plus' -> 'DeepLabV3Plus')."""
    return {n.lower(): n for n in ('Unet', 'UnetPlusPlus', 'FPN', 'Linknet', 'MAnet', 'PAN', 'PSPNet',
                                   'DeepLabV3', 'DeepLabV3Plus')}[name]


def build_fused_step(batch, size, base_channel, device, use_graph=True, distributed=False, optimizer='adam',
                     lr=1e-3, model_name='ducknet', syncbn=True, teacher_name=None, feed=None, total_steps=100000):
    from .bench_step import synthetic_batch
    torch.manual_seed(1)
    model = make_model(model_name, base_channel).to(device).train()
    teacher = make_model(teacher_name).to(device).eval() if teacher_name else None
    if distributed:   # identical initial weights on every rank (DDP broadcast semantics)
        for m in (model, teacher):
            if m is None:
                continue
            for t in list(m.parameters()) + list(m.buffers()):
                dist.broadcast(t.data, 0)
    if teacher is not None:
        for p in teacher.parameters():
            p.requires_grad_(False)
    images, masks = synthetic_batch(batch, size, device, seed=dist.get_rank() if distributed else 0)
    return FusedStep(model, images, masks, optimizer=optimizer, lr=lr, use_graph=use_graph, distributed=distributed,
                     syncbn=syncbn, teacher=teacher, feed=feed, total_steps=total_steps)
