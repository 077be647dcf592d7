"""The fused MI355X training step used by ``bench.py`` (and, in full, by ``core.SegTrainer``).

One step = reference ``core/seg_trainer.py:24-95`` semantics: zero_grad, forward, CE loss,
backward with DDP-style averaged gradients (RCCL buckets overlapped with backward) and SyncBN,
optimizer step, OneCycle lr/momentum step, EMA update -- nothing skipped.  The whole step is
captured once into a hipGraph (``torch.cuda.CUDAGraph`` is HIP graphs on ROCm) and replayed; the
only per-step host work is writing the OneCycle values into the hyper-parameter tensor.
"""
from __future__ import annotations

import contextlib
import copy
import gc

import torch
import torch.distributed as dist

from ..ops._ext import require
from ..ops.bn import flush_pending
from ..ops.losses import cross_entropy, kd_kl_div
from .engine import Arena, FlatOptimizer, GradBucketer, OneCycle, StagedScalars, stat_group
from .fused_model import FusedExecutor


class FusedStep:
    def __init__(self, model, images, masks, optimizer='adam', lr=1e-3, weight_decay=0.0, momentum=0.9,
                 total_steps=100000, pct_start=3 / 400, use_ema=False, use_graph=True, distributed=False,
                 syncbn=True, bucket_cap_mb=64.0, ignore_index=255, teacher=None, kd_temperature=4.0,
                 kd_coef=1.0, feed=None):
        require()
        dev = images.device
        self.model = model
        self.images, self.masks = images, masks
        self.ignore_index = ignore_index
        self.world = dist.get_world_size() if distributed else 1
        group = dist.group.WORLD if distributed else None
        self.ema_model = copy.deepcopy(model).eval()
        self.arena = Arena(model, dev)
        self.bucketer = GradBucketer(self.arena, group, bucket_cap_mb) if distributed else None
        self.ex = FusedExecutor(model, group=stat_group(group) if syncbn else None, sinks=self.arena.sinks(),
                                count_nbt=False,
                                ready_hook=self.bucketer.ready if self.bucketer else None)
        kind = optimizer
        self.opt = FlatOptimizer(self.arena, kind, lr=lr, weight_decay=weight_decay, momentum=momentum)
        self.opt.grad_scale = 1.0 / self.world
        self.sched = OneCycle(lr, total_steps, pct_start)
        # EMA: flat copy of the parameter arena + running statistics (reference ModelEmaV2)
        self.ema_arena = Arena(self.ema_model, dev, with_grad=False)
        self.use_ema = use_ema
        self.ema_staged = StagedScalars(1, dev)
        self.ema_hyper = self.ema_staged.dev
        self.total_steps = total_steps
        self.itrs = 0
        self.use_graph = use_graph
        self.graph = None
        self.loss = None
        # KD (reference core/seg_trainer.py:69-79): frozen eval-mode teacher on the same fused kernels
        self.teacher = FusedExecutor(teacher) if teacher is not None else None
        self.kd_temperature, self.kd_coef = kd_temperature, kd_coef
        # feed(images, masks): writes the next (augmented) batch into the static input buffers on the
        # current stream before each step -- the data pipeline runs inside the timed loop, outside the graph
        self.feed = feed

    def _body(self):
        C = require()
        self.arena.grad.zero_()
        self.ex.repack()
        out = self.ex(self.images, training=True)
        loss = cross_entropy(out, self.masks, None, self.ignore_index)
        if self.teacher is not None:
            with torch.no_grad():
                t_out = self.teacher(self.images, training=False)
            loss = loss + self.kd_coef * kd_kl_div(out, t_out, self.kd_temperature)
        loss.backward()
        flush_pending()   # SyncBN exchanges parked by the last BN backwards (normally none)
        if self.bucketer is not None:
            self.bucketer.finish()
        self.opt.step()
        self.arena.nbt.add_(1)
        C.ema_update(self.ema_arena.data, self.arena.data, self.ema_hyper)
        C.ema_update(self.ema_arena.bufdata, self.arena.bufdata, self.ema_hyper)
        return loss.detach()   # the autograd graph (and every ctx it holds) dies with this step

    def _prepare(self):
        lr, mom = self.sched.values()
        self.opt.lr = lr
        if self.opt.kind in ('adam', 'adamw'):
            self.opt.betas = (mom, self.opt.betas[1])
        else:
            self.opt.momentum = mom
        self.opt.prepare()
        self.itrs += 1
        d = min(max(self.itrs / self.total_steps, 0.0), 1.0) if self.use_ema else 0.0
        self.ema_staged.host()[0] = d
        self.ema_staged.push()
        self.sched.step()

    def __call__(self):
        """One training step (exactly one optimizer update per call).  Graph mode: call 1 runs eagerly
        on a side stream (allocator / autograd warm-up, every plan created), call 2 builds the pack
        program, captures the body and replays it; every later call is one replay."""
        if self.feed is not None:
            self.feed(self.images, self.masks)
        self._prepare()
        if self.ex.pack_program is None and self.itrs > 1:
            self.ex.build_pack_program(self.images.device)
        if not self.use_graph:
            self.loss = self._body()
            return self.loss
        if self.itrs == 1:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self.loss = self._body()
            torch.cuda.current_stream().wait_stream(s)
            return self.loss
        if self.graph is None:
            torch.cuda.synchronize()
            self.graph = torch.cuda.CUDAGraph()
            with no_gc(), torch.cuda.graph(self.graph, capture_error_mode=capture_mode()):
                self.loss = self._body()
        self.graph.replay()
        return self.loss


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
    watchdog thread polls its work events while the step is being captured, which the default
    'global' mode turns into a capture error and a SIGABRT (seen intermittently with --graph-ddp)."""
    import torch.distributed as dist
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
        if len(parts) == 3:   # smp-<decoder>-<encoder>, e.g. smp-fpn-resnet18 (fused encoder, eager decoder)
            from ..models import smp
            arch = {n.lower(): n for n in ('Unet', 'UnetPlusPlus', 'FPN', 'Linknet', 'MAnet', 'PAN', 'PSPNet',
                                           'DeepLabV3', 'DeepLabV3Plus')}[parts[1]]
            return getattr(smp, arch)(encoder_name=parts[2], encoder_weights=None, in_channels=3, classes=num_class)
        return Unet(encoder_name=model_name[4:], encoder_weights=None, in_channels=3, classes=num_class)
    raise ValueError(f'unknown model {model_name!r}')


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
