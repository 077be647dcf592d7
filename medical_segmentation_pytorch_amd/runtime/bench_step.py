"""Training-step factories used by ``bench.py`` and ``tools/test_speed.py``.

``eager``: stock PyTorch-ROCm step with the reference's exact semantics (DDP + SyncBN + autocast,
per-tensor EMA copy) -- the in-house reference speed.  ``fused``: the MI355X-native engine.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn


def synthetic_batch(batch, size, device, num_class=2, seed=0):
    """Polyp-like synthetic batch: textured RGB image + one elliptical foreground blob per image."""
    g = torch.Generator(device='cpu').manual_seed(seed)
    yy, xx = torch.meshgrid(torch.arange(size, dtype=torch.float32),
                            torch.arange(size, dtype=torch.float32), indexing='ij')
    masks = torch.zeros(batch, size, size, dtype=torch.long)
    for i in range(batch):
        cy, cx = (torch.rand(2, generator=g) * 0.5 + 0.25) * size
        ry, rx = (torch.rand(2, generator=g) * 0.2 + 0.1) * size
        masks[i] = ((((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2) <= 1).long()
    images = torch.randn(batch, 3, size, size, generator=g) * 0.5
    images += masks[:, None].float() * torch.tensor([0.8, -0.3, -0.2])[None, :, None, None]
    if num_class == 1:
        masks = masks.float()
    return images.to(device), masks.to(device)


class _OneCycle:
    """Lightweight handle so eager and fused paths step an identical OneCycle schedule."""

    def __init__(self, optimizer, max_lr, total_steps, pct_start=3 / 400):
        self.sched = torch.optim.lr_scheduler.OneCycleLR(optimizer, max_lr=max_lr,
                                                         total_steps=total_steps, pct_start=pct_start)

    def step(self):
        self.sched.step()


def build_eager_step(batch, size, base_channel, device, channels_last=False, distributed=False,
                     lr=1e-3, total_steps=100000, model_name='ducknet', teacher_name=None, kd_temperature=4.0,
                     feed=None):
    from .trainer_engine import make_model
    torch.manual_seed(1)
    model = make_model(model_name, base_channel).to(device)
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    model = model.to(memory_format=fmt)
    ema = make_model(model_name, base_channel).to(device).eval()
    ema.load_state_dict(model.state_dict())
    teacher = make_model(teacher_name).to(device).to(memory_format=fmt).eval() if teacher_name else None
    if distributed:
        model = nn.SyncBatchNorm.convert_sync_batchnorm(model)
        model = nn.parallel.DistributedDataParallel(model, device_ids=[device.index],
                                                    output_device=device.index)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    sched = _OneCycle(opt, lr, total_steps)
    loss_fn = nn.CrossEntropyLoss(ignore_index=255)
    images, masks = synthetic_batch(batch, size, device)
    images = images.contiguous(memory_format=fmt)
    ema_vals = list(ema.state_dict().values())

    nchw = torch.empty(images.shape, dtype=images.dtype, device=device)

    def step():
        if feed is not None:   # same data pipeline as the fused step (GPU augmentation per batch)
            feed(nchw, masks)
            images.copy_(nchw)
        opt.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16):
            preds = model(images)
            loss = loss_fn(preds, masks)
            if teacher is not None:   # reference core/seg_trainer.py:69-79 + core/loss.py:42-49
                with torch.no_grad():
                    t_out = teacher(images)
                T = kd_temperature
                loss = loss + nn.functional.kl_div(nn.functional.log_softmax(preds.float() / T, 1),
                                                   nn.functional.softmax(t_out.float() / T, 1)) * T * T
        loss.backward()
        opt.step()
        sched.step()
        src = model.module if distributed else model
        with torch.no_grad():   # reference ModelEmaV2 with use_ema=False: copy every tensor
            for e, m in zip(ema_vals, src.state_dict().values()):
                e.copy_(m)
        return loss

    step.model_ref = model.module if distributed else model
    step.ema_model = ema
    return step


def bench_config(model_name, base_channel, batch, size, lr, total_steps, train_images, val_images, save_dir,
                 device_index=None, teacher_name=None, use_graph=True, dist_backend=None, world=1,
                 dist_world1_bucketer=False):
    """The MyConfig a bench / tool run trains with: reference defaults (adam, CE, OneCycle 'cos_warmup',
    MyConfig augmentation, use_ema False) on a synthetic polyp split of ``train_images``/``val_images``
    images at ``size``, one OneCycle over ``total_steps`` iterations, lr = ``lr`` per GPU
    (reference rule: 0.1 * base_lr * gpu_num)."""
    from ..configs import MyConfig
    cfg = MyConfig()
    cfg.save_dir = save_dir
    cfg.dataset = 'synthetic'
    cfg.synthetic_num = (train_images, max(val_images, 1), 0)
    cfg.synthetic_size = size
    cfg.use_test_set = False
    cfg.crop_size = size
    if model_name in ('ducknet', 'unet'):
        cfg.model, cfg.base_channel = model_name, base_channel
    else:   # smp-<encoder> | smp-<decoder>-<encoder>
        from .trainer_engine import smp_arch
        parts = model_name.split('-')
        cfg.model = 'smp'
        # the reference hub's key of that smp class (models/__init__.py decoder_hub: 'DeepLabV3Plus' ->
        # 'deeplabv3p', 'UnetPlusPlus' -> 'unetpp', else the lower-case name)
        arch = smp_arch(parts[1].lower()).lower() if len(parts) == 3 else 'unet'
        cfg.decoder = {'deeplabv3plus': 'deeplabv3p', 'unetplusplus': 'unetpp'}.get(arch, arch)
        cfg.encoder = parts[-1]
        cfg.encoder_weights = None
    cfg.train_bs = batch
    cfg.base_lr = lr * 10.0
    # one OneCycle over the run: iters_per_epoch as utils.scheduler.get_scheduler derives it (train_num =
    # the split rounded down to whole batches; / world under DDP); a batch larger than the split spans
    # epochs of it (DeviceAugLoader.stream)
    ipe = max(-(-(train_images // batch * batch) // (batch * world)), 1)
    cfg.total_epoch = -(-total_steps // ipe)
    cfg.device_index = device_index
    cfg.dist_backend = dist_backend
    cfg.use_graph = use_graph
    cfg.bucketer_world1 = dist_world1_bucketer
    cfg.graph_warmup = 1
    cfg.use_tb = False
    cfg.progress_bar = False
    cfg.save_ckpt = False
    cfg.load_ckpt = False
    cfg.val_bs = 16
    if teacher_name:
        parts = teacher_name.split('-')
        from .trainer_engine import smp_arch
        cfg.kd_training = True
        cfg.teacher_model = 'smp'
        cfg.teacher_decoder = smp_arch(parts[1]).lower() if len(parts) == 3 else 'unet'
        cfg.teacher_encoder = parts[-1]
        cfg.teacher_ckpt = os.path.join(save_dir, 'teacher_random_init.pth')
    cfg.init_dependent_config()
    return cfg


class TrainerStep:
    """``bench.py``'s fused step IS the trainer's: a real :class:`core.SegTrainer` built from
    :func:`bench_config`, its model wrapped by ``parallel_model`` (FusedModel, SyncBN + RCCL buckets
    under torch.distributed), and every call = one ``SegTrainer.train_step`` on the next batch of the
    trainer's own ``DeviceAugLoader`` (HBM-resident split, MyConfig augmentation on the GPU), written
    straight into the step engine's static graph inputs."""

    def __init__(self, cfg, fixed=False):
        import torch.distributed as dist
        from ..core import SegTrainer
        if cfg.kd_training:   # random-init teacher checkpoint (no weights can be downloaded here)
            rank = dist.get_rank() if dist.is_initialized() else 0
            if rank == 0 and not os.path.isfile(cfg.teacher_ckpt):
                from ..models import decoder_hub
                torch.manual_seed(1)
                t = decoder_hub[cfg.teacher_decoder](encoder_name=cfg.teacher_encoder, encoder_weights=None,
                                                     in_channels=3, classes=cfg.num_class)
                os.makedirs(os.path.dirname(cfg.teacher_ckpt), exist_ok=True)
                tmp = cfg.teacher_ckpt + '.tmp'
                torch.save({'state_dict': t.state_dict()}, tmp)
                os.replace(tmp, cfg.teacher_ckpt)
            if dist.is_initialized():
                dist.barrier()
        self.cfg = cfg
        self.trainer = SegTrainer(cfg)
        self.trainer.parallel_model(cfg)
        self.trainer.config_ref = cfg
        self.trainer.model.train()
        self.loader = self.trainer.train_loader
        # the GPU run draws from the HBM-resident DeviceAugLoader; without a GPU (the CPU rehearsal of the
        # bench contract) the trainer's host DataLoader is cycled epoch after epoch
        self.order = self.loader.stream() if hasattr(self.loader, 'stream') else self._host_batches()
        self.bucketer = getattr(self.trainer.optimizer, 'bucketer', None)
        self.images = self.masks = None
        self.fixed = fixed   # replay the first batch (isolates the model step from the data pipeline)
        self._drawn = False

    def _host_batches(self):
        epoch = 0
        while True:
            if hasattr(self.loader.sampler, 'set_epoch'):
                self.loader.sampler.set_epoch(epoch)
            for images, masks in self.loader:
                yield images, masks
            epoch += 1

    @property
    def ema_model(self):
        return self.trainer.ema_model.ema

    @property
    def engine(self):
        return self.trainer.engine

    def __call__(self):
        if not hasattr(self.loader, 'stream'):   # host loader (CPU rehearsal)
            images, masks = next(self.order)
            dev = self.trainer.device
            return self.trainer.train_step(images.to(dev, torch.float32), masks.to(dev))
        eng = self.trainer.engine
        if eng is not None and eng.images is not None:   # the loader writes into the graph inputs
            out = (eng.images, eng.masks)
        else:
            if self.images is None:
                B, S = self.cfg.train_bs, self.cfg.crop_size
                dev = self.trainer.device
                self.images = torch.empty(B, 3, S, S, device=dev)
                self.masks = torch.empty(B, S, S, dtype=torch.long, device=dev)
            out = (self.images, self.masks)
        if self.fixed and self._drawn:
            images, masks = out
        else:
            images, masks = self.loader.batch(next(self.order), out=out)
            self._drawn = eng is not None and out[0] is eng.images
        return self.trainer.train_step(images, masks)

    def validate(self):
        """The trainer's validation (EMA model, device confusion matrix, reference Dice/IoU) on the
        synthetic val split -> (macro Dice, foreground Dice)."""
        score = self.trainer.validate(self.cfg, self.trainer.val_loader)
        iou_fg = float(self.trainer.last_scores['iou'][-1])   # per-class IoU -> foreground Dice = 2J / (1 + J)
        self.trainer.model.train()
        return float(score), 2 * iou_fg / (1 + iou_fg)


def build_bench_step(impl, batch, size, base_channel, device, channels_last=False,
                     use_graph=True, distributed=False, model_name='ducknet', teacher_name=None, feed=None,
                     total_steps=100000, lr=1e-3):
    if impl == 'eager':
        return build_eager_step(batch, size, base_channel, device, channels_last, distributed, lr=lr,
                                total_steps=total_steps, model_name=model_name, teacher_name=teacher_name, feed=feed)
    from .trainer_engine import build_fused_step
    return build_fused_step(batch=batch, size=size, base_channel=base_channel, device=device,
                            use_graph=use_graph, distributed=distributed, model_name=model_name,
                            teacher_name=teacher_name, feed=feed, total_steps=total_steps, lr=lr)
