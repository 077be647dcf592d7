"""Training-step factories used by ``bench.py`` and ``tools/test_speed.py``.

``eager``: stock PyTorch-ROCm step with the reference's exact semantics (DDP + SyncBN + autocast,
per-tensor EMA copy) -- the in-house reference speed.  ``fused``: the MI355X-native engine.
"""
from __future__ import annotations

import math

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
