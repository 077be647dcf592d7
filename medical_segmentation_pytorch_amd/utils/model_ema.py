"""Weight EMA -- reference ``utils/model_ema.py:12-40`` (ModelEmaV2 with the reference's ramped decay
``clamp(cur_itrs / total_itrs, 0, 1)``; with ``use_ema=False`` the EMA is a per-step copy).

Fast path (fused engine): parameters and float buffers of both models live in flat arenas, so an
update is two ``ema_update`` kernel launches instead of 1733 ``copy_`` launches; the int64
``num_batches_tracked`` counters follow the reference's float-then-truncate arithmetic.
"""
from __future__ import annotations

from copy import deepcopy

import torch
import torch.nn as nn

from .parallel import de_parallel


def get_ema_model(config, model, device):
    return ModelEmaV2(config, model, device=device)


class ModelEmaV2(nn.Module):
    def __init__(self, config, model, device=None, src_arena=None):
        super().__init__()
        self.ema = deepcopy(de_parallel(model))
        self.ema.eval()
        self.device = device
        if self.device is not None:
            self.ema.to(device=device)
        self.use_ema = config.use_ema
        self.total_itrs = config.total_itrs
        self.src_arena = src_arena
        self.ema_arena = None
        self.hyper = None
        if src_arena is not None:
            from ..runtime.engine import Arena
            self.ema_arena = Arena(self.ema, src_arena.data.device, with_grad=False)
            self.hyper = torch.zeros(1, device=src_arena.data.device)

    def _decay(self, cur_itrs):
        return min(max(cur_itrs / self.total_itrs, 0), 1) if self.use_ema else 0.0

    @torch.no_grad()
    def _update(self, model, update_fn):
        for ema_v, model_v in zip(self.ema.state_dict().values(), model.state_dict().values()):
            if self.device is not None:
                model_v = model_v.to(device=self.device)
            ema_v.copy_(update_fn(ema_v, model_v))

    @torch.no_grad()
    def update(self, model, cur_itrs):
        d = self._decay(cur_itrs)
        if self.ema_arena is not None:
            from ..ops._ext import require
            C = require()
            self.hyper.fill_(d)
            C.ema_update(self.ema_arena.data, self.src_arena.data, self.hyper)
            C.ema_update(self.ema_arena.bufdata, self.src_arena.bufdata, self.hyper)
            e, m = self.ema_arena.nbt, self.src_arena.nbt
            if d == 0.0:
                e.copy_(m)
            else:
                e.copy_((d * e + (1.0 - d) * m).long())
            return
        if self.use_ema:
            self._update(de_parallel(model), update_fn=lambda e, m: d * e + (1. - d) * m)
        else:
            self._update(de_parallel(model), update_fn=lambda e, m: m)
