"""Optimizers -- reference ``utils/optimizer.py:4-21`` (same lr scaling rules).

Eager engine: ``torch.optim.{SGD, Adam, AdamW}``.  Fused MI355X engine: :class:`FusedOptimizer`,
a real ``torch.optim.Optimizer`` (so ``OneCycleLR`` drives its param_groups and its
``state_dict`` has torch's format: 'momentum_buffer' / 'exp_avg' / 'exp_avg_sq' / 'step') whose
parameters, gradients and states are views into flat arenas; ``step`` is ONE HIP kernel launch.
"""
from __future__ import annotations

import torch
from torch.optim import SGD, Adam, AdamW


class FusedOptimizer(torch.optim.Optimizer):
    def __init__(self, model, kind='adam', lr=1e-3, momentum=0.9, weight_decay=0.0, betas=(0.9, 0.999), eps=1e-8,
                 device=None):
        from ..runtime.engine import Arena
        device = device or next(model.parameters()).device
        self.kind = kind
        self.arena = Arena(model, device)
        params = self.arena.params
        if kind == 'sgd':
            defaults = dict(lr=lr, momentum=momentum, dampening=0, weight_decay=weight_decay, nesterov=False,
                            maximize=False, foreach=None, differentiable=False, fused=None)
        else:
            defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                            foreach=None, capturable=False, differentiable=False, fused=None)
            if kind == 'adamw' and weight_decay == 0.0:
                defaults['weight_decay'] = 1e-2     # torch.optim.AdamW default
        super().__init__(params, defaults)
        n = self.arena.numel
        if kind == 'sgd':
            self.buf = torch.zeros(n, device=device)
        else:
            self.m = torch.zeros(n, device=device)
            self.v = torch.zeros(n, device=device)
        for i, p in enumerate(params):
            o, k = self.arena.offsets[i], p.numel()
            if kind == 'sgd':
                self.state[p] = {'momentum_buffer': self.buf[o:o + k].view_as(p)}
            else:
                self.state[p] = {'step': torch.tensor(0.0), 'exp_avg': self.m[o:o + k].view_as(p),
                                 'exp_avg_sq': self.v[o:o + k].view_as(p)}
        self.step_count = 0
        from ..runtime.engine import StagedScalars
        self.staged = StagedScalars(8, device)
        self.hyper = self.staged.dev
        self.bucketer = None
        self.grad_scale = 1.0

    def attach_bucketer(self, bucketer):
        self.bucketer = bucketer
        self.grad_scale = 1.0 / bucketer.world

    def zero_grad(self, set_to_none: bool = True):
        self.arena.grad.zero_()

    def prepare(self):
        """Write this step's hyper-parameters to the device (host work, outside any hipGraph)."""
        self.step_count += 1
        g = self.param_groups[0]
        h = self.staged.host()
        if self.kind == 'sgd':
            h[0], h[1], h[2], h[3] = g['lr'], g['momentum'], g['weight_decay'], self.grad_scale
        else:
            b1, b2 = g['betas']
            h[0], h[1], h[2], h[3], h[4] = g['lr'], b1, b2, g['eps'], g['weight_decay']
            h[5] = 1 - b1 ** self.step_count
            h[6] = 1 - b2 ** self.step_count
            h[7] = self.grad_scale
        self.staged.push()

    def launch(self, scaler=None):
        """Device work of a step (capturable): all-reduce wait + one optimizer kernel.  ``scaler``: a
        :class:`FusedGradScaler` -- finite check of the reduced gradients, then an update that unscales
        or is skipped entirely on inf/NaN (one more launch, no host sync)."""
        from ..ops._ext import require
        C = require()
        if self.bucketer is not None:
            self.bucketer.finish()
        a = self.arena
        amp = None
        if scaler is not None and scaler.is_enabled():
            C.amp_check(a.grad, scaler.state)
            amp = scaler.state
            self._amp = scaler.state
        if self.kind == 'sgd':
            C.sgd_step(a.data, a.grad, self.buf, self.hyper, amp)
        else:
            C.adam_step(a.data, a.grad, self.m, self.v, self.hyper, self.kind == 'adamw', amp)

    @torch.no_grad()
    def step(self, closure=None, scaler=None):
        loss = closure() if closure is not None else None
        self.prepare()
        self.launch(scaler)
        return loss

    def state_dict(self):
        if self.kind != 'sgd':
            amp = getattr(self, '_amp', None)   # fp16 loss scaling: skipped steps do not count
            n = float(amp[3]) if amp is not None else float(self.step_count)
            for p in self.arena.params:
                self.state[p]['step'] = torch.tensor(n)
        return super().state_dict()

    def load_state_dict(self, state_dict):
        groups = state_dict['param_groups']
        for g, sg in zip(self.param_groups, groups):
            for k, v in sg.items():
                if k != 'params':
                    g[k] = v
        params = self.arena.params
        for idx, st in state_dict['state'].items():
            p = params[int(idx)]
            for k, v in st.items():
                if k == 'step':
                    self.step_count = int(float(v))
                    if 'step' in self.state[p]:
                        self.state[p]['step'] = torch.tensor(float(v))
                elif k in self.state[p] and v is not None:
                    self.state[p][k].copy_(v)


class FusedGradScaler:
    """``torch.amp.GradScaler`` for the fused engine (reference ``core/base_trainer.py:30``,
    ``core/seg_trainer.py:82-84``) with its state on the DEVICE -- ``[scale, growth_tracker, found_inf,
    applied_steps]`` -- so a captured hipGraph step scales the loss, checks the reduced gradients,
    unscales inside the optimizer kernel, skips the update on overflow and adjusts the scale
    (``csrc/optim.hip`` amp_check / amp_update) without a host round-trip."""

    def __init__(self, device, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True):
        self._enabled = enabled
        self.growth_factor, self.backoff_factor, self.growth_interval = growth_factor, backoff_factor, growth_interval
        self.state = torch.tensor([init_scale, 0.0, 0.0, 0.0], dtype=torch.float32, device=device)

    def is_enabled(self):
        return self._enabled

    def scale(self, loss):
        return loss * self.state[0] if self._enabled else loss

    def step(self, optimizer):
        if isinstance(optimizer, FusedOptimizer):
            return optimizer.step(scaler=self if self._enabled else None)
        raise TypeError('FusedGradScaler drives FusedOptimizer only')

    def update(self):
        if self._enabled:
            from ..ops._ext import require
            require().amp_update(self.state, self.growth_factor, self.backoff_factor, self.growth_interval)

    def get_scale(self):
        return float(self.state[0]) if self._enabled else 1.0

    def state_dict(self):
        if not self._enabled:
            return {}
        st = self.state.tolist()
        return {'scale': st[0], 'growth_factor': self.growth_factor, 'backoff_factor': self.backoff_factor,
                'growth_interval': self.growth_interval, '_growth_tracker': int(st[1])}

    def load_state_dict(self, sd):
        if not sd:
            return
        self.growth_factor = sd.get('growth_factor', self.growth_factor)
        self.backoff_factor = sd.get('backoff_factor', self.backoff_factor)
        self.growth_interval = sd.get('growth_interval', self.growth_interval)
        self.state[0] = float(sd['scale'])
        self.state[1] = float(sd.get('_growth_tracker', 0))

    def sync_optimizer_step(self, optimizer):
        """After a resume: the fused Adam kernels take the bias-correction step from the scaler's device
        count (state[3], applied = non-skipped updates), which the checkpoint stores as the optimizer's
        'step' -- write it back so the next update continues the interrupted run's t, not t = 1."""
        if self._enabled and isinstance(optimizer, FusedOptimizer):
            self.state[3] = float(optimizer.step_count)


def lr_batch_factor(config):
    """Large-batch learning-rate scaling on top of the reference rule.

    ``config.lr_scale`` = ``'reference'`` (default; reference ``utils/optimizer.py:9,15``: x gpu_num, the
    per-GPU batch is fixed at MyConfig's 16), ``'sqrt'`` (x sqrt(global batch / lr_ref_batch)) or
    ``'linear'`` (x global batch / lr_ref_batch).  The global batch is train_bs x gpu_num x accum_steps;
    lr_ref_batch (16) is the batch the reference's base_lr was tuned for.  With Adam the square-root rule is
    the stable one (the update is scale-free, so its noise falls as 1/sqrt(batch)); warm-up comes from the
    OneCycle schedule's warmup_epochs.  Gradient accumulation counts as replicas for the reference rule
    (x gpu_num x accum_steps): one GPU accumulating 8 micro-batches takes the lr of the 8-GPU run it emulates."""
    rule = getattr(config, 'lr_scale', 'reference') or 'reference'
    accum = max(1, int(getattr(config, 'accum_steps', 1) or 1))
    if rule == 'reference':
        return float(config.gpu_num * accum)
    ratio = config.train_bs * config.gpu_num * accum / float(getattr(config, 'lr_ref_batch', 16) or 16)
    if rule == 'sqrt':
        return ratio ** 0.5
    if rule == 'linear':
        return ratio
    raise ValueError(f"lr_scale must be 'reference', 'sqrt' or 'linear', got {rule!r}")


def get_optimizer(config, model):
    fused = getattr(config, '_fused', False)
    if config.optimizer_type == 'sgd':
        config.lr = config.base_lr * lr_batch_factor(config)
        if fused:
            return FusedOptimizer(model, 'sgd', lr=config.lr, momentum=config.momentum,
                                  weight_decay=config.weight_decay)
        return SGD(model.parameters(), lr=config.lr, momentum=config.momentum, weight_decay=config.weight_decay)
    if config.optimizer_type in ['adam', 'adamw']:
        config.lr = 0.1 * config.base_lr * lr_batch_factor(config)
        if fused:
            return FusedOptimizer(model, config.optimizer_type, lr=config.lr)
        cls = Adam if config.optimizer_type == 'adam' else AdamW
        return cls(model.parameters(), lr=config.lr)
    raise NotImplementedError(f'Unsupported optimizer type: {config.optimizer_type}')
