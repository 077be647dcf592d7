"""LR schedules stepped per iteration -- reference ``utils/scheduler.py:5-26``.

``step`` uses ``config.step_size`` (the reference never defines it; default here: one third of
training) -- SURVEY Appendix E.3.
"""
from math import ceil

from torch.optim.lr_scheduler import OneCycleLR, StepLR


def get_scheduler(config, optimizer):
    if config.DDP:
        config.iters_per_epoch = ceil(config.train_num / config.train_bs / config.gpu_num)
    else:
        config.iters_per_epoch = ceil(config.train_num / config.train_bs)
    config.iters_per_epoch = max(config.iters_per_epoch, 1)
    # the schedule (and the EMA decay ramp) counts OPTIMIZER steps: with gradient accumulation one step takes
    # accum_steps loader iterations (an incomplete group at an epoch end carries into the next epoch)
    accum = max(1, int(getattr(config, 'accum_steps', 1) or 1))
    config.total_itrs = max(int(config.total_epoch * config.iters_per_epoch) // accum, 1)

    if config.lr_policy == 'cos_warmup':
        warmup_ratio = config.warmup_epochs / config.total_epoch
        if not 0 <= warmup_ratio < 1:   # reference crashes here (warmup >= total epochs); torch default
            warmup_ratio = 0.3
        return OneCycleLR(optimizer, max_lr=config.lr, total_steps=config.total_itrs, pct_start=warmup_ratio)
    if config.lr_policy == 'linear':
        return OneCycleLR(optimizer, max_lr=config.lr, total_steps=config.total_itrs, pct_start=0.,
                          anneal_strategy='linear')
    if config.lr_policy == 'step':
        step_size = config.step_size or max(config.total_itrs // 3, 1)
        return StepLR(optimizer, step_size=step_size, gamma=0.1)
    raise NotImplementedError(f'Unsupported scheduler type: {config.lr_policy}')
