"""Process-group, device and model-parallel wrappers -- reference ``utils/parallel.py:7-54``.

* ``set_device``: torchrun env -> one process per GPU, process group on RCCL (backend ``nccl``) for
  GPUs or ``gloo`` on CPU; ``config.gpu_num`` = world size.  The reference's single-process DP path
  (``nn.DataParallel``) is kept for API parity, but on CPU it no longer zeroes the batch size
  (``train_bs *= device_count()`` with 0 devices).
* ``parallel_model``: fused engine -> :class:`FusedModel` (HIP executor + SyncBN over RCCL + the
  flat-arena gradient bucketer); eager engine -> SyncBatchNorm conversion + torch DDP (or DP).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
import torch.nn as nn
from torch.nn.parallel import DistributedDataParallel as DDP


class FusedModel(nn.Module):
    """Wraps a DuckNet/UNet so forward runs on the MI355X fused executor (training and eval).
    ``.module`` is the reference-shaped model (state_dict keys unchanged)."""

    def __init__(self, module, group=None, sinks=None, ready_hook=None, count_nbt=True):
        super().__init__()
        from ..runtime.fused_model import FusedExecutor
        self.module = module
        self.executor = FusedExecutor(module, group=group, sinks=sinks, count_nbt=count_nbt,
                                      ready_hook=ready_hook)

    def forward(self, x, is_training=None):
        if is_training:
            raise ValueError('auxiliary heads are not supported by the native models')
        return self.executor(x, training=self.training)


def get_group(config=None):
    """Process group of this run: ``config.dist_group`` (a trial sub-group for concurrent HPO) or WORLD."""
    g = getattr(config, 'dist_group', None) if config is not None else None
    if g is not None:
        return g
    return dist.group.WORLD if dist.is_available() and dist.is_initialized() else None


def group_size(config=None):
    g = get_group(config)
    return dist.get_world_size(g) if g is not None else 1


def group_rank(config=None):
    g = get_group(config)
    return dist.get_rank(g) if g is not None else 0


def is_parallel(model):
    return isinstance(model, (nn.parallel.DataParallel, nn.parallel.DistributedDataParallel, FusedModel))


def de_parallel(model):
    return model.module if is_parallel(model) else model


def set_device(config, rank):
    if config.DDP:
        use_gpu = torch.cuda.is_available()
        if getattr(config, 'device_index', None) is not None:
            rank = config.device_index   # every rank on one device (gloo rehearsal of the N-rank path)
        if use_gpu:
            torch.cuda.set_device(rank)
        if not dist.is_initialized():
            backend = config.dist_backend or ('nccl' if use_gpu else 'gloo')
            kw = {'device_id': torch.device('cuda', rank)} if (use_gpu and backend == 'nccl') else {}
            from .watchdog import process_group_timeout
            timeout = process_group_timeout(config)
            if timeout is not None:
                kw['timeout'] = timeout
            dist.init_process_group(backend=backend, init_method='env://', **kw)
        device = torch.device('cuda', rank) if use_gpu else torch.device('cpu')
        config.gpu_num = group_size(config)
    elif getattr(config, 'device_index', None) is not None:
        # one explicit device, no DataParallel batch scaling (bench.py; tests)
        device = torch.device('cuda', config.device_index) if torch.cuda.is_available() else torch.device('cpu')
        if device.type == 'cuda':
            torch.cuda.set_device(device)
        config.gpu_num = 1
    else:
        device = torch.device('cuda' if torch.cuda.is_available() else 'cpu')
        config.gpu_num = max(torch.cuda.device_count(), 1)
        config.train_bs *= config.gpu_num
    config.num_workers = min(config.gpu_num * config.base_workers, max(os.cpu_count() or 1, 1)) \
        if config.cap_workers else config.gpu_num * config.base_workers
    return device


def use_fused(config, model, device) -> bool:
    from ..ops import _ext
    from ..runtime.fused_model import supports
    if config.engine == 'eager' or device.type != 'cuda':
        return False
    if _ext.stale():
        # engine='auto' must not fall back to the slow eager path silently on a GPU because the build is
        # out of date: a benchmark or a training run would quietly switch engines
        _ext.require()
    ok = supports(model) and _ext.available()
    if config.engine == 'fused' and not ok:
        _ext.require()
        raise NotImplementedError(f'fused engine does not support {type(model).__name__}')
    return ok


def parallel_model(config, model, rank, device, optimizer=None):
    if getattr(config, '_fused', False):
        group = get_group(config) if config.DDP else None
        arena = getattr(optimizer, 'arena', None)
        bucketer = None
        if group is not None and arena is not None and (dist.get_world_size(group) > 1 or
                                                        getattr(config, 'bucketer_world1', False)):
            from ..runtime.engine import GradBucketer
            bucketer = GradBucketer(arena, group, config.bucket_cap_mb,
                                    compress=getattr(config, 'grad_compress', None))
            optimizer.attach_bucketer(bucketer)
        from ..runtime import comm as ipc_comm
        from ..runtime.engine import stat_group
        ipc_comm.POLICY['mode'] = os.environ.get('MSP_SYNCBN_COMM', getattr(config, 'syncbn_comm', 'rccl'))
        ipc_comm.POLICY['timeout_s'] = ipc_comm.default_timeout_s(config)
        from ..runtime.fused_model import eager_parts
        if group is not None and config.synBN:
            # modules that run eagerly inside the fused model (smp decoders over a fused encoder): torch
            # SyncBatchNorm on the same group (parameters / buffers are kept, so arena views survive)
            for name in eager_parts(model):
                setattr(model, name, nn.SyncBatchNorm.convert_sync_batchnorm(getattr(model, name), group))
        return FusedModel(model, group=stat_group(group) if config.synBN else None,
                          sinks=arena.sinks() if arena is not None else None,
                          ready_hook=bucketer.ready if bucketer is not None else None,
                          count_nbt=arena is None)   # with an arena: one counter add per step (StepEngine)
    if config.DDP:
        if config.synBN and device.type == 'cuda':
            model = nn.SyncBatchNorm.convert_sync_batchnorm(model)
        pg = get_group(config)
        if device.type == 'cuda':
            model = DDP(model.to(device), device_ids=[rank], output_device=rank,
                        bucket_cap_mb=config.bucket_cap_mb, process_group=pg)
        else:
            model = DDP(model, process_group=pg)
        if getattr(config, 'grad_compress', None) == 'bf16':
            from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
            model.register_comm_hook(pg, default_hooks.bf16_compress_hook)
    elif device.type == 'cuda' and torch.cuda.device_count() > 1:
        model = nn.DataParallel(model)
        model.to(device)
    return model


def destroy_ddp_process(config):
    if config.DDP and config.destroy_ddp_process and dist.is_initialized() and \
            getattr(config, 'dist_group', None) is None:
        dist.destroy_process_group()


def sampler_set_epoch(config, loader, cur_epochs):
    if config.DDP and hasattr(loader.sampler, 'set_epoch'):
        loader.sampler.set_epoch(cur_epochs)
