"""Trainer lifecycle -- reference ``core/base_trainer.py:14-205``.

Same construction order, run loop, checkpoint dict and auto-resume as the reference:
``{'cur_epoch', 'best_score', 'state_dict', 'optimizer', 'scheduler'}`` (``best.pth`` holds the EMA
weights with optimizer/scheduler ``None``; ``last.pth`` the raw model).  Extra keys (ignored by
reference readers): ``'scaler'``, ``'ema_state_dict'``, ``'rng'``, ``'train_itrs'``.  Checkpoints are
read with ``torch.load(..., weights_only=True)``.

MI355X specifics: ``config.engine`` ('auto' | 'fused' | 'eager') selects the fused HIP executor for
DUCKNet/UNet on a ROCm device; with it the optimizer is :class:`FusedOptimizer` (flat arenas) and
``parallel_model`` returns :class:`FusedModel` (SyncBN + bucketed RCCL all-reduce built in).
Fixed quirks: ``ckpt_name`` works, recursive ``mkdir``.
"""
from __future__ import annotations

import os
import random
import time
from copy import deepcopy

import numpy as np
import torch

from ..datasets import get_loader, get_test_loader
from ..models import get_model
from ..utils import (de_parallel, destroy_ddp_process, get_ema_model, get_logger, get_optimizer, get_scheduler,
                     get_writer, log_config, mkdir, parallel_model, save_config, set_device, set_seed, use_fused)
from ..utils.model_ema import ModelEmaV2
from ..utils.optimizer import FusedGradScaler
from .loss import get_loss_fn


def _compact(sd):
    """state_dict whose tensors own compact storage (params may be views into flat arenas)."""
    return {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in sd.items()}


class BaseTrainer:
    def __init__(self, config):
        self.rank = int(os.getenv('RANK', -1))
        self.local_rank = int(os.getenv('LOCAL_RANK', -1))
        self.world_size = int(os.getenv('WORLD_SIZE', 1))
        config.DDP = self.local_rank != -1
        self.device = set_device(config, self.local_rank)
        # main rank = rank 0 of this run's process group (a trial sub-group in concurrent HPO)
        from ..utils.parallel import group_rank
        self.main_rank = (group_rank(config) == 0) if config.DDP else True
        self.logger = get_logger(config, self.main_rank)
        amp_fp16 = config.amp_training and config.amp_dtype == 'fp16' and self.device.type == 'cuda'
        if self.main_rank:
            mkdir(config.save_dir)
        set_seed(config.random_seed)
        self.model = get_model(config).to(self.device)
        config._fused = use_fused(config, self.model, self.device)
        self.fused = config._fused
        # eager engine on a GPU: channels-last parameters/activations (before the optimizer holds them)
        self.channels_last = (not self.fused and self.device.type == 'cuda'
                              and getattr(config, 'eager_channels_last', False))
        if self.channels_last:
            self.model = self.model.to(memory_format=torch.channels_last)
        # fp16 loss scaling: torch GradScaler on the eager engine; on the fused engine the same semantics
        # with device-side state inside the captured step (the fused kernels compute in bf16, so overflow
        # skips are rare, but the reference's fp16 protocol -- scaled loss, skipped steps -- is kept)
        self.scaler = FusedGradScaler(self.device, enabled=amp_fp16) if self.fused \
            else torch.amp.GradScaler('cuda', enabled=amp_fp16)
        if self.fused and not config.DDP and config.gpu_num > 1:
            # The reference's single-process DP (`train_bs *= gpu_num`, lr * gpu_num;
            # reference utils/parallel.py:26-27,40-42) has no fused equivalent: the fused engine is one
            # process per GPU.  Never train gpu_num x the batch on GPU 0 alone -- undo the scaling.
            if self.main_rank and self.logger:
                self.logger.warning(f'fused engine: {config.gpu_num} GPUs visible but no torchrun; training on '
                                    f'{self.device} only. Launch `torchrun --nproc-per-node {config.gpu_num} '
                                    f'main.py` for data-parallel training on every GPU.')
            config.train_bs //= config.gpu_num
            config.gpu_num = 1
            config.num_workers = config.base_workers
        if self.main_rank and self.logger:
            self.logger.info(f'engine: {"fused MI355X HIP kernels" if self.fused else "eager PyTorch"} '
                             f'on {self.device}')
        self.optimizer = None
        if config.is_testing:
            assert config.load_ckpt, 'Need to load a pretrained checkpoint in `test` mode.'
            self.test_loader = get_test_loader(config)
        else:
            self.writer = get_writer(config, self.main_rank)
            self.loss_fn = get_loss_fn(config, self.device)
            self.train_loader = get_loader(config, self.local_rank, 'train', device=self.device)
            self.val_loader = get_loader(config, self.local_rank, 'val')
            if config.use_test_set:
                self.test_loader = get_loader(config, self.local_rank, 'test')
            self.optimizer = get_optimizer(config, self.model)
            self.scheduler = get_scheduler(config, self.optimizer)
            self.best_score = 0.
            self.cur_epoch = 0
            self.train_itrs = 0
        self.load_ckpt(config)
        if not config.is_testing:
            arena = getattr(self.optimizer, 'arena', None)
            self.ema_model = ModelEmaV2(config, self.model, self.device, src_arena=arena) if arena is not None \
                else get_ema_model(config, self.model, self.device)
            if getattr(self, '_pending_ema', None) is not None:
                self.ema_model.ema.load_state_dict(self._pending_ema)
                self._pending_ema = None

    # ------------------------------------------------------------------------------------------------
    def run(self, config):
        from ..utils.tracing import set_tracing
        from ..utils.watchdog import StepWatchdog
        self.parallel_model(config)
        if self.main_rank:
            save_config(config)
            log_config(config, self.logger)
        set_tracing(getattr(config, 'trace', False))
        self.watchdog = None
        if getattr(config, 'watchdog_timeout_s', 0):
            rank = int(os.getenv('RANK', 0))
            self.watchdog = StepWatchdog(config.watchdog_timeout_s, config.save_dir, rank).start()
        start_epoch = self.cur_epoch
        self._t_run = time.perf_counter()
        for cur_epoch in range(start_epoch, config.total_epoch):
            self.cur_epoch = cur_epoch
            self.train_one_epoch(config)
            if cur_epoch >= config.begin_val_epoch and cur_epoch % config.val_interval == 0:
                val_score = self.validate(config, self.val_loader)
                if self.main_rank and val_score > self.best_score:
                    self.best_score = val_score
                    if config.save_ckpt:
                        self.save_ckpt(config, save_best=True)
            if self.main_rank and config.save_ckpt:
                self.save_ckpt(config)
            if config.DDP and config.save_ckpt:
                # rank 0 alone wrote checkpoints: the others wait here, not inside the next epoch's first
                # collective (a SyncBN exchange would count the skew against its deadline)
                from ..utils.parallel import get_group
                torch.distributed.barrier(group=get_group(config))
        if self.accum_micro() != 0 and self.main_rank and self.logger:
            self.logger.warning(f'training ended inside a gradient-accumulation group ({self.accum_micro()} of '
                                f'{getattr(config, "accum_steps", 1)} micro-batches): their gradients were never '
                                f'applied (make iters_per_epoch * total_epoch a multiple of accum_steps)')
        if config.use_tb and self.main_rank and self.writer is not None:
            self.writer.flush()
            self.writer.close()
        if config.DDP:
            from ..utils.parallel import get_group
            torch.distributed.barrier(group=get_group(config))
        best_score = self.best_score
        if config.save_ckpt:
            best_score = self.val_best(config, self.val_loader)
            if config.use_test_set:
                self.test_score = self.val_best(config, self.test_loader)
        if self.watchdog is not None:
            self.watchdog.stop()
        if self.main_rank:
            self.write_val_history(config, best_score)
        destroy_ddp_process(config)
        return best_score

    def write_val_history(self, config, best_score):
        """save_dir/val_history.json: every validation (epoch, iterations, wall seconds since run start,
        score, per-class metrics) + the val_best score of the best checkpoint."""
        import json
        hist = getattr(self, 'val_history', [])
        out = {'best_score': float(best_score), 'total_epoch': config.total_epoch, 'train_bs': config.train_bs,
               'gpu_num': config.gpu_num, 'iters_per_epoch': getattr(config, 'iters_per_epoch', None),
               'wall_s': round(time.perf_counter() - self._t_run, 2), 'history': hist}
        with open(os.path.join(config.save_dir, 'val_history.json'), 'w') as f:
            json.dump(out, f, indent=1)

    def parallel_model(self, config):
        self.model = parallel_model(config, self.model, self.local_rank, self.device, self.optimizer)

    def accum_micro(self):
        """Micro-batch index inside the current gradient-accumulation group (0: at a group boundary)."""
        eng = getattr(self, 'engine', None)
        return eng.micro if eng is not None else getattr(self, '_micro', 0)

    def train_one_epoch(self, config):
        raise NotImplementedError()

    def validate(self, config, loader, val_best=False):
        raise NotImplementedError()

    def predict(self, config):
        raise NotImplementedError()

    # ------------------------------------------------------------------------------------------------
    def load_ckpt(self, config):
        if config.load_ckpt and config.load_ckpt_path and os.path.isfile(config.load_ckpt_path):
            ckpt = torch.load(config.load_ckpt_path, map_location=self.device, weights_only=True)
            de_parallel(self.model).load_state_dict(ckpt['state_dict'])
            if self.main_rank and self.logger:
                self.logger.info(f'Load model state dict from {config.load_ckpt_path}')
            if not config.is_testing and config.resume_training and ckpt.get('optimizer') is not None:
                self.cur_epoch = ckpt['cur_epoch'] + 1
                self.best_score = ckpt['best_score']
                self.optimizer.load_state_dict(ckpt['optimizer'])
                self.scheduler.load_state_dict(ckpt['scheduler'])
                self.train_itrs = ckpt.get('train_itrs', self.cur_epoch * config.iters_per_epoch)
                if ckpt.get('scaler') is not None:
                    self.scaler.load_state_dict(ckpt['scaler'])
                if hasattr(self.scaler, 'sync_optimizer_step'):   # fused fp16 Adam: restore its device step
                    self.scaler.sync_optimizer_step(self.optimizer)
                self._pending_ema = ckpt.get('ema_state_dict')
                if ckpt.get('accum_micro', 0) and self.main_rank and self.logger:
                    self.logger.warning(f'checkpoint was saved {ckpt["accum_micro"]} micro-batches into a '
                                        f'gradient-accumulation group; that partial group is restarted')
                rng = ckpt.get('rng')
                if rng is not None:
                    torch.set_rng_state(rng['torch'].cpu())
                    keys, pos, has_gauss, gauss = rng['numpy']
                    np.random.set_state(('MT19937', keys.numpy().astype(np.uint32), pos, has_gauss, gauss))
                    random.setstate((rng['python'][1], tuple(rng['python'][0]), None))
                if self.main_rank and self.logger:
                    self.logger.info(f'Resume training from {config.load_ckpt_path}')
            del ckpt
        else:
            if config.is_testing:
                raise ValueError(f'Could not find any pretrained checkpoint at path: {config.load_ckpt_path}.')
            if self.main_rank and self.logger:
                self.logger.info('[!] Train from scratch')

    def save_ckpt(self, config, save_best=False):
        if config.ckpt_name is None:
            save_name = 'best.pth' if save_best else 'last.pth'
        else:
            stem, ext = os.path.splitext(config.ckpt_name)
            save_name = f'{stem}_best{ext or ".pth"}' if save_best else (config.ckpt_name if ext else stem + '.pth')
        save_path = f'{config.save_dir}/{save_name}'
        state_dict = self.ema_model.ema.state_dict() if save_best else de_parallel(self.model).state_dict()
        ckpt = {
            'cur_epoch': self.cur_epoch,
            'best_score': float(self.best_score),
            'state_dict': _compact(state_dict),
            'optimizer': self.optimizer.state_dict() if not save_best else None,
            'scheduler': self.scheduler.state_dict() if not save_best else None,
        }
        if config.ckpt_extra_state and not save_best:
            ckpt['train_itrs'] = self.train_itrs
            # gradient accumulation: the micro-batch index at save time (the partial group's gradients are not
            # saved: a resume restarts that group, and warns)
            ckpt['accum_micro'] = int(self.accum_micro())
            ckpt['scaler'] = self.scaler.state_dict() if self.scaler.is_enabled() else None
            ckpt['ema_state_dict'] = _compact(self.ema_model.ema.state_dict())
            npst = np.random.get_state()
            ckpt['rng'] = {'torch': torch.get_rng_state(),
                           'numpy': [torch.from_numpy(npst[1].astype(np.int64)), int(npst[2]), int(npst[3]),
                                     float(npst[4])],
                           'python': [list(random.getstate()[1]), random.getstate()[0]]}
        if ckpt.get('optimizer') is not None:
            opt = ckpt['optimizer']
            opt['state'] = {k: _compact(v) for k, v in opt['state'].items()}
        torch.save(ckpt, save_path)

    def val_best(self, config, loader, ckpt_path=None):
        ckpt_path = f'{config.save_dir}/best.pth' if ckpt_path is None else ckpt_path
        if not os.path.isfile(ckpt_path):
            raise ValueError(f'Best checkpoint does not exist at {ckpt_path}')
        if self.main_rank and self.logger:
            self.logger.info(f'\nTrain {config.total_epoch} epochs finished!\n')
            self.logger.info(f'{"#" * 50}\nValidation for the best checkpoint...')
        model = de_parallel(self.model)
        ckpt = torch.load(ckpt_path, map_location=self.device, weights_only=True)
        model.load_state_dict(ckpt['state_dict'])
        del ckpt
        self.ema_model.ema = deepcopy(model).eval()
        val_score = self.validate(config, loader, val_best=True)
        if self.main_rank and self.logger:
            self.logger.info(f'Best validation score is {val_score}.\n')
        return val_score
