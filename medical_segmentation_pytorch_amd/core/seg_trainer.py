"""Segmentation trainer -- reference ``core/seg_trainer.py:15-181``.

Hot loop (``train_one_epoch``) keeps the reference's step semantics: zero_grad -> forward (autocast
for the eager engine; the fused engine is bf16 by construction) -> loss (+ KD term) -> backward ->
scaler.step(optimizer) -> scaler.update -> scheduler.step (per iteration) -> EMA update.

MI355X changes:
  * no per-iteration host sync: losses stay on the device and are flushed to TensorBoard / the
    progress bar every ``config.log_interval`` iterations (the reference syncs twice per step);
  * fused engine + static shapes: after ``graph_warmup`` eager iterations the whole step
    (weight repack, forward, loss, backward, all-reduce, optimizer) is captured into ONE hipGraph
    and replayed; the scheduler writes lr/momentum through the optimizer's device hyper tensor;
  * validation metrics accumulate a device confusion matrix (HIP kernel) and all-reduce it once.
"""
from __future__ import annotations

import contextlib
import os
import time

import numpy as np
import torch
from PIL import Image

from ..models import get_teacher_model
from ..ops.bn import flush_pending
from ..runtime.trainer_engine import StepEngine, iteration
from ..utils import FusedModel, de_parallel, get_colormap, get_seg_metrics, sampler_set_epoch
from .base_trainer import BaseTrainer
from ..ops.resample import colorize, resize_bilinear
from ..utils.tracing import trace_range
from ..utils.watchdog import check_finite
from .loss import kd_loss_fn


def _tqdm(it, enable):
    if not enable:
        return it
    try:
        from tqdm import tqdm
        return tqdm(it)
    except Exception:   # pragma: no cover
        return it


class SegTrainer(BaseTrainer):
    def __init__(self, config):
        super().__init__(config)
        if config.is_testing:
            self.colormap = torch.tensor(get_colormap(config)).to(self.device)
        else:
            self.teacher_model = get_teacher_model(config, self.device)
            if self.teacher_model is not None and self.fused:
                from ..runtime.fused_model import supports
                if supports(self.teacher_model):   # KD teacher fwd on the HIP kernels (eval-mode BN)
                    for p in self.teacher_model.parameters():
                        p.requires_grad_(False)
                    self.teacher_model = FusedModel(self.teacher_model).eval()
            self.metrics = [get_seg_metrics(config, m).to(self.device) for m in config.metrics]
        self.engine = None
        self._ema_exec = (None, None)
        self._loss_hist = []
        self.val_history = []

    # ------------------------------------------------------------------------------------------------
    def _accum(self):
        return max(1, int(getattr(self.config_ref, 'accum_steps', 1) or 1))

    def eager_step(self, images, masks):
        """One eager micro-step.  Gradient accumulation (``config.accum_steps`` K): zero_grad on a group's
        first micro-batch, ``loss / K`` back-propagated on each (torch DDP: ``no_sync`` on all but the last),
        ``scaler.step`` / ``update`` on its last; ``self._stepped`` tells the caller."""
        config = self.config_ref
        accum = self._accum()
        micro = getattr(self, '_micro', 0)
        first, last = micro == 0, micro == accum - 1
        self._micro = 0 if last else micro + 1
        self._stepped = last
        if getattr(self, 'channels_last', False) and images.dim() == 4:
            images = images.contiguous(memory_format=torch.channels_last)
        if first:
            self.optimizer.zero_grad()
            ex = getattr(self.model, 'executor', None)
            if ex is not None:   # prepacked conv weights must follow the last optimizer step
                ex.repack()
        amp = config.amp_training and not self.fused and self.device.type == 'cuda'
        dtype = torch.float16 if config.amp_dtype == 'fp16' else torch.bfloat16
        with torch.autocast('cuda', dtype=dtype, enabled=amp):
            preds = self.model(images)
            loss = self.loss_fn(preds, masks)
        if config.kd_training:
            with torch.autocast('cuda', dtype=dtype, enabled=self.device.type == 'cuda'):
                with torch.no_grad():
                    teacher_preds = self.teacher_model(images)
            loss_kd = kd_loss_fn(config, preds.float(), teacher_preds.detach().float())
            loss = loss + config.kd_loss_coefficient * loss_kd
            self._last_kd = loss_kd.detach()
        obj = loss if accum == 1 else loss * (1.0 / accum)
        no_sync = self.model.no_sync() if (not last and hasattr(self.model, 'no_sync')) else contextlib.nullcontext()
        with no_sync:   # torch DDP: the gradient all-reduce only on the group's last micro-batch
            self.scaler.scale(obj).backward()
        flush_pending()
        if last:
            self.scaler.step(self.optimizer)
            self.scaler.update()
        return loss.detach()

    def _use_graph(self, config):
        # every loss (CE, device-side OHEM, BCE+Dice), the KD term and the fused fp16 GradScaler are
        # capture-safe; the eager teacher fallback is not.  A step that issues torch.distributed
        # collectives (gradient buckets, SyncBN over RCCL) is captured too when config.graph_collectives:
        # torch 2.10's process group records captured RCCL calls as graph nodes and keeps their works off
        # its watchdog (round 6: tools/dev/graph_rccl_probe.py, tests/test_gpu_distributed.py).  The
        # bucket rebuild (first step) and every communicator init happen in the eager warm-up steps.
        kd_ok = not config.kd_training or isinstance(self.teacher_model, FusedModel)
        collectives = getattr(self.optimizer, 'bucketer', None) is not None or \
            (config.DDP and config.gpu_num > 1)
        # (RCCL only: gloo collectives run on the host and cannot be captured -- the same-GPU gloo rehearsal)
        nccl = torch.distributed.is_available() and torch.distributed.is_initialized() and \
            torch.distributed.get_backend() == 'nccl'
        coll_ok = not collectives or (getattr(config, 'graph_collectives', True) and nccl)
        return self.fused and config.use_graph and kd_ok and not config.use_aux and coll_ok

    def step_engine(self, config):
        """The fused engine's device step (:class:`runtime.trainer_engine.StepEngine`) -- the same object
        ``bench.py`` times; built on first use, after ``parallel_model`` wrapped the model."""
        if self.engine is None and self.fused and isinstance(self.model, FusedModel):
            kd_fn = (lambda s, t: kd_loss_fn(config, s, t)) if config.kd_training else None
            self.engine = StepEngine(self.model, self.optimizer, self.loss_fn, self.scaler,
                                     teacher=self.teacher_model if config.kd_training else None, kd_fn=kd_fn,
                                     kd_coef=config.kd_loss_coefficient, use_graph=self._use_graph(config),
                                     warmup=config.graph_warmup, accum_steps=getattr(config, 'accum_steps', 1))
            if self.main_rank and self.logger:
                self.logger.info(f'step engine: hipGraph capture {"on" if self.engine.use_graph else "off"} '
                                 f'(world {config.gpu_num if config.DDP else 1}, gradient bucketer '
                                 f'{"on" if getattr(self.optimizer, "bucketer", None) is not None else "off"})')
        return self.engine

    def train_step(self, images, masks):
        """One training iteration (reference core/seg_trainer.py:24-95 body): the device step (fused
        engine: :class:`StepEngine`, hipGraph-replayed; eager engine: autocast + GradScaler), then the
        per-iteration scheduler step and EMA update.  ``train_one_epoch`` and ``bench.py`` call this."""
        config = self.config_ref
        self.train_itrs += 1
        self._last_kd = None
        engine = self.step_engine(config)
        if engine is not None:
            loss = iteration(engine, self.scheduler, self.ema_model, self.train_itrs, images, masks)
            self._last_kd = engine.last_kd.clone() if engine.last_kd is not None else None
            return loss
        loss = self.eager_step(images, masks)
        if self._stepped:   # (gradient accumulation: only after an optimizer step)
            self.scheduler.step()
            self.ema_model.update(self.model, self.train_itrs // self._accum())
        return loss

    def _flush_logs(self, config, pbar=None):
        if not self._loss_hist:
            return
        vals = torch.stack([v for _, v, _ in self._loss_hist]).float().cpu().tolist()
        if config.DDP:
            from ..runtime import comm as ipc_comm
            ipc_comm.check()   # a timed-out peer-memory exchange poisons the step with NaN: name the cause
        check_finite(vals, self._loss_hist[-1][0])
        kds = [k for _, _, k in self._loss_hist]
        kdv = torch.stack(kds).float().cpu().tolist() if all(k is not None for k in kds) else None
        if config.use_tb and self.main_rank and self.writer is not None:
            for (itr, _, _), v in zip(self._loss_hist, vals):
                self.writer.add_scalar('train/loss', v, itr)
            if kdv is not None:
                for (itr, _, _), v, tot in zip(self._loss_hist, kdv, vals):
                    self.writer.add_scalar('train/loss_kd', v, itr)
                    self.writer.add_scalar('train/loss_total', tot, itr)
        if pbar is not None and hasattr(pbar, 'set_description'):
            pbar.set_description(f'Epoch:{self.cur_epoch}/{config.total_epoch}    |Loss:{vals[-1]:4.4g}    |')
        self.last_loss = vals[-1]
        self._loss_hist = []

    def train_one_epoch(self, config):
        self.config_ref = config
        self.model.train()
        sampler_set_epoch(config, self.train_loader, self.cur_epoch)
        pbar = _tqdm(self.train_loader, self.main_rank and config.progress_bar)
        wd = getattr(self, 'watchdog', None)
        for cur_itrs, (images, masks) in enumerate(pbar):
            self.cur_itrs = cur_itrs
            with trace_range('train/h2d'):
                images = images.to(self.device, dtype=torch.float32, non_blocking=True)
                masks = masks.to(self.device, dtype=torch.float32 if config.num_class == 1 else torch.long,
                                 non_blocking=True)
            with trace_range('train/step'):
                loss = self.train_step(images, masks)
            if wd is not None:
                wd.beat()
            self._loss_hist.append((self.train_itrs, loss.clone(), self._last_kd))
            if len(self._loss_hist) >= config.log_interval:
                self._flush_logs(config, pbar)
        self._flush_logs(config, pbar)

    # ------------------------------------------------------------------------------------------------
    def _ema_forward(self, images):
        ema = self.ema_model.ema
        if not self.fused or getattr(self.config_ref, 'val_fp32', False):
            # reference protocol: the EMA model in fp32 without autocast (core/seg_trainer.py:114)
            return ema(images).float()
        owner, ex = self._ema_exec
        if owner is not ema:
            ex = FusedModel(ema).eval()
            self._ema_exec = (ema, ex)
        return ex(images)

    @torch.no_grad()
    def validate(self, config, loader, val_best=False):
        self.config_ref = config
        pbar = _tqdm(loader, self.main_rank and config.progress_bar)
        for images, masks in pbar:
            images = images.to(self.device, dtype=torch.float32)
            _, _, H, W = images.shape
            stride = config.val_img_stride
            resized = H % stride != 0 or W % stride != 0
            if resized:
                images = resize_bilinear(images, (H // stride * stride, W // stride * stride))
            masks = masks.to(self.device, dtype=torch.long)
            with trace_range('val/forward'):
                preds = self._ema_forward(images)
            if resized:
                preds = resize_bilinear(preds, masks.size()[1:], align_corners=True)
            if preds.shape[1] == 1:   # binary (sigmoid) path -> two-class logits for the confmat
                preds = torch.cat([torch.zeros_like(preds), preds], 1)
            for metric in self.metrics:
                metric.update(preds.detach().float(), masks)
        scores = [metric.compute() for metric in self.metrics]
        score = scores[0].mean()
        if self.main_rank and self.logger:
            for i in range(len(config.metrics)):
                if val_best:
                    self.logger.info(f'\n\nTrain {config.total_epoch} epochs finished.' +
                                     f'\n\nBest m{config.metrics[i]} is: {scores[i].mean():.4f}\n')
                else:
                    infos = f' Epoch{self.cur_epoch} m{config.metrics[i]}: {scores[i].mean():.4f} \t| ' + \
                            f'best m{config.metrics[0]} so far: {self.best_score:.4f}\n'
                    if len(config.metrics) > 1 and i != len(config.metrics) - 1:
                        infos = infos[:-1]
                    self.logger.info(infos)
                if config.use_tb and self.writer is not None and self.cur_epoch < config.total_epoch:
                    self.writer.add_scalar(f'val/m{config.metrics[i]}', scores[i].mean().item(), self.cur_epoch + 1)
                    if config.metrics[i] == 'iou':
                        for j in range(scores[i].numel()):
                            self.writer.add_scalar(f'val/IoU_cls{j:02d}', scores[i][j].item(), self.cur_epoch + 1)
        self.last_scores = {m: s.detach().cpu() for m, s in zip(config.metrics, scores)}
        # per-validation record (save_dir/val_history.json, written by BaseTrainer.run): accuracy vs time
        rec = {'epoch': int(self.cur_epoch), 'train_itrs': int(getattr(self, 'train_itrs', 0)),
               'elapsed_s': round(time.perf_counter() - getattr(self, '_t_run', time.perf_counter()), 2),
               'score': float(score), 'val_best': bool(val_best), 'fp32': bool(getattr(config, 'val_fp32', False))}
        for m, v in self.last_scores.items():
            rec[m] = v.tolist()
        self.val_history.append(rec)
        for metric in self.metrics:
            metric.reset()
        return score

    @torch.no_grad()
    def predict(self, config):
        if config.DDP:
            raise ValueError('Predict mode currently does not support DDP.')
        if self.logger:
            self.logger.info('\nStart predicting...\n')
        model = de_parallel(self.model).eval()
        fwd = FusedModel(model).eval() if self.fused else model
        for images, images_aug, img_names in _tqdm(self.test_loader, config.progress_bar):
            images_aug = images_aug.to(self.device, dtype=torch.float32)
            preds = fwd(images_aug)
            preds = colorize(preds, self.colormap).cpu().numpy()
            images = images.cpu().numpy()
            for i in range(preds.shape[0]):
                save_path = os.path.join(config.save_dir, img_names[i])
                suffix = img_names[i].split('.')[-1]
                pred = Image.fromarray(preds[i].astype(np.uint8))
                if config.save_mask:
                    pred.save(save_path)
                if config.blend_prediction:
                    blend_path = save_path.replace(f'.{suffix}', f'_blend.{suffix}')
                    image = Image.fromarray(images[i].astype(np.uint8))
                    if image.size != pred.size:
                        image = image.resize(pred.size, Image.BILINEAR)
                    Image.blend(image, pred, config.blend_alpha).save(blend_path)
