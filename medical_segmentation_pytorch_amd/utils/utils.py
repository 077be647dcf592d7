"""Runtime glue -- reference ``utils/utils.py:5-87``.

loguru / tensorboard are not available in this image, so the logger is stdlib ``logging`` with the
reference's line format (``[YYYY-MM-DD HH:mm] msg``) and the TensorBoard writer is the native event
writer in :mod:`.tb_writer` (same ``add_scalar`` / ``flush`` / ``close`` API).
"""
from __future__ import annotations

import json
import logging
import os
import random
import sys

import numpy as np
import torch


def mkdir(path):
    """Recursive (the reference's ``os.mkdir`` fails for ``save/trial_N`` -- Appendix E.7)."""
    os.makedirs(path, exist_ok=True)


def set_seed(seed):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def get_writer(config, main_rank):
    if config.use_tb and main_rank:
        from .tb_writer import SummaryWriter
        return SummaryWriter(config.tb_log_dir)
    return None


class _Logger:
    """Tiny facade with the loguru calls the trainer uses (``info``/``warning``/``error``)."""

    def __init__(self, name, log_path=None):
        self._log = logging.getLogger(f'medseg.{name}.{id(self)}')
        self._log.setLevel(logging.INFO)
        self._log.propagate = False
        fmt = logging.Formatter('[%(asctime)s] %(message)s', datefmt='%Y-%m-%d %H:%M')
        handlers = [logging.StreamHandler(sys.stderr)]
        if log_path:
            mkdir(os.path.dirname(log_path) or '.')
            handlers.append(logging.FileHandler(log_path))
        for h in handlers:
            h.setFormatter(fmt)
            self._log.addHandler(h)

    def info(self, msg):
        self._log.info(msg)

    def warning(self, msg):
        self._log.warning(msg)

    def error(self, msg):
        self._log.error(msg)

    def close(self):
        for h in list(self._log.handlers):
            h.close()
            self._log.removeHandler(h)


def get_logger(config, main_rank):
    if not main_rank:
        return None
    name = config.logger_name or 'seg_trainer'
    return _Logger(name, f'{config.save_dir}/{name}.log')


def _jsonable(v):
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if isinstance(v, torch.Tensor):
        return v.tolist()
    return str(v)


def save_config(config):
    with open(f'{config.save_dir}/config.json', 'w') as f:
        json.dump({k: _jsonable(v) for k, v in vars(config).items()}, f, indent=4)


LOG_KEYS = ['dataset', 'subset', 'num_class', 'model', 'encoder', 'decoder', 'loss_type',
            'optimizer_type', 'lr_policy', 'total_epoch', 'train_bs', 'val_bs', 'train_num',
            'val_num', 'gpu_num', 'num_workers', 'amp_training', 'DDP', 'kd_training', 'synBN',
            'use_ema', 'engine']


def log_config(config, logger):
    cfg = vars(config)
    body = '\n'.join(f'{k}: {cfg.get(k)}' for k in LOG_KEYS)
    logger.info(f"\n\n\n{'#' * 25} Config Informations {'#' * 25}\n{body}\n{'#' * 71}\n\n")


def get_colormap(config):
    if config.colormap_path is not None and os.path.isfile(config.colormap_path):
        assert config.colormap_path.endswith('json')
        with open(config.colormap_path) as f:
            colormap = {k: tuple(v) for k, v in json.load(f).items()}
    else:
        if config.colormap == 'random':
            colors = np.random.randint(0, 256, size=(config.num_class, 3))
            colormap = {i: tuple(int(c) for c in color) for i, color in enumerate(colors)}
        elif config.colormap == 'custom':
            raise NotImplementedError()
        else:
            raise ValueError(f'Unsupport colormap type: {config.colormap}.')
        mkdir(config.save_dir)
        with open(f'{config.save_dir}/colormap.json', 'w') as f:
            json.dump({k: list(v) for k, v in colormap.items()}, f, indent=1)
    colors = list(colormap.values())
    if len(colors) < config.num_class:
        raise ValueError('Length of colormap is smaller than the number of class.')
    return colors[:config.num_class]
