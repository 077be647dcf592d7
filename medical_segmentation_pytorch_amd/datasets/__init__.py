"""Datasets and loaders -- reference ``datasets/__init__.py:7-59``.

Differences: the DistributedSampler uses the GLOBAL rank (the reference passes
LOCAL_RANK, i.e. single-node only); ``dataset='synthetic'`` (or ``synthetic_data=True`` with a
missing ``data_root``) generates a polyp-like set in the reference layout first.
"""
from __future__ import annotations

import os

import torch.distributed as dist
from torch.utils.data import DataLoader

from .polyp import PolypDataset, seed_worker
from .synthetic import make_synthetic_polyp, synthetic_tensors  # noqa: F401

dataset_hub = {'polyp': PolypDataset, 'synthetic': PolypDataset}


def _ensure_data(config):
    # Only rank 0 looks at the file system; every rank takes the barrier.  (A slower rank that
    # decided by itself would see the directory rank 0 is still writing, skip the barrier and read a
    # half-written split.)
    if getattr(config, '_synthetic_ready', False) or not (config.dataset == 'synthetic' or config.synthetic_data):
        return
    root = config.data_root if config.data_root and config.data_root != '/path/to/your/dataset' \
        else os.path.join(config.save_dir, 'synthetic_polyp')
    from ..utils.parallel import get_group, group_rank
    if group_rank(config) == 0 and (config.dataset == 'synthetic' or not os.path.isdir(str(config.data_root))):
        make_synthetic_polyp(root, config.synthetic_num, config.synthetic_size, config.random_seed)
    if get_group(config) is not None:
        dist.barrier(group=get_group(config))
    config.data_root = root
    config._synthetic_ready = True


def get_dataset(config, mode):
    _ensure_data(config)
    if config.dataset in dataset_hub:
        return dataset_hub[config.dataset](config=config, mode=mode)
    raise NotImplementedError('Unsupported dataset!')


def _device_loader_ok(config, mode, dataset, device):
    if mode != 'train' or not getattr(config, 'gpu_augment', False) or device is None or device.type != 'cuda':
        return False
    from ..ops import _ext
    from ..utils.transforms import SegAugment
    return _ext.available() and isinstance(getattr(dataset, 'transform', None), SegAugment)


def get_loader(config, rank, mode, pin_memory=True, drop_last=True, device=None):
    """Host ``DataLoader`` (reference semantics), or -- train split on a GPU with ``gpu_augment`` --
    the HBM-resident :class:`DeviceAugLoader` (same sampler order, same augmentation draws)."""
    dataset = get_dataset(config, mode)
    if mode == 'train':
        config.train_num = int(len(dataset) // config.train_bs * config.train_bs)
    elif mode == 'val':
        config.val_num = len(dataset)
    elif mode == 'test':
        config.test_num = len(dataset)
    shuffle = mode == 'train'
    bs = config.train_bs if mode == 'train' else config.val_bs
    workers = config.num_workers
    common = dict(num_workers=workers, worker_init_fn=seed_worker, persistent_workers=workers > 0)
    if _device_loader_ok(config, mode, dataset, device):
        from .device_loader import DeviceAugLoader
        sampler = None
        grank = 0
        if config.DDP:
            from torch.utils.data.distributed import DistributedSampler
            from ..utils.parallel import group_rank
            grank = group_rank(config) if dist.is_initialized() else max(rank, 0)
            sampler = DistributedSampler(dataset, num_replicas=config.gpu_num, rank=grank, shuffle=True,
                                         seed=config.random_seed)
        return DeviceAugLoader(dataset, bs, device, sampler=sampler, shuffle=True, drop_last=drop_last,
                               seed=config.random_seed + grank, binary_float=config.num_class == 1)
    if config.DDP:
        from torch.utils.data.distributed import DistributedSampler
        from ..utils.parallel import group_rank
        grank = group_rank(config) if dist.is_initialized() else max(rank, 0)
        sampler = DistributedSampler(dataset, num_replicas=config.gpu_num, rank=grank, shuffle=shuffle,
                                     seed=config.random_seed)
        return DataLoader(dataset, batch_size=bs, shuffle=False, pin_memory=pin_memory, sampler=sampler,
                          drop_last=drop_last and mode == 'train', **common)
    return DataLoader(dataset, batch_size=bs, shuffle=shuffle, pin_memory=pin_memory,
                      drop_last=drop_last and mode == 'train', **common)


def get_test_loader(config):
    from .test_dataset import TestDataset
    dataset = TestDataset(config)
    config.test_num = len(dataset)
    if config.DDP:
        raise NotImplementedError('predict mode does not support DDP (reference datasets/__init__.py:54)')
    return DataLoader(dataset, batch_size=config.test_bs, shuffle=False, num_workers=config.num_workers)
