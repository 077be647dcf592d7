"""Polyp segmentation datasets (Kvasir-SEG, CVC-ClinicDB, CVC-ColonDB, ETIS) -- reference
``datasets/polyp.py:9-71``: ``data_root/{train,validation,test}/{images,masks}``, only ``*jpg``
images, mask with the same file name, PIL RGB image, mask ``convert('1')`` -> {0, 1}.
Train: the native augmentation pipeline (:class:`SegAugment`); val/test: Normalize only.
"""
from __future__ import annotations

import os

import numpy as np
from PIL import Image
from torch.utils.data import Dataset

from ..utils.transforms import SegAugment, normalize_to_tensor


class PolypDataset(Dataset):
    def __init__(self, config, mode='train'):
        assert mode in ['train', 'val', 'test']
        mode_folder = mode if mode in ['train', 'test'] else 'validation'
        data_root = os.path.expanduser(config.data_root)
        data_folder = os.path.join(data_root, mode_folder)
        img_dir = os.path.join(data_folder, 'images')
        msk_dir = os.path.join(data_folder, 'masks')
        if not os.path.isdir(img_dir):
            raise RuntimeError(f'Image directory does not exist: {img_dir}\n')
        if not os.path.isdir(msk_dir):
            raise RuntimeError(f'Mask directory does not exist: {msk_dir}\n')
        self.images, self.masks = [], []
        for file_name in sorted(os.listdir(img_dir)):
            if file_name.endswith('jpg'):
                img_path = os.path.join(img_dir, file_name)
                msk_path = os.path.join(msk_dir, file_name)
                if not os.path.isfile(msk_path):
                    raise RuntimeError(f'Mask file: {msk_path} not found.\n')
                self.images.append(img_path)
                self.masks.append(msk_path)
        self.mode = mode
        self.binary_float = config.num_class == 1
        if mode == 'train':
            self.transform = SegAugment(config.crop_h, config.crop_w, config.randscale, config.brightness,
                                        config.contrast, config.saturation, h_flip=config.h_flip,
                                        v_flip=config.v_flip)
        else:
            self.transform = None

    def __len__(self):
        return len(self.images)

    def __getitem__(self, index):
        image = np.asarray(Image.open(self.images[index]).convert('RGB'))
        mask = np.asarray(Image.open(self.masks[index]).convert('1')).astype(np.int64)
        if self.transform is not None:
            image, mask = self.transform(image, mask)
        else:
            import torch
            image, mask = normalize_to_tensor(image), torch.from_numpy(mask)
        return image, mask


def seed_worker(worker_id):
    """DataLoader worker init: decorrelate augmentation RNG streams (the reference seeds nothing)."""
    import torch
    info = torch.utils.data.get_worker_info()
    seed = (torch.initial_seed() + worker_id) % 2 ** 32
    ds = info.dataset
    if getattr(ds, 'transform', None) is not None and hasattr(ds.transform, 'seed'):
        ds.transform.seed(seed)
    np.random.seed(seed % 2 ** 32)
