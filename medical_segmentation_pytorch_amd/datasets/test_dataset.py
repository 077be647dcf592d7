"""Inference dataset -- reference ``datasets/test_dataset.py:10-40``: every file of
``test_data_folder`` -> (raw HWC image, Scale(scale)+Normalize tensor, file name)."""
from __future__ import annotations

import os

import numpy as np
from PIL import Image
from torch.utils.data import Dataset

from ..utils.transforms import Scale, normalize_to_tensor


class TestDataset(Dataset):
    def __init__(self, config):
        data_folder = os.path.expanduser(config.test_data_folder)
        if not os.path.isdir(data_folder):
            raise RuntimeError(f'Test image directory: {data_folder} does not exist.')
        self.scale = Scale(scale=config.scale, is_testing=True)
        self.images, self.img_names = [], []
        for file_name in sorted(os.listdir(data_folder)):
            self.images.append(os.path.join(data_folder, file_name))
            self.img_names.append(file_name)

    def __len__(self):
        return len(self.images)

    def __getitem__(self, index):
        image = np.asarray(Image.open(self.images[index]).convert('RGB'))
        image_aug = normalize_to_tensor(self.scale(image=image)['image'])
        return image, image_aug, self.img_names[index]
