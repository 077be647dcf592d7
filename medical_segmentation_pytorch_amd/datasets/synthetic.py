"""Synthetic polyp dataset in the reference directory layout (no dataset download is possible):
textured RGB frames with 1-3 elliptical "polyps" (brighter, redder blobs with a soft rim) and the
matching binary masks, written as ``{train,validation,test}/{images,masks}/*.jpg``.
Also used as an in-memory tensor source by ``bench.py``.
"""
from __future__ import annotations

import os

import numpy as np
from PIL import Image


def make_sample(size, rng):
    h = w = size
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    mask = np.zeros((h, w), np.uint8)
    base = np.stack([rng.uniform(120, 180), rng.uniform(60, 100), rng.uniform(50, 90)]).astype(np.float32)
    img = np.ones((h, w, 3), np.float32) * base
    # mucosa texture: a few random low-frequency waves + noise
    for _ in range(4):
        fx, fy, ph = rng.uniform(0.01, 0.08), rng.uniform(0.01, 0.08), rng.uniform(0, 6.28)
        img += rng.uniform(5, 20) * np.sin(fx * xx + fy * yy + ph)[..., None]
    for _ in range(rng.integers(1, 4)):
        cy, cx = rng.uniform(0.2, 0.8) * h, rng.uniform(0.2, 0.8) * w
        ry, rx = rng.uniform(0.06, 0.22) * h, rng.uniform(0.06, 0.22) * w
        th = rng.uniform(0, np.pi)
        dy, dx = yy - cy, xx - cx
        u = (dx * np.cos(th) + dy * np.sin(th)) / rx
        v = (-dx * np.sin(th) + dy * np.cos(th)) / ry
        r = u * u + v * v
        inside = r <= 1.0
        mask[inside] = 1
        shade = np.clip(1.2 - r, 0, 1)[..., None]
        img += shade * np.array([rng.uniform(40, 80), rng.uniform(-10, 20), rng.uniform(-20, 10)], np.float32)
    img += rng.normal(0, 6, img.shape).astype(np.float32)
    return np.clip(img, 0, 255).astype(np.uint8), mask


def make_synthetic_polyp(root, num=(64, 16, 16), size=352, seed=0):
    """Writes the dataset (idempotent: existing complete splits are kept). Returns ``root``."""
    rng = np.random.default_rng(seed)
    for split, n in zip(('train', 'validation', 'test'), num):
        idir = os.path.join(root, split, 'images')
        mdir = os.path.join(root, split, 'masks')
        if os.path.isdir(idir) and len([f for f in os.listdir(idir) if f.endswith('jpg')]) >= n:
            continue
        os.makedirs(idir, exist_ok=True)
        os.makedirs(mdir, exist_ok=True)
        for i in range(n):
            img, msk = make_sample(size, rng)
            Image.fromarray(img).save(os.path.join(idir, f'{split}_{i:05d}.jpg'), quality=95)
            Image.fromarray(msk * 255).save(os.path.join(mdir, f'{split}_{i:05d}.jpg'), quality=100)
    return root


def synthetic_tensors(n, size, seed=0):
    """In-memory (images normalised NCHW float32, masks NHW int64)."""
    import torch
    from ..utils.transforms import normalize_to_tensor
    rng = np.random.default_rng(seed)
    imgs, msks = [], []
    for _ in range(n):
        img, msk = make_sample(size, rng)
        imgs.append(normalize_to_tensor(img))
        msks.append(torch.from_numpy(msk.astype(np.int64)))
    return torch.stack(imgs), torch.stack(msks)
