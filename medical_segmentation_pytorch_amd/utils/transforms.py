"""Data augmentation with the reference's albumentations 1.3.0 semantics (SURVEY Appendix D;
reference ``datasets/polyp.py:37-53``, ``utils/transforms.py:11-32``), implemented natively
(albumentations / OpenCV are not available):

  RandomScale(scale_limit, p=0.5)   factor ~ U[1+lo, 1+hi]; image bilinear, mask nearest
  PadIfNeeded(h, w)                 centred BORDER_REFLECT_101 padding
  RandomCrop(h, w)
  ColorJitter(b, c, s, hue=0.2, p=0.5)  factors ~ U[max(0,1-x), 1+x], random order
  HorizontalFlip(p), VerticalFlip(p)
  Normalize(ImageNet mean/std, max_pixel 255) + ToTensor (HWC -> CHW; mask stays HW)
"""
from __future__ import annotations

import math
import random

import numpy as np
import torch
import torch.nn.functional as F

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def to_numpy(array):
    if not isinstance(array, np.ndarray):
        array = np.asarray(array)
    return array


def resize(img, h, w, mode='bilinear'):
    """HWC uint8/float or HW array -> resized (cv2.INTER_LINEAR / INTER_NEAREST equivalents)."""
    t = torch.from_numpy(np.ascontiguousarray(img))
    squeeze = t.dim() == 2
    if squeeze:
        t = t[..., None]
    x = t.permute(2, 0, 1)[None].float()
    if mode == 'nearest':
        y = F.interpolate(x, size=(h, w), mode='nearest')
    else:
        y = F.interpolate(x, size=(h, w), mode='bilinear', align_corners=False)
    y = y[0].permute(1, 2, 0)
    if img.dtype == np.uint8:
        y = y.round().clamp(0, 255).to(torch.uint8)
    else:
        y = y.to(torch.from_numpy(np.zeros(0, dtype=img.dtype)).dtype)
    y = y.numpy()
    return y[..., 0] if squeeze else y


class Scale:
    """Deterministic resize by ``scale`` (reference utils/transforms.py:11-32)."""

    def __init__(self, scale, interpolation=1, p=1, is_testing=False):
        self.scale, self.interpolation, self.p, self.is_testing = scale, interpolation, p, is_testing

    def __call__(self, image, mask=None):
        img = to_numpy(image)
        h, w = img.shape[:2]
        nh, nw = int(h * self.scale), int(w * self.scale)
        out = {'image': resize(img, nh, nw, 'nearest' if self.interpolation == 0 else 'bilinear')}
        if not self.is_testing and mask is not None:
            out['mask'] = resize(to_numpy(mask), nh, nw, 'nearest')
        return out


def _reflect101_pad(a, top, bottom, left, right):
    pad = [(top, bottom), (left, right)] + [(0, 0)] * (a.ndim - 2)
    return np.pad(a, pad, mode='reflect')   # numpy 'reflect' == OpenCV BORDER_REFLECT_101


def _gray(img):
    return img[..., 0] * 0.299 + img[..., 1] * 0.587 + img[..., 2] * 0.114


def _adjust_hue(img, shift):
    """Hue rotation in HSV space (shift in [-0.5, 0.5] of a full turn); img float RGB 0..255."""
    x = img / 255.0
    r, g, b = x[..., 0], x[..., 1], x[..., 2]
    mx, mn = x.max(-1), x.min(-1)
    d = mx - mn
    h = np.zeros_like(mx)
    m = d > 1e-12
    rc = np.where(m, (mx - r) / np.where(m, d, 1), 0)
    gc = np.where(m, (mx - g) / np.where(m, d, 1), 0)
    bc = np.where(m, (mx - b) / np.where(m, d, 1), 0)
    h = np.where(r == mx, bc - gc, np.where(g == mx, 2.0 + rc - bc, 4.0 + gc - rc))
    h = (h / 6.0) % 1.0
    h = np.where(m, h, 0)
    s = np.where(mx > 1e-12, d / np.where(mx > 1e-12, mx, 1), 0)
    v = mx
    h = (h + shift) % 1.0
    i = np.floor(h * 6.0)
    f = h * 6.0 - i
    p, q, t = v * (1 - s), v * (1 - s * f), v * (1 - s * (1 - f))
    i = i.astype(np.int32) % 6
    out = np.stack([np.choose(i, [v, q, p, p, t, v]), np.choose(i, [t, v, v, q, p, p]),
                    np.choose(i, [p, p, t, v, v, q])], -1)
    return out * 255.0


class SegAugment:
    """Train-time pipeline of the reference (polyp.py:38-47); ``rng`` is a ``random.Random``."""

    def __init__(self, crop_h, crop_w, randscale=0.0, brightness=0.0, contrast=0.0, saturation=0.0, hue=0.2,
                 h_flip=0.0, v_flip=0.0, scale_p=0.5, jitter_p=0.5, mean=IMAGENET_MEAN, std=IMAGENET_STD):
        if isinstance(randscale, (list, tuple)):
            lo, hi = randscale
        else:
            lo, hi = -float(randscale), float(randscale)
        self.scale_range = (1 + lo, 1 + hi)
        self.crop = (crop_h, crop_w)
        self.jitter = (brightness, contrast, saturation, hue)
        self.h_flip, self.v_flip = h_flip, v_flip
        self.scale_p, self.jitter_p = scale_p, jitter_p
        self.mean = np.asarray(mean, np.float32) * 255.0
        self.std = np.asarray(std, np.float32) * 255.0
        self.rng = random.Random()

    def seed(self, s):
        self.rng.seed(s)

    def sample_params(self, h, w):
        """Draw every random number of one sample (same calls, same order as the pixel pipeline), for
        an ``h x w`` source.  The CPU pipeline (:meth:`__call__`) and the GPU one
        (``datasets.device_loader``) both evaluate these records, so a seed gives the same batch."""
        rng = self.rng
        prm = {'nh': h, 'nw': w, 'scaled': False}
        if self.scale_range != (1.0, 1.0) and rng.random() < self.scale_p:
            f = rng.uniform(*self.scale_range)
            prm.update(nh=max(int(round(h * f)), 1), nw=max(int(round(w * f)), 1), scaled=True)
        ch, cw = self.crop
        h2, w2 = prm['nh'], prm['nw']
        ph, pw = max(ch - h2, 0), max(cw - w2, 0)
        prm['pad'] = (ph // 2, ph - ph // 2, pw // 2, pw - pw // 2)
        h2, w2 = h2 + ph, w2 + pw
        prm['y0'] = rng.randint(0, h2 - ch)
        prm['x0'] = rng.randint(0, w2 - cw)
        ops = []
        b, c, s, hue = self.jitter
        jittered = bool(b or c or s or hue) and rng.random() < self.jitter_p
        if jittered:
            if b:
                ops.append(('b', rng.uniform(max(0.0, 1 - b), 1 + b)))
            if c:
                ops.append(('c', rng.uniform(max(0.0, 1 - c), 1 + c)))
            if s:
                ops.append(('s', rng.uniform(max(0.0, 1 - s), 1 + s)))
            if hue:
                ops.append(('h', rng.uniform(-hue, hue)))
            rng.shuffle(ops)
        prm['jittered'], prm['ops'] = jittered, ops
        prm['hflip'] = rng.random() < self.h_flip
        prm['vflip'] = rng.random() < self.v_flip
        return prm

    def __call__(self, image, mask):
        img, msk = to_numpy(image), to_numpy(mask)
        prm = self.sample_params(*img.shape[:2])
        if prm['scaled']:
            img = resize(img, prm['nh'], prm['nw'], 'bilinear')
            msk = resize(msk, prm['nh'], prm['nw'], 'nearest')
        if any(prm['pad']):
            t, bt, l, r = prm['pad']
            img = _reflect101_pad(img, t, bt, l, r)
            msk = _reflect101_pad(msk, t, bt, l, r)
        ch, cw = self.crop
        y0, x0 = prm['y0'], prm['x0']
        img = img[y0:y0 + ch, x0:x0 + cw]
        msk = msk[y0:y0 + ch, x0:x0 + cw]
        img = img.astype(np.float32)
        if prm['jittered']:
            for op, v in prm['ops']:
                if op == 'b':
                    img = np.clip(img * v, 0, 255)
                elif op == 'c':
                    m = _gray(img).mean()
                    img = np.clip((img - m) * v + m, 0, 255)
                elif op == 's':
                    g = _gray(img)[..., None]
                    img = np.clip((img - g) * v + g, 0, 255)
                else:
                    img = np.clip(_adjust_hue(img, v), 0, 255)
            img = np.round(img)
        if prm['hflip']:
            img, msk = img[:, ::-1], msk[:, ::-1]
        if prm['vflip']:
            img, msk = img[::-1], msk[::-1]
        return normalize_to_tensor(img, self.mean, self.std), torch.from_numpy(np.ascontiguousarray(msk)).long()


def normalize_to_tensor(img, mean=None, std=None):
    mean = np.asarray(IMAGENET_MEAN, np.float32) * 255.0 if mean is None else mean
    std = np.asarray(IMAGENET_STD, np.float32) * 255.0 if std is None else std
    x = (np.asarray(img, np.float32) - mean) / std
    return torch.from_numpy(np.ascontiguousarray(x.transpose(2, 0, 1)))
