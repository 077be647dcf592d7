"""HBM-resident training loader with GPU augmentation.

The reference decodes and augments every sample on CPU workers (``datasets/polyp.py:58-71`` with
albumentations, ``datasets/__init__.py:16-44``).  A polyp split is ~1k images (a few hundred MB as
uint8), so here the split is decoded ONCE into one flat uint8 buffer on the GPU; each batch is then
one host-side parameter draw (:meth:`SegAugment.sample_params`, the same random stream the CPU
pipeline consumes) plus a handful of kernel launches (``csrc/augment.hip``): geometry gather
(scale / reflect-pad / crop / flips), ColorJitter stages, normalize.  At 8 x MI355X x ~376 img/s the
CPU path would need ~3k decoded + augmented 352^2 images per second; this path needs none.

Batches come out as (fp32 NCHW images, int64 / fp32 masks) already on the device, in the order of a
``DistributedSampler`` / shuffled ``RandomSampler`` identical to :func:`datasets.get_loader`'s.
"""
from __future__ import annotations

import numpy as np
import torch
from PIL import Image

from ..ops._ext import require
from ..utils.transforms import IMAGENET_MEAN, IMAGENET_STD, SegAugment

_OPS = {'b': 1, 'c': 2, 's': 3, 'h': 4}


def pack_params(prms, indices, n_iparams=14):
    """Per-sample parameter records -> (int32 [B, n_iparams], fp32 [B, 4]) in ``augment.hip`` layout."""
    B = len(prms)
    ip = np.zeros((B, n_iparams), np.int32)
    fp = np.zeros((B, 4), np.float32)
    for i, (p, idx) in enumerate(zip(prms, indices)):
        t, _, l, _ = p['pad']
        ip[i, :10] = (idx, p['nh'], p['nw'], t, l, p['y0'], p['x0'], p['hflip'], p['vflip'], p['jittered'])
        for k, (op, v) in enumerate(p['ops'] if p['jittered'] else []):
            ip[i, 10 + k] = _OPS[op]
            fp[i, k] = v
    return ip, fp


class DeviceDataset:
    """Every (image, mask) of a :class:`PolypDataset` split decoded once into device memory."""

    def __init__(self, dataset, device, arrays=None):
        if arrays is None:
            arrays = ((np.asarray(Image.open(ip).convert('RGB'), dtype=np.uint8),
                       np.asarray(Image.open(mp).convert('1'), dtype=np.uint8))
                      for ip, mp in zip(dataset.images, dataset.masks))
        imgs, msks, meta = [], [], []
        off = moff = 0
        for im, mk in arrays:
            assert im.dtype == np.uint8 and mk.dtype == np.uint8 and im.shape[:2] == mk.shape, (im.shape, mk.shape)
            h, w = mk.shape
            meta.append((off, h, w, moff))
            imgs.append(im.reshape(-1))
            msks.append(mk.reshape(-1))
            off += im.size
            moff += mk.size
        self.shapes = [(m[1], m[2]) for m in meta]
        self.images = torch.from_numpy(np.concatenate(imgs)).to(device)
        self.masks = torch.from_numpy(np.concatenate(msks)).to(device)
        self.meta = torch.tensor(meta, dtype=torch.int64, device=device)
        self.device = device

    @classmethod
    def from_arrays(cls, images, masks, device):
        """From in-memory HWC uint8 images and HW {0,1} uint8 masks (synthetic data, tests)."""
        return cls(None, device, arrays=zip(images, masks))

    def __len__(self):
        return len(self.shapes)

    @property
    def nbytes(self):
        return self.images.numel() + self.masks.numel()


class DeviceAugLoader:
    """Drop-in for the train ``DataLoader``: iterates device batches; ``.sampler`` supports
    ``set_epoch`` (DistributedSampler) exactly like the host loader."""

    def __init__(self, dataset, batch_size, device, sampler=None, shuffle=True, drop_last=True, seed=0,
                 binary_float=False, data=None, aug=None):
        C = require()
        self.dataset = dataset
        self.data = data if data is not None else DeviceDataset(dataset, device)
        self.batch_size = batch_size
        self.sampler = sampler
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.binary_float = binary_float
        self.epoch = 0
        self.seed = seed
        aug = aug if aug is not None else dataset.transform
        assert isinstance(aug, SegAugment), 'DeviceAugLoader needs the train SegAugment pipeline'
        self.aug = aug
        # pinned parameter staging ring: the per-batch H2D copies stay asynchronous (a pageable copy
        # would make the host wait for the GPU before it can draw the next batch)
        self._ring = [None] * 4
        self._ring_ev = [None] * 4
        self._ri = 0
        self.aug.seed(seed)
        ch, cw = aug.crop
        B = batch_size
        self.work = torch.empty(B * ch * cw * 3, dtype=torch.float32, device=device)
        # [B] per-sample gray means + (8-B aligned) the fp64 slice partials of their reduction
        self.mean = torch.empty((B + 1) // 2 * 2 + 2 * C.aug_gray_scratch_doubles(B), dtype=torch.float32,
                                device=device)
        self.norm_mean = [float(v) for v in aug.mean]
        self.norm_std = [float(v) for v in aug.std]
        self.device = device

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.data)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def _order(self):
        if self.sampler is not None:
            return list(iter(self.sampler))
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            self.epoch += 1
            return torch.randperm(len(self.data), generator=g).tolist()
        return list(range(len(self.data)))

    def _stage(self, ip, fp):
        """Device copies of the parameter tables through the pinned ring (async H2D)."""
        if self.device.type != 'cuda':
            return torch.from_numpy(ip).to(self.device), torch.from_numpy(fp).to(self.device)
        i = self._ri
        self._ri = (i + 1) % len(self._ring)
        ev = self._ring_ev[i]
        if ev is not None:
            ev.synchronize()   # that slot's previous copy has been consumed
        slot = self._ring[i]
        if slot is None or slot[0].shape != ip.shape:
            slot = self._ring[i] = (torch.empty(ip.shape, dtype=torch.int32).pin_memory(),
                                    torch.empty(fp.shape, dtype=torch.float32).pin_memory())
        slot[0].numpy()[...] = ip
        slot[1].numpy()[...] = fp
        ip_d = slot[0].to(self.device, non_blocking=True)
        fp_d = slot[1].to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ring_ev[i] = ev
        return ip_d, fp_d

    def batch(self, indices, prms=None, out=None):
        """Augment the samples ``indices`` -> (images [B,3,ch,cw] fp32, masks [B,ch,cw]) on the device.
        ``prms``: pre-drawn parameter records (tests); default = draw from the pipeline's RNG.
        ``out``: optional (images, int64 masks) buffers to write into (static graph inputs)."""
        C = require()
        ch, cw = self.aug.crop
        B = len(indices)
        assert B <= self.batch_size
        if prms is None:
            prms = [self.aug.sample_params(*self.data.shapes[i]) for i in indices]
        ip, fp = pack_params(prms, indices, C.aug_iparams())
        ip_d, fp_d = self._stage(ip, fp)
        stages = [k for k in range(4) if ip[:, 10 + k].any()]
        contrast = [k for k in stages if (ip[:, 10 + k] == _OPS['c']).any()]
        if out is not None:
            out, masks = out
            assert out.shape == (B, 3, ch, cw) and masks.shape == (B, ch, cw) and masks.dtype == torch.int64
        else:
            out = torch.empty(B, 3, ch, cw, dtype=torch.float32, device=self.device)
            masks = torch.empty(B, ch, cw, dtype=torch.int64, device=self.device)
        work = self.work[:B * ch * cw * 3]
        C.aug_batch(self.data.images, self.data.masks, self.data.meta, ip_d, fp_d, work, self.mean, out, masks,
                    stages, contrast, self.norm_mean, self.norm_std)
        return out, (masks.float() if self.binary_float else masks)

    def __iter__(self):
        order = self._order()
        B = self.batch_size
        stop = len(order) - (len(order) % B if self.drop_last else 0)
        for i in range(0, stop, B):
            yield self.batch(order[i:i + B])

    def stream(self):
        """Endless epoch-after-epoch index batches (bench / step-based training).  A batch larger than
        the split spans consecutive epochs (each epoch a fresh permutation) instead of never filling."""
        B = self.batch_size
        if B > len(self.data):
            buf = []
            while True:
                while len(buf) < B:
                    buf.extend(self._order())
                yield buf[:B]
                buf = buf[B:]
        while True:
            order = self._order()
            for i in range(0, len(order) - B + 1, B):
                yield order[i:i + B]


def reference_batch(aug: SegAugment, dataset, indices, prms):
    """CPU oracle: the host pipeline evaluated on the SAME parameter records."""
    imgs, msks = [], []
    it = iter(prms)
    aug.sample_params = lambda h, w: next(it)
    try:
        for i in indices:
            im = np.asarray(Image.open(dataset.images[i]).convert('RGB'))
            mk = np.asarray(Image.open(dataset.masks[i]).convert('1')).astype(np.int64)
            x, y = aug(im, mk)
            imgs.append(x)
            msks.append(y)
    finally:
        del aug.sample_params
    return torch.stack(imgs), torch.stack(msks)


__all__ = ['DeviceAugLoader', 'DeviceDataset', 'pack_params', 'reference_batch', 'IMAGENET_MEAN', 'IMAGENET_STD']
