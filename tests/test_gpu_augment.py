"""GPU augmentation over the HBM-resident dataset (csrc/augment.hip) vs the host SegAugment pipeline
evaluated on the SAME random draws (MI355X only)."""
import random
from types import SimpleNamespace

import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu


def _make_split(root, sizes, seed=0):
    rng = np.random.default_rng(seed)
    for split in ('train', 'validation', 'test'):
        for sub in ('images', 'masks'):
            (root / split / sub).mkdir(parents=True, exist_ok=True)
    for i, (h, w) in enumerate(sizes):
        yy, xx = np.mgrid[0:h, 0:w]
        img = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)),
                        rng.integers(0, 256, (h, w))], -1).astype(np.uint8)
        msk = ((((yy - h / 2) / (h / 3)) ** 2 + ((xx - w / 2) / (w / 4)) ** 2) < 1).astype(np.uint8) * 255
        Image.fromarray(img).save(root / 'train' / 'images' / f'{i:03d}.jpg', quality=95)
        Image.fromarray(msk).save(root / 'train' / 'masks' / f'{i:03d}.jpg', quality=95)


@pytest.mark.parametrize('jitter', [False, True])
def test_device_aug_matches_host(gpu, tmp_path, jitter):
    from medical_segmentation_pytorch_amd.datasets.device_loader import DeviceAugLoader, reference_batch
    from medical_segmentation_pytorch_amd.datasets.polyp import PolypDataset
    sizes = [(96, 128), (64, 64), (150, 90), (48, 70), (120, 120), (33, 200)]
    _make_split(tmp_path, sizes)
    cfg = SimpleNamespace(data_root=str(tmp_path), crop_h=64, crop_w=80, randscale=[-0.5, 1.0],
                          brightness=0.5 if jitter else 0.0, contrast=0.5 if jitter else 0.0,
                          saturation=0.5 if jitter else 0.0, h_flip=0.5, v_flip=0.5, num_class=2)
    ds = PolypDataset(cfg, 'train')
    if not jitter:
        ds.transform.jitter = (0.0, 0.0, 0.0, 0.0)
    else:
        ds.transform.jitter_p = 1.0
    loader = DeviceAugLoader(ds, 6, gpu, seed=3)
    aug = ds.transform
    for rep in range(3):
        idx = list(range(len(ds)))
        random.Random(rep).shuffle(idx)
        prms = [aug.sample_params(*loader.data.shapes[i]) for i in idx]
        x, m = loader.batch(idx, prms)
        xr, mr = reference_batch(aug, ds, idx, prms)
        torch.cuda.synchronize()
        assert x.shape == xr.shape and m.shape == mr.shape
        d = (x.cpu() - xr).abs()
        lvl = 1.0 / (0.225 * 255)     # one uint8 level after Normalize
        print(f'rep {rep}: max {d.max().item() / lvl:.2f} levels, mean {d.mean().item() / lvl:.4f}')
        assert d.max().item() < 2.5 * lvl
        assert d.mean().item() < 0.02 * lvl
        assert (m.cpu() != mr).float().mean().item() < 1e-3


def test_device_loader_epoch(gpu, tmp_path):
    from medical_segmentation_pytorch_amd.datasets.device_loader import DeviceAugLoader
    from medical_segmentation_pytorch_amd.datasets.polyp import PolypDataset
    _make_split(tmp_path, [(80, 80)] * 10)
    cfg = SimpleNamespace(data_root=str(tmp_path), crop_h=64, crop_w=64, randscale=[-0.5, 1.0], brightness=0.3,
                          contrast=0.3, saturation=0.3, h_flip=0.5, v_flip=0.5, num_class=2)
    loader = DeviceAugLoader(PolypDataset(cfg, 'train'), 4, gpu, seed=1)
    assert len(loader) == 2
    batches = list(loader)
    assert len(batches) == 2
    for x, m in batches:
        assert x.shape == (4, 3, 64, 64) and m.shape == (4, 64, 64) and x.is_cuda
        assert torch.isfinite(x).all() and set(m.unique().tolist()) <= {0, 1}
