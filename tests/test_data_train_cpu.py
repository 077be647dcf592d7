import os

import numpy as np
import pytest
import torch

from medical_segmentation_pytorch_amd.configs import MyConfig, load_parser
from medical_segmentation_pytorch_amd.datasets import get_loader, make_synthetic_polyp
from medical_segmentation_pytorch_amd.datasets.polyp import PolypDataset
from medical_segmentation_pytorch_amd.utils.transforms import SegAugment, Scale, _reflect101_pad


def test_reflect101_matches_opencv_semantics():
    a = np.arange(5)[None].repeat(2, 0)
    p = _reflect101_pad(a, 0, 0, 2, 2)
    assert p[0].tolist() == [2, 1, 0, 1, 2, 3, 4, 3, 2]


def test_augment_shapes_and_determinism():
    img = (np.random.RandomState(0).rand(40, 50, 3) * 255).astype(np.uint8)
    msk = (np.random.RandomState(1).rand(40, 50) > 0.5).astype(np.int64)
    aug = SegAugment(64, 64, [-0.5, 1.0], 0.5, 0.5, 0.5, h_flip=0.5, v_flip=0.5)
    aug.seed(3)
    x1, y1 = aug(img, msk)
    aug.seed(3)
    x2, y2 = aug(img, msk)
    assert x1.shape == (3, 64, 64) and y1.shape == (64, 64) and y1.dtype == torch.long
    assert torch.equal(x1, x2) and torch.equal(y1, y2)
    assert set(y1.unique().tolist()) <= {0, 1}


def test_scale():
    out = Scale(0.5, is_testing=True)(image=np.zeros((40, 60, 3), np.uint8))
    assert out['image'].shape == (20, 30, 3)


def _cfg(tmp, **kw):
    c = MyConfig()
    c.data_root = str(tmp / 'data')
    c.save_dir = str(tmp / 'save')
    c.crop_size = 64
    c.train_bs, c.val_bs = 4, 2
    c.base_workers = 0
    c.synthetic_data, c.synthetic_num, c.synthetic_size = True, (8, 4, 4), 64
    c.progress_bar = False
    for k, v in kw.items():
        setattr(c, k, v)
    c.init_dependent_config()
    c.DDP, c.gpu_num, c.num_workers = False, 1, 0
    return c


def test_synthetic_dataset_and_loader(tmp_path):
    c = _cfg(tmp_path)
    make_synthetic_polyp(c.data_root, (8, 4, 4), 64)
    ds = PolypDataset(c, 'val')
    x, y = ds[0]
    assert x.shape == (3, 64, 64) and y.shape == (64, 64) and set(y.unique().tolist()) <= {0, 1}
    ld = get_loader(c, -1, 'train')
    assert c.train_num == 8
    xb, yb = next(iter(ld))
    assert xb.shape == (4, 3, 64, 64)


@pytest.mark.slow
def test_train_resume_predict_cpu(tmp_path):
    """BASELINE config #1 plumbing: UNet on 64x64 synthetic polyps, CPU; interrupted run, auto-resume,
    best/last checkpoints, then predict."""
    from medical_segmentation_pytorch_amd.core import SegTrainer
    mk = lambda **kw: _cfg(tmp_path, model='unet', base_channel=8, total_epoch=2, warmup_epochs=1,  # noqa: E731
                           base_lr=0.01, **kw)
    c = mk()
    t = SegTrainer(c)
    t.parallel_model(c)
    t.cur_epoch = 0
    t.train_one_epoch(c)
    t.save_ckpt(c)                                  # "crash" after epoch 0
    ck = torch.load(os.path.join(c.save_dir, 'last.pth'), weights_only=True)
    assert set(['cur_epoch', 'best_score', 'state_dict', 'optimizer', 'scheduler']) <= set(ck)
    assert ck['cur_epoch'] == 0 and ck['train_itrs'] == 2
    c2 = mk()
    t2 = SegTrainer(c2)                             # auto-resume from save_dir/last.pth
    assert t2.cur_epoch == 1 and t2.train_itrs == 2
    for k, v in ck['state_dict'].items():
        assert torch.equal(t2.model.state_dict()[k], v), k
    score = t2.run(c2)
    assert 0.0 <= float(score) <= 1.0
    for f in ('best.pth', 'last.pth', 'config.json'):
        assert os.path.isfile(os.path.join(c.save_dir, f))
    assert torch.load(os.path.join(c.save_dir, 'best.pth'), weights_only=True)['optimizer'] is None
    assert torch.load(os.path.join(c.save_dir, 'last.pth'), weights_only=True)['cur_epoch'] == 1
    c3 = mk(is_testing=True, test_data_folder=os.path.join(c.data_root, 'test', 'images'))
    c3.load_ckpt_path = os.path.join(c.save_dir, 'best.pth')
    c3.save_dir = str(tmp_path / 'pred')
    os.makedirs(c3.save_dir, exist_ok=True)
    c3.test_bs = 1
    t3 = SegTrainer(c3)
    t3.predict(c3)
    assert any(o.endswith('_blend.jpg') for o in os.listdir(c3.save_dir))
