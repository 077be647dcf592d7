import copy

import torch
import torch.nn as nn

from medical_segmentation_pytorch_amd.configs import MyConfig
from medical_segmentation_pytorch_amd.runtime.engine import OneCycle
from medical_segmentation_pytorch_amd.utils.model_ema import ModelEmaV2
from medical_segmentation_pytorch_amd.utils.scheduler import get_scheduler


def _torch_trace(pct, anneal='cos', steps=50):
    p = nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=0.1)
    s = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=0.1, total_steps=steps, pct_start=pct, anneal_strategy=anneal)
    out = []
    for _ in range(steps):
        g = opt.param_groups[0]
        out.append((g['lr'], g['betas'][0]))
        opt.step()
        s.step()
    return out


def test_onecycle_host_matches_torch():
    for pct, anneal in [(3 / 400, 'cos'), (0.3, 'cos'), (0.0, 'linear')]:
        ref = _torch_trace(pct, anneal)
        oc = OneCycle(0.1, 50, pct, anneal)
        for lr, mom in ref:
            a, b = oc.values()
            assert abs(a - lr) < 1e-9 and abs(b - mom) < 1e-9
            oc.step()


def test_onecycle_reference_shape():
    c = MyConfig().init_dependent_config()
    c.DDP, c.train_num, c.train_bs, c.total_epoch, c.lr = False, 64, 16, 10, 1e-3
    p = nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=c.lr, momentum=0.9)
    s = get_scheduler(c, opt)
    assert c.iters_per_epoch == 4 and c.total_itrs == 40
    lrs = []
    for _ in range(40):
        lrs.append(opt.param_groups[0]['lr'])
        opt.step()
        s.step()
    assert abs(lrs[0] - 1e-3 / 25) < 1e-12 and max(lrs) <= 1e-3 + 1e-12 and lrs[-1] < 1e-6


def test_ema_ramp_and_copy():
    c = MyConfig()
    c.total_itrs, c.use_ema = 10, True
    m = nn.Sequential(nn.Linear(2, 2), nn.BatchNorm1d(2))
    ema = ModelEmaV2(c, m)
    e0 = copy.deepcopy(ema.ema.state_dict())
    with torch.no_grad():
        for p in m.parameters():
            p.add_(1.0)
    ema.update(m, 5)              # decay 0.5
    w = ema.ema.state_dict()['0.weight']
    assert torch.allclose(w, 0.5 * e0['0.weight'] + 0.5 * m.state_dict()['0.weight'])
    c.use_ema = False
    ema2 = ModelEmaV2(c, m)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(1.0)
    ema2.update(m, 5)
    assert torch.equal(ema2.ema.state_dict()['0.weight'], m.state_dict()['0.weight'])
