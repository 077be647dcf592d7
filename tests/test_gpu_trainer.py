"""SegTrainer end-to-end on the fused MI355X engine (hipGraph step, EMA arena, confmat kernel)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(tmp, **kw):
    from medical_segmentation_pytorch_amd.configs import MyConfig
    c = MyConfig()
    c.model, c.base_channel = 'ducknet', 17
    c.data_root, c.save_dir = str(tmp / 'data'), str(tmp / 'save')
    c.synthetic_data, c.synthetic_num, c.synthetic_size = True, (16, 4, 4), 64
    c.crop_size, c.train_bs, c.val_bs, c.base_workers = 64, 4, 2, 0
    c.total_epoch, c.warmup_epochs, c.progress_bar, c.log_interval = 3, 1, False, 3
    c.graph_warmup = 2
    for k, v in kw.items():
        setattr(c, k, v)
    return c.init_dependent_config()


@pytest.mark.parametrize('engine,ema', [('fused', False), ('fused', True), ('eager', False)])
def test_trainer_runs(gpu, tmp_path, engine, ema):
    from medical_segmentation_pytorch_amd.core import SegTrainer
    c = _cfg(tmp_path, engine=engine, use_ema=ema)
    t = SegTrainer(c)
    assert t.fused == (engine == 'fused')
    score = t.run(c)
    assert 0.0 <= float(score) <= 1.0
    assert torch.isfinite(torch.tensor(t.last_loss))
    if engine == 'fused':
        assert t.engine is not None and t.engine.graph is not None   # hipGraph path really ran
    ck = torch.load(os.path.join(c.save_dir, 'last.pth'), weights_only=True)
    assert len(ck['state_dict']) == 1733
    # resume works on the fused optimizer (state_dict in torch's format)
    assert 'exp_avg' in next(iter(ck['optimizer']['state'].values()))


def test_fused_optimizer_matches_torch_adam(gpu):
    import torch.nn as nn
    from medical_segmentation_pytorch_amd.utils.optimizer import FusedOptimizer
    torch.manual_seed(0)
    m1 = nn.Sequential(nn.Linear(64, 32), nn.Linear(32, 8)).to(gpu)
    m2 = nn.Sequential(nn.Linear(64, 32), nn.Linear(32, 8)).to(gpu)
    m2.load_state_dict(m1.state_dict())
    o1 = FusedOptimizer(m1, 'adam', lr=1e-2)
    o2 = torch.optim.Adam(m2.parameters(), lr=1e-2)
    s1 = torch.optim.lr_scheduler.OneCycleLR(o1, 1e-2, total_steps=10)
    s2 = torch.optim.lr_scheduler.OneCycleLR(o2, 1e-2, total_steps=10)
    for _ in range(5):
        x = torch.randn(4, 64, device=gpu)
        for m, o, s in ((m1, o1, s1), (m2, o2, s2)):
            o.zero_grad()
            m(x).pow(2).mean().backward()
            o.step()
            s.step()
    for p, q in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize('mode', ['ohem', 'kd'])
def test_trainer_graph_with_ohem_and_kd(gpu, tmp_path, mode):
    """OHEM (device-side selection) and KD (frozen fused teacher) steps run inside the hipGraph."""
    from medical_segmentation_pytorch_amd.core import SegTrainer
    kw = {'loss_type': 'ohem'} if mode == 'ohem' else {}
    if mode == 'kd':
        from medical_segmentation_pytorch_amd.models.smp import Unet
        teacher = Unet(encoder_name='resnet18', encoder_weights=None, in_channels=3, classes=2)
        ck = tmp_path / 'teacher.pth'
        torch.save({'state_dict': teacher.state_dict()}, ck)
        kw = dict(kd_training=True, teacher_ckpt=str(ck), teacher_model='smp', teacher_encoder='resnet18',
                  teacher_decoder='unet')
    c = _cfg(tmp_path, engine='fused', **kw)
    t = SegTrainer(c)
    t.run(c)
    assert t.engine is not None and t.engine.graph is not None
    assert torch.isfinite(torch.tensor(t.last_loss))


def test_fused_grad_scaler_matches_torch(gpu):
    """FusedGradScaler + FusedOptimizer == torch GradScaler + Adam: same unscaled updates, the step is
    skipped on an inf gradient (params, moments and Adam's step count untouched) and the scale backs
    off / grows exactly as torch's ``_amp_update_scale_``."""
    import torch.nn as nn
    from medical_segmentation_pytorch_amd.utils.optimizer import FusedGradScaler, FusedOptimizer
    torch.manual_seed(0)
    m1 = nn.Sequential(nn.Linear(64, 32), nn.Linear(32, 8)).to(gpu)
    m2 = nn.Sequential(nn.Linear(64, 32), nn.Linear(32, 8)).to(gpu)
    m2.load_state_dict(m1.state_dict())
    o1 = FusedOptimizer(m1, 'adam', lr=1e-2)
    o2 = torch.optim.Adam(m2.parameters(), lr=1e-2)
    sc1 = FusedGradScaler(gpu, init_scale=1024.0, growth_interval=3)
    sc2 = torch.amp.GradScaler('cuda', init_scale=1024.0, growth_interval=3)
    for it in range(8):
        x = torch.randn(4, 64, device=gpu)
        for m, o, sc in ((m1, o1, sc1), (m2, o2, sc2)):
            o.zero_grad()
            loss = m(x).pow(2).mean()
            sc.scale(loss).backward()
            if it == 4:   # poison one gradient: this step must be skipped
                next(m.parameters()).grad.view(-1)[3] = float('inf')
            sc.step(o)
            sc.update()
        assert sc1.get_scale() == sc2.get_scale(), (it, sc1.get_scale(), sc2.get_scale())
        for p, q in zip(m1.parameters(), m2.parameters()):
            assert torch.allclose(p, q, atol=1e-5, rtol=1e-4), it
    st = o1.state_dict()['state']
    assert float(next(iter(st.values()))['step']) == 7.0   # 8 steps, one skipped
    assert sc1.state_dict()['_growth_tracker'] == sc2.state_dict()['_growth_tracker']


def test_fused_fp16_adam_resume_continues_step(gpu):
    """Resume with fp16 loss scaling: the fused Adam takes its bias-correction step from the scaler's
    device count; after optimizer + scaler state_dict round trips (what a checkpoint resume does) the
    next updates equal those of the uninterrupted run (not restarted at t = 1)."""
    import torch.nn as nn
    from medical_segmentation_pytorch_amd.utils.optimizer import FusedGradScaler, FusedOptimizer
    torch.manual_seed(0)
    ma = nn.Sequential(nn.Linear(32, 16), nn.Linear(16, 4)).to(gpu)
    mb = nn.Sequential(nn.Linear(32, 16), nn.Linear(16, 4)).to(gpu)
    mb.load_state_dict(ma.state_dict())
    oa, sa = FusedOptimizer(ma, 'adam', lr=1e-2), FusedGradScaler(gpu, init_scale=256.0)
    xs = [torch.randn(4, 32, device=gpu) for _ in range(10)]

    def step(m, o, sc, x):
        o.zero_grad()
        sc.scale(m(x).pow(2).mean()).backward()
        sc.step(o)
        sc.update()

    for x in xs[:5]:
        step(ma, oa, sa, x)
    # "checkpoint" after 5 steps, resume into fresh objects
    osd, ssd = oa.state_dict(), sa.state_dict()
    mb.load_state_dict(ma.state_dict())
    ob, sb = FusedOptimizer(mb, 'adam', lr=1e-2), FusedGradScaler(gpu, init_scale=1.0)
    ob.load_state_dict(osd)
    sb.load_state_dict(ssd)
    sb.sync_optimizer_step(ob)
    for x in xs[5:]:
        step(ma, oa, sa, x)
        step(mb, ob, sb, x)
    for p, q in zip(ma.parameters(), mb.parameters()):
        assert torch.allclose(p, q, atol=1e-6, rtol=1e-5)


def test_trainer_fp16_amp_graph(gpu, tmp_path):
    """amp_dtype='fp16' on the fused engine keeps the hipGraph (loss scaling on device state)."""
    from medical_segmentation_pytorch_amd.core import SegTrainer
    from medical_segmentation_pytorch_amd.utils.optimizer import FusedGradScaler
    c = _cfg(tmp_path, engine='fused', amp_training=True, amp_dtype='fp16')
    t = SegTrainer(c)
    assert isinstance(t.scaler, FusedGradScaler) and t.scaler.is_enabled()
    t.run(c)
    assert t.engine is not None and t.engine.graph is not None
    assert torch.isfinite(torch.tensor(t.last_loss))
    assert t.scaler.get_scale() == 2.0 ** 16   # no overflow in a few bf16-computed steps
    ck = torch.load(os.path.join(c.save_dir, 'last.pth'), weights_only=True)
    assert ck['scaler']['scale'] == 2.0 ** 16


def test_bench_step_is_the_trainer_step(gpu, tmp_path):
    """bench.py's timed step is SegTrainer.train_step: one StepEngine (hipGraph-captured) driven by a real
    trainer over its own DeviceAugLoader, with the trainer's scheduler and EMA -- and it trains."""
    from medical_segmentation_pytorch_amd.runtime.bench_step import TrainerStep, bench_config
    from medical_segmentation_pytorch_amd.runtime.trainer_engine import StepEngine
    cfg = bench_config('ducknet', 8, 4, 64, 1e-3, 12, 16, 4, str(tmp_path / 'b'), device_index=0)
    step = TrainerStep(cfg)
    losses = [float(step()) for _ in range(10)]
    tr = step.trainer
    assert isinstance(tr.engine, StepEngine) and tr.engine.graph is not None
    assert step.engine is tr.engine and tr.train_itrs == 10
    assert tr.scheduler.last_epoch == 10                      # the trainer's own OneCycleLR stepped per iteration
    assert all(l == l for l in losses) and min(losses[5:]) < losses[0]
    dice, fg = step.validate()
    assert 0.0 <= dice <= 1.0 and 0.0 <= fg <= 1.0
