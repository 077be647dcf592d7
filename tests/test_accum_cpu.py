"""Gradient accumulation (``config.accum_steps``; runtime/trainer_engine.StepEngine and the eager path of
core/seg_trainer.SegTrainer.eager_step): K micro-batches per optimizer step with DDP averaging semantics.

Oracle: accumulating the SAME micro-batch twice (loss / 2 each) yields exactly the gradient of one step on
it (halving is exact in floating point), so the weights after one optimizer step must equal the accum=1
trainer's; BN running statistics see two updates (per-micro-batch statistics, as torch DDP + no_sync), and
the scheduler / EMA advance once per optimizer step.  Reference step: /root/reference/core/seg_trainer.py:24-95.
"""
import torch

from test_data_train_cpu import _cfg


def _trainer(tmp_path, accum):
    from medical_segmentation_pytorch_amd.core import SegTrainer
    # base_lr / accum: the reference lr rule counts accumulation as replicas (x accum), so both trainers run
    # the same lr and their first optimizer steps are comparable
    c = _cfg(tmp_path / f'a{accum}', model='unet', base_channel=8, total_epoch=8, warmup_epochs=2,
             base_lr=0.01 / accum, accum_steps=accum)
    torch.manual_seed(0)
    t = SegTrainer(c)
    t.parallel_model(c)
    t.config_ref = c
    return t, c


def test_accumulation_matches_single_step(tmp_path):
    t1, c1 = _trainer(tmp_path, 1)
    t2, c2 = _trainer(tmp_path, 2)
    for (k, a), b in zip(t1.model.state_dict().items(), t2.model.state_dict().values()):
        assert torch.equal(a, b), k   # same seed, same init
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 3, 64, 64, generator=g)
    y = (torch.rand(4, 64, 64, generator=g) > 0.5).long()
    lr0 = t2.optimizer.param_groups[0]['lr']
    t1.train_step(x, y)
    t2.train_step(x, y)
    assert not t2._stepped and t2.optimizer.param_groups[0]['lr'] == lr0   # micro-step: no optimizer / schedule
    w_mid = {k: v.clone() for k, v in t2.model.state_dict().items() if 'running' not in k and 'num_batches' not in k}
    t2.train_step(x, y)
    assert t2._stepped
    p1 = dict(t1.model.named_parameters())
    for n, p in t2.model.named_parameters():
        assert torch.allclose(p, p1[n], rtol=1e-5, atol=1e-6), n
        assert not torch.equal(p.detach(), w_mid[n]), n   # the second micro-step DID step the optimizer
    # one scheduler step per optimizer step; total schedule length counts optimizer steps
    assert t1.scheduler.last_epoch == 1 and t2.scheduler.last_epoch == 1
    assert c2.total_itrs == max(c1.total_itrs // 2, 1)
    # BN: two updates of the running statistics with accum 2 (the same batch twice)
    bn1 = [m for m in t1.model.modules() if isinstance(m, torch.nn.BatchNorm2d)][0]
    bn2 = [m for m in t2.model.modules() if isinstance(m, torch.nn.BatchNorm2d)][0]
    assert int(bn2.num_batches_tracked) == 2 * int(bn1.num_batches_tracked) == 2


def test_accumulation_lr_rule_counts_micro_batches():
    from types import SimpleNamespace

    from medical_segmentation_pytorch_amd.utils.optimizer import lr_batch_factor
    c = SimpleNamespace(lr_scale='reference', gpu_num=1, train_bs=320, lr_ref_batch=16, accum_steps=8)
    assert lr_batch_factor(c) == 8.0          # = the 8-GPU run it emulates (reference rule: x replicas)
    c.lr_scale = 'sqrt'
    assert abs(lr_batch_factor(c) - (2560 / 16) ** 0.5) < 1e-9
