"""Multi-process (gloo, world_size=2) tests of the distributed layer, CPU only."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)


def _bucketer_worker(rank, world, port, q, compress=None):
    _init(rank, world, port)
    from medical_segmentation_pytorch_amd.runtime.engine import Arena, GradBucketer
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(300, 200), nn.ReLU(), nn.Linear(200, 100), nn.Linear(100, 7))
    arena = Arena(model, torch.device('cpu'))
    b = GradBucketer(arena, None, bucket_cap_mb=0.1, first_bucket_mb=0.05, compress=compress)
    for i, p in enumerate(arena.params):
        p.grad.fill_(float(rank + 1) * (i + 1))
    # report readiness in backward order, as the fused ops do
    for p in reversed(arena.params):
        b.ready([p])
    b.finish()
    ok = all(torch.allclose(p.grad, torch.full_like(p.grad, 3.0 * (i + 1))) for i, p in enumerate(arena.params))
    q.put((rank, ok, len(b.buckets)))
    dist.destroy_process_group()


@pytest.mark.parametrize('compress', [None, 'bf16'])
def test_grad_bucketer_allreduce(compress):
    """Bucketed all-reduce (SUM) of the grad arena; values 1*(i+1) + 2*(i+1) are exact in bf16 too."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    mp.spawn(_bucketer_worker, args=(2, port, q, compress), nprocs=2, join=True)
    res = [q.get() for _ in range(2)]
    assert all(ok for _, ok, _ in res) and all(nb > 1 for _, _, nb in res)


def _metric_sampler_worker(rank, world, port, q):
    _init(rank, world, port)
    from medical_segmentation_pytorch_amd.utils.metrics import Dice, JaccardIndex
    torch.manual_seed(rank)
    logits = torch.randn(2, 2, 6, 6)
    tgt = torch.randint(0, 2, (2, 6, 6))
    m = JaccardIndex(num_classes=2, ignore_index=255)
    m.update(logits, tgt)
    iou = m.compute()
    d = Dice(num_classes=2)
    d.update(logits, tgt)
    dice = d.compute()
    # sampler sharding: disjoint, covering
    from torch.utils.data.distributed import DistributedSampler
    s = DistributedSampler(list(range(10)), num_replicas=world, rank=rank, shuffle=True, seed=1)
    s.set_epoch(3)
    q.put((rank, iou.tolist(), dice.item(), list(s), logits.tolist(), tgt.tolist()))
    dist.destroy_process_group()


def test_distributed_metrics_and_sampler():
    from medical_segmentation_pytorch_amd.utils.metrics import Dice, JaccardIndex
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    mp.spawn(_metric_sampler_worker, args=(2, _port(), q), nprocs=2, join=True)
    res = sorted([q.get() for _ in range(2)], key=lambda r: r[0])
    m, d = JaccardIndex(num_classes=2, sync=False), Dice(num_classes=2, sync=False)
    for r in res:
        m.update(torch.tensor(r[4]), torch.tensor(r[5]))
        d.update(torch.tensor(r[4]), torch.tensor(r[5]))
    assert torch.allclose(torch.tensor(res[0][1]), m.compute()) and torch.allclose(torch.tensor(res[1][1]), m.compute())
    assert abs(res[0][2] - d.compute().item()) < 1e-6
    a, b = res[0][3], res[1][3]
    assert not set(a) & set(b) and sorted(a + b) == list(range(10))


def _trainer_worker(rank, world, port, root, q):
    _init(rank, world, port)
    from medical_segmentation_pytorch_amd.configs import MyConfig
    from medical_segmentation_pytorch_amd.core import SegTrainer
    c = MyConfig()
    c.model, c.base_channel = 'unet', 8
    c.data_root, c.save_dir = os.path.join(root, 'data'), os.path.join(root, 'save')
    c.synthetic_data, c.synthetic_num, c.synthetic_size = True, (8, 4, 4), 64
    c.crop_size, c.train_bs, c.val_bs, c.base_workers = 64, 2, 1, 0
    c.total_epoch, c.warmup_epochs, c.progress_bar, c.use_test_set = 1, 0, False, False
    c.dist_backend = 'gloo'
    c.init_dependent_config()
    t = SegTrainer(c)
    assert c.DDP and c.gpu_num == 2
    c.destroy_ddp_process = False
    score = t.run(c)
    w = [p.detach().clone() for p in t.model.module.parameters()]
    q.put((rank, float(score), [x.sum().item() for x in w]))
    dist.destroy_process_group()


@pytest.mark.slow
def test_ddp_trainer_gloo(tmp_path):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    mp.spawn(_trainer_worker, args=(2, _port(), str(tmp_path), q), nprocs=2, join=True)
    res = sorted([q.get() for _ in range(2)])
    assert res[0][1] == res[1][1]                      # same all-reduced validation score
    assert all(abs(a - b) < 1e-5 for a, b in zip(res[0][2], res[1][2]))   # replicas stay in sync


@pytest.mark.slow
def test_main_spawns_dataparallel_workers(tmp_path):
    """``python main.py`` without a launcher on an N-device box starts N workers (one per device, torchrun
    environment) with DataParallel's global batch and lr: rehearsed with MSP_SPAWN_PROCS=2 on gloo/CPU."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('LOCAL_RANK', 'RANK', 'WORLD_SIZE')}
    env.update(PYTHONPATH=root, MSP_SPAWN_PROCS='2')
    cmd = [sys.executable, os.path.join(root, 'main.py'), '--dataset', 'synthetic', '--synthetic_num', '8', '4', '4',
           '--synthetic_size', '64', '--crop_size', '64', '--total_epoch', '1', '--warmup_epochs', '0',
           '--train_bs', '2', '--val_bs', '2', '--base_workers', '0', '--model', 'unet', '--base_channel', '8',
           '--no_progress_bar', '--save_dir', str(tmp_path / 'save'), '--data_root', str(tmp_path / 'data'),
           '--engine', 'eager']
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    cfg = json.load(open(tmp_path / 'save' / 'config.json'))
    assert cfg['DDP'] and cfg['gpu_num'] == 2 and cfg['train_bs'] == 2   # per-process 2 -> global 4
    assert cfg['synBN'] is False          # DataParallel: per-replica BatchNorm statistics
    assert abs(cfg['lr'] - cfg['base_lr'] * 0.1 * 2) < 1e-12   # adam: 0.1 * base_lr * gpu_num
    assert os.path.isfile(tmp_path / 'save' / 'last.pth')
