"""Multi-process (gloo, world_size 2, 4 and 8 -- the 8-GPU node's rank count) tests of the distributed layer, CPU only."""
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
    tot = world * (world + 1) / 2
    ok = all(torch.allclose(p.grad, torch.full_like(p.grad, tot * (i + 1))) for i, p in enumerate(arena.params))
    q.put((rank, ok, len(b.buckets)))
    dist.destroy_process_group()


def _rebuild_worker(rank, world, port, q, compress=None):
    """Gradients land in a scrambled (non-registration) order; step 1 uses the initial reverse-registration
    buckets, then the bucketer re-buckets along the observed order; step 2 must still sum exactly and every
    bucket must launch right when its last gradient lands (never deferred to finish())."""
    _init(rank, world, port)
    import random
    from medical_segmentation_pytorch_amd.runtime.engine import Arena, GradBucketer
    torch.manual_seed(0)
    model = nn.Sequential(*[nn.Linear(64, 64) for _ in range(6)])
    arena = Arena(model, torch.device('cpu'))
    b = GradBucketer(arena, None, bucket_cap_mb=0.03, first_bucket_mb=0.02, compress=compress)
    n = len(arena.params)
    order = list(range(n))
    random.Random(5).shuffle(order)   # same on every rank (as the executor's backward order is)
    before = [list(bk.members) for bk in b.buckets]
    res = []
    for step in range(2):
        for i, p in enumerate(arena.params):
            p.grad.fill_(float(rank + 1) * (i + 1) + step)
        launched_at = []
        for k, i in enumerate(order):
            b.ready([arena.params[i]])
            launched_at.append(len(b.launch_order))
        late = [lt for _, lt in b.launch_order]
        b.finish()
        ok = all(torch.allclose(p.grad, torch.full_like(p.grad, 3.0 * (i + 1) + 2 * step))
                 for i, p in enumerate(arena.params))
        res.append((ok, any(late)))
    q.put((rank, res, before, [list(bk.members) for bk in b.buckets], order, b.bucket_order(),
           [bk.span is None for bk in b.buckets]))
    dist.destroy_process_group()


@pytest.mark.parametrize('compress', [None, 'bf16'])
def test_grad_bucketer_rebuilds_in_ready_order(compress):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    mp.spawn(_rebuild_worker, args=(2, _port(), q, compress), nprocs=2, join=True)
    for rank, res, before, after, order, border, packed in [q.get() for _ in range(2)]:
        assert all(ok for ok, _ in res), res
        assert before != after and len(after) > 1
        assert border == order                     # buckets follow the observed grad-ready order
        assert res[1][1] is False                  # after the rebuild no bucket waits for finish()
        assert any(packed)                         # scrambled order: some buckets go through the staging buffer


@pytest.mark.parametrize('world', [2, 4, 8])
@pytest.mark.parametrize('compress', [None, 'bf16'])
def test_grad_bucketer_allreduce(compress, world):
    """Bucketed all-reduce (SUM) of the grad arena; values sum_r (r+1)*(i+1) are exact in bf16 too."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    mp.spawn(_bucketer_worker, args=(world, port, q, compress), nprocs=world, join=True)
    res = [q.get() for _ in range(world)]
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
    s = DistributedSampler(list(range(24)), num_replicas=world, rank=rank, shuffle=True, seed=1)
    s.set_epoch(3)
    q.put((rank, iou.tolist(), dice.item(), list(s), logits.tolist(), tgt.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4, 8])
def test_distributed_metrics_and_sampler(world):
    """One confusion-matrix all-reduce gives every rank the pooled (exact) IoU / Dice; the sampler's shards
    are disjoint and cover the set (reference utils/parallel.py + torchmetrics sync)."""
    from medical_segmentation_pytorch_amd.utils.metrics import Dice, JaccardIndex
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    mp.spawn(_metric_sampler_worker, args=(world, _port(), q), nprocs=world, join=True)
    res = sorted([q.get() for _ in range(world)], key=lambda r: r[0])
    m, d = JaccardIndex(num_classes=2, sync=False), Dice(num_classes=2, sync=False)
    for r in res:
        m.update(torch.tensor(r[4]), torch.tensor(r[5]))
        d.update(torch.tensor(r[4]), torch.tensor(r[5]))
    for r in res:
        assert torch.equal(torch.tensor(r[1]), m.compute())    # exact: integer confusion-matrix counts
        assert abs(r[2] - d.compute().item()) < 1e-6
    shards = [set(r[3]) for r in res]
    assert sum(len(s) for s in shards) == len(set().union(*shards))   # disjoint
    assert set().union(*shards) == set(range(24))                      # covering


def _full_batch_worker(rank, world, port, q):
    """DDP semantics at world ``world``: every rank back-propagates the mean loss of ITS shard into the grad
    arena, the bucketer sums the ranks' gradients and the optimizer's 1/world makes it the mean -- which must
    equal one process's gradient of the mean loss over the whole batch.  Same for SyncBN statistics: every
    rank parks its (sum, sum^2) row in the exchange queue (ops.bn._Pending), one all-reduce, and the
    finalized mean / biased variance must equal the full batch's."""
    _init(rank, world, port)
    try:
        from medical_segmentation_pytorch_amd.ops import bn
        from medical_segmentation_pytorch_amd.runtime.engine import Arena, GradBucketer
        torch.manual_seed(0)
        model = nn.Sequential(nn.Linear(24, 48), nn.Tanh(), nn.Linear(48, 5))
        arena = Arena(model, torch.device('cpu'))
        b = GradBucketer(arena, None, bucket_cap_mb=0.002, first_bucket_mb=0.001)
        g = torch.Generator().manual_seed(3)
        x, y = torch.randn(8 * world, 24, generator=g), torch.randn(8 * world, 5, generator=g)
        ref = nn.Sequential(nn.Linear(24, 48), nn.Tanh(), nn.Linear(48, 5))
        ref.load_state_dict(model.state_dict())
        ((ref(x) - y) ** 2).mean().backward()                       # the single-process full batch
        xs, ys = x[rank::world], y[rank::world]
        arena.grad.zero_()
        ((model(xs) - ys) ** 2).mean().backward()
        for p in reversed(list(model.parameters())):
            b.ready([p])
        b.finish()
        ok_grad = all(torch.allclose(p.grad / world, r.grad, rtol=1e-5, atol=1e-7)
                      for p, r in zip(model.parameters(), ref.parameters()))
        feats = torch.randn(6 * world, 7, generator=g) * 3 + 1
        mine = feats[rank::world]
        row = torch.cat([mine.sum(0), (mine * mine).sum(0)]).double().view(1, -1)
        out = {}
        bn._FWD.add(row, dist.group.WORLD, lambda s: out.__setitem__('s', s.clone()), 12345)
        bn.need_stats_all()
        s = out['s'].view(2, 7)
        n = feats.shape[0]
        mean, var = s[0] / n, s[1] / n - (s[0] / n) ** 2
        ok_bn = torch.allclose(mean.float(), feats.mean(0), atol=1e-5) and \
            torch.allclose(var.float(), feats.var(0, unbiased=False), atol=1e-4)
        q.put((rank, ok_grad, ok_bn, len(b.buckets)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [4, 8])
def test_bucketed_ddp_step_and_syncbn_equal_full_batch(world):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    mp.spawn(_full_batch_worker, args=(world, _port(), q), nprocs=world, join=True)
    res = [q.get() for _ in range(world)]
    assert all(ok_g for _, ok_g, _, _ in res), res
    assert all(ok_b for _, _, ok_b, _ in res), res
    assert all(nb > 1 for *_, nb in res)


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


@pytest.mark.slow
def test_bench_self_launches_ranks(tmp_path):
    """``python bench.py --gpus 2`` WITHOUT torchrun starts 2 ranks itself (before any GPU call) and the
    JSON line is the 2-rank job's: n_gpus 2, dp2, the evidence pass sees a 2-rank process group.  Without a
    GPU the contract runs on the CPU over gloo."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('LOCAL_RANK', 'RANK', 'WORLD_SIZE', 'MASTER_PORT')}
    env.update(OMP_NUM_THREADS='2', BENCH_SAVE_DIR=str(tmp_path / 'save'))
    cmd = [sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '2', '--warmup', '1',
           '--batch', '2', '--size', '64', '--model', 'unet', '--base-channel', '8', '--train-images', '8',
           '--val-images', '2', '--comm-steps', '1']
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['config']['parallelism'] == 'dp2' and d['config']['global_batch'] == 4
    assert d['comm']['world_size'] == 2 and d['value'] > 0


def test_bench_refuses_mismatched_world(tmp_path):
    """A rank whose process group does not have --gpus ranks exits non-zero instead of benching a
    different job size."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1',
               MASTER_PORT=str(_port()))
    cmd = [sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '1', '--warmup', '0']
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and 'job has 1 rank' in out.stderr, out.stderr[-2000:]


def test_spawn_ranks_tears_down_on_failure(tmp_path):
    """The launcher-less supervisor (bench / main.py DP mode) stops the surviving ranks as soon as one rank
    fails instead of waiting on rank 0 forever (torchrun semantics)."""
    import time
    from medical_segmentation_pytorch_amd.utils.launch import spawn_ranks
    script = tmp_path / 'r.py'
    script.write_text('import os, sys, time\n'
                      'if os.environ["RANK"] == "1":\n    sys.exit(7)\n'
                      'time.sleep(120)\n')
    t0 = time.monotonic()
    rc = spawn_ranks(3, [str(script)], grace_s=5.0)
    assert rc == 7 and time.monotonic() - t0 < 60
