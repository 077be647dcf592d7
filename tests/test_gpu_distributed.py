"""Distributed fused engine on ONE GPU: 2 ranks over gloo (RCCL forbids two ranks per device), both on
cuda:0.  Checks that the SyncBN exchange + bucketed gradient all-reduce of the fused step reproduce a
single-process step on the concatenated batch."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ['ROOT'])
from medical_segmentation_pytorch_amd.models.ducknet import DuckNet
from medical_segmentation_pytorch_amd.runtime.trainer_engine import FusedStep
dist.init_process_group('gloo')
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device('cuda', 0)
torch.manual_seed(0)
model = DuckNet(2, 3, 8).to(dev).train()
g = torch.Generator().manual_seed(1)
x = torch.randn(4, 3, 128, 128, generator=g).to(dev)   # the global batch, same for every world size
y = (torch.rand(4, 128, 128, generator=g) > 0.5).long().to(dev)
if world == 1:
    xs, ys = x, y
else:
    xs, ys = x[2 * rank:2 * rank + 2].contiguous(), y[2 * rank:2 * rank + 2].contiguous()
w0 = torch.cat([p.detach().float().flatten() for p in model.parameters()]).cpu()
step = FusedStep(model, xs, ys, optimizer='sgd', lr=0.05, momentum=0.0, use_graph=False,
                 distributed=world > 1, syncbn=True, bucket_cap_mb=0.5)
step.sched.max_lr = 0.05
loss = step()
torch.cuda.synchronize()
loss = torch.tensor([float(loss)])
dist.all_reduce(loss)                     # mean of the per-rank half-batch losses == full-batch loss
loss = loss / world
if rank == 0:
    w = torch.cat([p.detach().float().flatten() for p in model.parameters()]).cpu() - w0   # the SGD update
    rms = [b.detach().float().cpu() for n, b in model.named_buffers() if 'running_mean' in n]
    torch.save({'w': w, 'rm': torch.cat(rms), 'rms': rms, 'loss': float(loss)}, os.environ['OUT'])
dist.destroy_process_group()
'''


def _run(world, out, tmp):
    s = socket.socket(); s.bind(('127.0.0.1', 0)); port = s.getsockname()[1]; s.close()
    script = tmp / 'w.py'
    script.write_text(WORKER)
    env = dict(os.environ, ROOT=ROOT, OUT=str(out), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={world}',
           '--master-addr', '127.0.0.1', '--master-port', str(port), str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(out, weights_only=True)


def test_syncbn_ddp_matches_single_process(gpu, tmp_path):
    one = _run(1, tmp_path / 'one.pt', tmp_path)
    two = _run(2, tmp_path / 'two.pt', tmp_path)
    # SyncBN => identical batch statistics; averaged grads of two half batches == full-batch grad.
    # The first BN layer sees bit-identical inputs (exact up to fp64 summation order); deeper layers
    # drift by bf16 rounding amplified through ~100 layers at tiny BN batches, while a missing SyncBN /
    # gradient exchange shows up as tens of percent from the FIRST layer on.
    rel = [((a - b).norm() / a.norm().clamp_min(1e-12)).item() for a, b in zip(one['rms'], two['rms'])]
    print('per-layer running_mean rel diff:', ' '.join(f'{r:.1e}' for r in rel))
    # observed: ~1e-7 for the first ~25 layers, growing smoothly to ~1e-1 at the 2x2 bottleneck of a
    # 64x64 input; a missing exchange is ~30 % already at layer 0.
    assert max(rel[:16]) < 1e-5, rel[:16]
    assert max(rel) < 0.25, rel
    wrel = ((one['w'] - two['w']).norm() / one['w'].norm()).item()   # update = -lr * (averaged) grad
    print('update rel diff', wrel, 'loss', one['loss'], two['loss'])
    assert wrel < 0.1, wrel
    assert abs(one['loss'] - two['loss']) < 1e-2 * abs(one['loss']), (one['loss'], two['loss'])
