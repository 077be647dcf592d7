"""IPC peer-memory all-reduce (``csrc/comm.hip``, ``runtime/comm.py``): two processes on the ONE GPU of the
box map each other's exchange buffers and reduce through the one-shot kernel.  Results must equal the
gloo all-reduce of the same rows BITWISE (two ranks: one fp64 addition, same order), across many epochs
(parity-slot reuse), sizes up to the capacity, and when the exchange is captured in a hipGraph and
replayed (the epoch counter lives on the device)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, time, json, torch, torch.distributed as dist
sys.path.insert(0, os.environ['ROOT'])
from medical_segmentation_pytorch_amd.runtime import comm
dist.init_process_group('gloo')
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
comm.POLICY['mode'] = 'ipc'
c = comm.attach(dist.group.WORLD, dev)
assert c is not None
res = {'self_test': True, 'mismatch': 0, 'checked': 0}
g = torch.Generator().manual_seed(100 + rank)
for it in range(300):
    n = [1, 7, 1088, 4099, c.cap][it % 5]
    x = torch.randn(n, generator=g, dtype=torch.float64) * 10 ** (it % 7 - 3)
    ref = x.clone()
    dist.all_reduce(ref)                       # gloo, CPU
    buf = x.to(dev)
    c.all_reduce(buf)
    res['mismatch'] += int(not torch.equal(buf.cpu(), ref))
    res['checked'] += 1
# hipGraph: capture one exchange, replay with fresh inputs
buf = torch.zeros(2 * 544, dtype=torch.float64, device=dev)
src = torch.zeros_like(buf)
torch.cuda.synchronize()
dist.barrier()
graph = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    buf.copy_(src)
    c.all_reduce(buf)   # warm-up outside the capture (both ranks run it)
torch.cuda.synchronize()
dist.barrier()
with torch.cuda.graph(graph):
    buf.copy_(src)
    c.all_reduce(buf)
gmis = 0
for it in range(20):
    v = torch.randn(buf.numel(), generator=g, dtype=torch.float64)
    ref = v.clone()
    dist.all_reduce(ref)
    src.copy_(v.to(dev))
    torch.cuda.synchronize()
    dist.barrier()
    graph.replay()
    torch.cuda.synchronize()
    gmis += int(not torch.equal(buf.cpu(), ref))
res['graph_mismatch'] = gmis
# latency: back-to-back exchanges of one DUCK level's rows (2 x 544 fp64 per BN, 6 BNs)
row = torch.randn(6 * 2 * 544, dtype=torch.float64, device=dev)
torch.cuda.synchronize(); dist.barrier()
for _ in range(20):
    c.all_reduce(row)
torch.cuda.synchronize(); dist.barrier()
t0 = time.perf_counter()
N = 500
for _ in range(N):
    c.all_reduce(row)
torch.cuda.synchronize()
res['us_per_exchange'] = (time.perf_counter() - t0) / N * 1e6
res['errors'] = c.errors()
if rank == 0:
    print('RESULT ' + json.dumps(res), flush=True)
dist.barrier()
dist.destroy_process_group()
'''


def test_ipc_allreduce_two_processes_one_gpu(gpu, tmp_path):
    s = socket.socket(); s.bind(('127.0.0.1', 0)); port = s.getsockname()[1]; s.close()
    script = tmp_path / 'w.py'
    script.write_text(WORKER)
    env = dict(os.environ, ROOT=ROOT)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2', '--master-addr',
           '127.0.0.1', '--master-port', str(port), str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith('RESULT ')]
    assert line, r.stdout[-2000:]
    res = json.loads(line[0][7:])
    print('IPC exchange:', res)
    assert res['checked'] == 300 and res['mismatch'] == 0, res
    assert res['graph_mismatch'] == 0 and res['errors'] == 0, res
