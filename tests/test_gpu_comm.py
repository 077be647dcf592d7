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
res = {'self_test': True, 'mismatch': 0, 'checked': 0, 'rank_disagree': 0}


def close(got, ref, x):
    if world == 2:   # one fp64 addition: bitwise the collective
        return torch.equal(got, ref)
    # the kernel sums in rank order, gloo in its own: equal up to the rounding of world - 1 additions,
    # bounded by the magnitude sum (cancellation makes any bound relative to the result meaningless)
    mag = x.abs()
    dist.all_reduce(mag)
    return bool(((got - ref).abs() <= world * 2.0 ** -52 * mag).all())

g = torch.Generator().manual_seed(100 + rank)
for it in range(300):
    n = [1, 7, 1088, 4099, c.cap][it % 5]
    x = torch.randn(n, generator=g, dtype=torch.float64) * 10 ** (it % 7 - 3)
    ref = x.clone()
    dist.all_reduce(ref)                       # gloo, CPU
    buf = x.to(dev)
    c.all_reduce(buf)
    got = buf.cpu()
    res['mismatch'] += int(not close(got, ref, x))
    # every rank must hold the SAME bits (rank-order reduction on every rank)
    mine = got.clone()
    dist.broadcast(mine, 0)
    res['rank_disagree'] += int(not torch.equal(mine, got))
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
    gmis += int(not close(buf.cpu(), ref, v))
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


@pytest.mark.parametrize('world', [2, 4])
def test_ipc_allreduce_processes_one_gpu(gpu, tmp_path, world):
    """2 and 4 ranks (all on the one GPU of the box): correctness vs gloo, identical bits on every rank,
    hipGraph capture / replay, no timeouts."""
    s = socket.socket(); s.bind(('127.0.0.1', 0)); port = s.getsockname()[1]; s.close()
    script = tmp_path / 'w.py'
    script.write_text(WORKER)
    env = dict(os.environ, ROOT=ROOT)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={world}', '--master-addr',
           '127.0.0.1', '--master-port', str(port), str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith('RESULT ')]
    assert line, r.stdout[-2000:]
    res = json.loads(line[0][7:])
    print('IPC exchange:', res)
    assert res['checked'] == 300 and res['mismatch'] == 0 and res['rank_disagree'] == 0, res
    assert res['graph_mismatch'] == 0 and res['errors'] == 0, res


TIMEOUT_WORKER = r'''
import os, sys, time, torch, torch.distributed as dist
sys.path.insert(0, os.environ['ROOT'])
from medical_segmentation_pytorch_amd.runtime import comm
dist.init_process_group('gloo')
rank = dist.get_rank()
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
comm.POLICY['mode'] = 'ipc'
c = comm.attach(dist.group.WORLD, dev)   # collective: both ranks, self-test included
assert c is not None and c.timeout_s == 2.0, c.timeout_s
dist.barrier()
if rank == 1:
    time.sleep(120)   # a rank that never reaches the exchange (killed by the supervisor meanwhile)
    sys.exit(0)
buf = torch.ones(64, dtype=torch.float64, device=dev)
c.all_reduce(buf)     # the peer never signals: the kernel gives up after 2 s and writes NaN
torch.cuda.synchronize()
print('RESULT nan=%d errors=%d' % (int(torch.isnan(buf).all().item()), c.errors()), flush=True)
comm.check()          # -> RuntimeError naming the timeout: rank 0 exits non-zero
'''

LAUNCH = r'''
import os, sys
sys.path.insert(0, os.environ['ROOT'])
from medical_segmentation_pytorch_amd.utils.launch import spawn_ranks
sys.exit(spawn_ranks(2, [sys.argv[1]], grace_s=5.0))
'''


def test_ipc_timeout_names_the_peer_and_tears_the_job_down(gpu, tmp_path):
    """A peer that never arrives: the exchange kernel's deadline (MSP_SYNCBN_IPC_TIMEOUT) turns the result into
    NaN and counts an error, ``comm.check()`` raises a named error, the rank exits non-zero and the launcher
    (utils.launch.spawn_ranks, the bench / main.py supervisor) stops the other rank -- instead of a hang."""
    import time
    (tmp_path / 'w.py').write_text(TIMEOUT_WORKER)
    (tmp_path / 'l.py').write_text(LAUNCH)
    env = dict(os.environ, ROOT=ROOT, MSP_SYNCBN_IPC_TIMEOUT='2')
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, str(tmp_path / 'l.py'), str(tmp_path / 'w.py')], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode != 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert 'RESULT nan=1 errors=1' in r.stdout, r.stdout[-2000:]
    assert 'timed out waiting for a peer' in r.stderr, r.stderr[-3000:]
    assert time.monotonic() - t0 < 100   # torn down, not left waiting for the sleeping rank
