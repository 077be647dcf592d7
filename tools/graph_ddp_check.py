#!/usr/bin/env python3
"""Graph-captured multi-rank step == eager multi-rank step, bitwise, on the real RCCL path.

Run under a launcher (one process per GPU, ``torchrun --nproc-per-node N tools/graph_ddp_check.py``; on a
one-GPU box N = 1): every rank builds the same DUCKNet from one seed and trains it twice over RCCL with the
gradient bucketer attached (at world 1 too) and SyncBN on -- once eager, once with the whole step (bucket
all-reduces and SyncBN collectives included) captured in a hipGraph after one eager warm-up step (the
bucket rebuild and every communicator init happen there) -- then compares parameters and per-step losses
bitwise.  Rank 0 prints one JSON line.  Reference DDP step: utils/parallel.py:17-44, core/seg_trainer.py:24-95.
"""
import copy
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    steps = int(os.environ.get('GDC_STEPS', '5'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    dist.init_process_group('nccl', device_id=dev)
    rank, world = dist.get_rank(), dist.get_world_size()
    from medical_segmentation_pytorch_amd.runtime.bench_step import synthetic_batch
    from medical_segmentation_pytorch_amd.runtime.trainer_engine import FusedStep, make_model
    torch.manual_seed(0)
    base = make_model('ducknet', 8).to(dev).train()
    x, t = synthetic_batch(4, 64, dev, seed=rank)
    mk = lambda g: FusedStep(copy.deepcopy(base), x.clone(), t.clone(), lr=1e-3, use_graph=g,  # noqa: E731
                             total_steps=50, distributed=True, bucket_world1=True)
    eager, graph = mk(False), mk(True)
    loss_eq, lossv = [], []
    for _ in range(steps):
        le = eager().detach().clone()
        lg = graph().detach().clone()
        loss_eq.append(bool(torch.equal(le, lg)))
        lossv.append(float(le))
    torch.cuda.synchronize()
    mism = [n for (n, p), q in zip(eager.model.named_parameters(), graph.model.parameters()) if not torch.equal(p, q)]
    out = {'world': world, 'steps': steps, 'graph_captured': graph.graph is not None,
           'bucketer': graph.bucketer is not None, 'buckets': len(graph.bucketer.buckets) if graph.bucketer else 0,
           'buckets_rebuilt': bool(graph.bucketer.rebuilt) if graph.bucketer else False,
           'losses_equal': loss_eq, 'losses': lossv, 'param_mismatches': mism[:5], 'n_mismatch': len(mism)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if (not mism and all(loss_eq) and out['graph_captured']) else 1


if __name__ == '__main__':
    sys.exit(main())
