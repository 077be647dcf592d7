"""Dev probe: can torch.distributed (nccl = RCCL) collectives be captured in a hipGraph and replayed?
World size 1 over RCCL (one GPU box).  Prints one JSON line per case."""
import json
import os
import sys

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29533')
    os.environ.setdefault('RANK', '0')
    os.environ.setdefault('WORLD_SIZE', '1')
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
    pg2 = dist.new_group([0])
    x = torch.ones(1 << 20, device='cuda')
    y = torch.ones(4096, device='cuda', dtype=torch.float64)
    # eager warm-up (communicator init outside the capture)
    dist.all_reduce(x)
    dist.all_reduce(y, group=pg2)
    torch.cuda.synchronize()
    res = {}
    for mode in ('sync', 'async_wait', 'two_groups'):
        try:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, capture_error_mode='thread_local'):
                    x.mul_(2.0)
                    if mode == 'sync':
                        dist.all_reduce(x)
                    elif mode == 'async_wait':
                        w = dist.all_reduce(x, async_op=True)
                        x.add_(0.0)
                        w.wait()
                    else:
                        w = dist.all_reduce(x, async_op=True)
                        dist.all_reduce(y, group=pg2)
                        w.wait()
                    x.add_(1.0)
            torch.cuda.current_stream().wait_stream(s)
            x.fill_(1.0)
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            res[mode] = {'ok': True, 'x0': x[0].item()}   # world 1: x = ((1*2)+1)*2+1 ... after 3 replays = 15
        except Exception as e:   # noqa: BLE001
            res[mode] = {'ok': False, 'err': repr(e)[:300]}
        print(json.dumps({mode: res[mode]}), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
