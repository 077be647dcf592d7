"""SyncBN exchange queue (``ops.bn._Pending``) over gloo, 2 CPU ranks: parked rows of different widths
leave as ONE all-reduce, every job sees its own slice of the global sum, and the flush-on-need hooks
(``need_stats`` / ``need_grads``) fire only for parked results."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from medical_segmentation_pytorch_amd.ops import bn
        ex0 = bn.EXCHANGES[0]
        got = {}
        widths = [6, 10, 4]
        for i, w in enumerate(widths):
            row = torch.full((1, w), float(rank + 1) * (i + 1), dtype=torch.float64)
            key = torch.empty(8, dtype=torch.float32)   # stands in for a parked stats / dy tensor
            got[i] = key
            bn._FWD.add(row, dist.group.WORLD, lambda s, i=i: got.__setitem__(('sum', i), s.clone()), key.data_ptr())
        assert bn.EXCHANGES[0] == ex0, 'nothing may leave before a consumer needs it'
        # an unrelated gradient does not flush the forward queue, nor the (empty) backward one
        bn.need_grads([torch.zeros(3)])
        assert bn.EXCHANGES[0] == ex0
        d = bn.Deferred(torch.zeros(2), got[1], True)
        d.stats = got[1]
        bn.need_stats([d])            # a consumer of parked BN #1 flushes the whole queue
        assert bn.EXCHANGES[0] == ex0 + 1
        bn.need_stats([d])            # idempotent
        assert bn.EXCHANGES[0] == ex0 + 1
        tot = sum(r + 1 for r in range(world))
        for i, w in enumerate(widths):
            s = got[('sum', i)]
            assert s.shape == (1, w)
            assert torch.allclose(s, torch.full((1, w), float(tot * (i + 1)), dtype=torch.float64))
        # backward queue: parked dy keys flush on need; flush_pending drains everything
        dy = torch.empty(4)
        bn._BWD.add(torch.ones(1, 2, dtype=torch.float64), dist.group.WORLD, lambda s: dy.fill_(float(s.sum())),
                    dy.data_ptr())
        bn.need_grads([None, dy])
        assert bn.EXCHANGES[0] == ex0 + 2 and float(dy[0]) == 2.0 * world
        bn._FWD.add(torch.ones(1, 2, dtype=torch.float64), dist.group.WORLD, lambda s: None, 1)
        bn.flush_pending()
        assert bn.EXCHANGES[0] == ex0 + 3 and not bn._FWD.rows and not bn._BWD.rows
        q.put((rank, 'ok'))
    except Exception as e:   # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_pending_exchange_batches_and_flushes_on_need():
    s = socket.socket(); s.bind(('127.0.0.1', 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: 'ok', 1: 'ok'}, res
