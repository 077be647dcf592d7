#!/usr/bin/env python3
"""Dev probe: which BatchNorm data-gradients of one DUCKNet-17 training step are still written by the apply
pass (resolved tokens, or BNs that never deferred), grouped by shape and by the conv that consumed them.
python tools/dev/resolve_probe.py [size] [batch]"""
import collections
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from medical_segmentation_pytorch_amd.models.ducknet import DuckNet  # noqa: E402
from medical_segmentation_pytorch_amd.ops import bn as bnmod  # noqa: E402
from medical_segmentation_pytorch_amd.ops import conv as convmod  # noqa: E402
from medical_segmentation_pytorch_amd.runtime.trainer_engine import FusedStep  # noqa: E402


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 352
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = DuckNet(2, 3, 17).to(dev)
    xs = torch.randn(batch, 3, size, size, device=dev)
    ys = (F.avg_pool2d(xs[:, :1], 9, 1, 4)[:, 0] > 0).long()
    step = FusedStep(model, xs, ys, optimizer='adam', lr=1e-3, use_graph=False, total_steps=4)
    step()
    torch.cuda.synchronize()

    resolved, fused, undeferred = collections.Counter(), collections.Counter(), collections.Counter()
    orig_resolve, orig_fused, orig_def = bnmod.resolve, convmod._fused_bwd, bnmod._dy_deferrable

    def resolve(g):
        if bnmod.peek_deferred(g) is not None:
            f = sys._getframe(1)
            resolved[(tuple(g.shape), f.f_code.co_name, f.f_back.f_code.co_name)] += 1
        return orig_resolve(g)

    def fused_bwd(ctx, plan, gys, xs_, shape, need_dx, dev_):
        r = orig_fused(ctx, plan, gys, xs_, shape, need_dx, dev_)
        fused[(tuple(gys[0].shape), plan.kh, plan.kw, r is not None)] += 1
        return r

    def deferrable(ts):
        ok = orig_def(ts)
        if not ok:
            undeferred[(tuple(ts[0].shape), tuple(type(t.grad_fn).__name__ for t in ts))] += 1
        return ok
    bnmod.resolve, convmod._fused_bwd, bnmod._dy_deferrable = resolve, fused_bwd, deferrable
    step()
    torch.cuda.synchronize()
    for title, cnt in (('resolved tokens (apply pass)', resolved), ('fused backward calls', fused),
                       ('BNs that did not defer (producer not a conv)', undeferred)):
        print(f'== {title}: {sum(cnt.values())}')
        for k, v in sorted(cnt.items(), key=lambda kv: -kv[1]):
            print(f'  {v:4d}  {k}')


if __name__ == '__main__':
    main()
