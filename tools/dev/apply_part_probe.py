"""Dev: bn_act_bwd_apply_part vs bn_act_bwd_apply + bn_act_bwd_partial on random data (bitwise?)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from medical_segmentation_pytorch_amd.ops._ext import require  # noqa: E402

C = require()
dev = 'cuda'
g = torch.Generator(device=dev).manual_seed(0)
for P, Cp in ((2 * 96 * 96, 24), (5000, 40), (777, 72)):
    r = lambda: torch.randn(P, Cp, device=dev, generator=g).to(torch.bfloat16)  # noqa: E731
    dz, y, y2 = r(), r(), r()
    st = torch.randn(4, Cp, device=dev, generator=g)
    st2 = torch.randn(4, Cp, device=dev, generator=g)
    coef = torch.randn(3, Cp, device=dev, generator=g)
    for relu, relu2 in ((True, True), (False, True), (True, False)):
        dy_a = torch.empty_like(dz)
        C.bn_act_bwd_apply(dz, y, st, coef, dy_a, P, Cp, relu)
        nb = C.bn_partial_blocks(P, Cp)
        pa = torch.empty(nb, 2, Cp, device=dev)
        C.bn_act_bwd_partial(dy_a, y2, st2, pa, P, Cp, relu2)
        dy_b = torch.empty_like(dz)
        pb = torch.empty(nb, 2, Cp, device=dev)
        C.bn_act_bwd_apply_part(dz, y, st, coef, dy_b, y2, st2, relu2, pb, P, Cp, relu)
        torch.cuda.synchronize()
        print(P, Cp, relu, relu2, 'dy equal', torch.equal(dy_a, dy_b), 'part equal', torch.equal(pa, pb),
              'max part diff', (pa - pb).abs().max().item(), 'rel', ((pa - pb).norm() / pa.norm()).item())
