#!/usr/bin/env python3
"""Dev probe: fused-vs-fp32 logits / grad cosine of a model under kernel-path switches (which conv path
breaks a model?).  python tools/dev/path_probe.py <model> [size]   (model: tools/conv_bench-style names, e.g. unet, smp-linknet-resnet18)"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from medical_segmentation_pytorch_amd.ops._ext import require  # noqa: E402
from medical_segmentation_pytorch_amd.runtime.fused_model import FusedExecutor  # noqa: E402
from medical_segmentation_pytorch_amd.runtime.trainer_engine import make_model  # noqa: E402


def cos(a, b):
    return F.cosine_similarity(a.flatten().float(), b.flatten().float(), dim=0).item()


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else 'unet'
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    C = require()
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = make_model(name, 32 if name == 'unet' else 17).to(dev).train()
    x = torch.randn(2, 3, size, size, device=dev)
    ref = copy.deepcopy(base)
    print('ref forward ...', flush=True)
    with torch.backends.cudnn.flags(enabled=False):
        out_ref = ref(x)
    print('ref forward done', flush=True)
    tgt = (F.avg_pool2d(x[:, :1], 9, 1, 4)[:, 0] > 0).long()
    with torch.backends.cudnn.flags(enabled=False):
        F.cross_entropy(out_ref, tgt).backward()
    torch.cuda.synchronize()
    print('ref backward done', flush=True)
    for label, gemm, halo, phase, wg in [('default', 1, 1, 1, 1), ('gemm off', 0, 1, 1, 1), ('halo off', 1, 0, 1, 1),
                                         ('phase off', 1, 1, 0, 1), ('wgrad gemm off', 1, 1, 1, 0),
                                         ('all off', 0, 0, 0, 0)]:
        C.conv_set_gemm(bool(gemm))
        C.conv_set_halo(bool(halo))
        C.conv_set_phase(bool(phase))
        C.conv_set_wgrad_gemm(wg)
        print(label, '...', flush=True)
        m = copy.deepcopy(base)
        ex = FusedExecutor(m)
        out = ex(x, training=True)
        torch.cuda.synchronize()
        print('  fwd ok', flush=True)
        F.cross_entropy(out, tgt).backward()
        torch.cuda.synchronize()
        gc = [cos(p.grad, q.grad) for p, q in zip(m.parameters(), ref.parameters()) if q.grad is not None and q.grad.abs().sum() > 0]
        print(f'{label:16s} logits cos {cos(out, out_ref):.4f}  grad cos mean {sum(gc) / len(gc):.4f} min {min(gc):.4f}',
              flush=True)
    C.conv_set_gemm(True); C.conv_set_halo(True); C.conv_set_phase(True); C.conv_set_wgrad_gemm(1)


if __name__ == '__main__':
    main()
