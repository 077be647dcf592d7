"""Dev: how well-conditioned is the DuckNet fused-vs-fp32 parity check?  Logits / mean / min grad cosine of
the fused engine and of bf16 autocast against the fp32 native-kernel reference, over input sizes, input
smoothness (white noise vs low-pass images) and label kinds (random vs input-correlated)."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from medical_segmentation_pytorch_amd.models.ducknet import DuckNet  # noqa: E402
from medical_segmentation_pytorch_amd.runtime.fused_model import FusedExecutor  # noqa: E402


def cos(a, b):
    return F.cosine_similarity(a.flatten().float(), b.flatten().float(), dim=0).item()


gpu = torch.device('cuda', 0)
for size, batch, smooth, base in [(128, 4, 0, 17), (128, 4, 9, 17), (128, 4, 25, 17), (256, 4, 25, 17),
                                  (128, 8, 25, 8), (256, 2, 25, 17), (352, 2, 25, 17)]:
    torch.manual_seed(0)
    model = DuckNet(2, 3, base).to(gpu).train()
    ref, ref16 = copy.deepcopy(model), copy.deepcopy(model)
    x = torch.randn(batch, 3, size, size, device=gpu)
    if smooth:
        x = F.avg_pool2d(x, smooth, 1, smooth // 2)
        x = (x - x.mean()) / x.std()
    tgt = (F.avg_pool2d(x[:, :1], 9, 1, 4)[:, 0] > 0).long()
    out = FusedExecutor(model)(x, training=True)
    with torch.backends.cudnn.flags(enabled=False):
        o32 = ref(x)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        o16 = ref16(x).float()
    F.cross_entropy(out, tgt).backward()
    with torch.backends.cudnn.flags(enabled=False):
        F.cross_entropy(o32, tgt).backward()
    F.cross_entropy(o16, tgt).backward()
    cf = [cos(p.grad, q.grad) for p, q in zip(model.parameters(), ref.parameters()) if q.grad.abs().sum() > 0]
    cb = [cos(r.grad, q.grad) for r, q in zip(ref16.parameters(), ref.parameters()) if q.grad.abs().sum() > 0]
    print(f'size {size} batch {batch} smooth {smooth} base {base}: logits fused {cos(out, o32):.4f} bf16 '
          f'{cos(o16, o32):.4f} | grads mean fused {sum(cf) / len(cf):.4f} bf16 {sum(cb) / len(cb):.4f} '
          f'| min fused {min(cf):.4f} bf16 {min(cb):.4f}', flush=True)
