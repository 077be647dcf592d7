"""Dev: DuckNet fused-vs-fp32 parity in EVAL mode (running-stat BN: no batch coupling) -- is the
end-to-end comparison well conditioned there?  Also train mode with momentum-warmed running stats."""
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
for size, batch, warm in [(128, 4, False), (128, 4, True), (256, 2, True)]:
    torch.manual_seed(0)
    model = DuckNet(2, 3, 17).to(gpu)
    x = torch.randn(batch, 3, size, size, device=gpu)
    x = F.avg_pool2d(x, 25, 1, 12)
    x = (x - x.mean()) / x.std()
    if warm:   # running stats = the batch statistics (momentum 1): eval BN == train BN of this batch
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.momentum = 1.0
        with torch.no_grad():
            model.train()(x)
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.momentum = 0.1
    model.eval()
    ref, ref16 = copy.deepcopy(model), copy.deepcopy(model)
    tgt = (F.avg_pool2d(x[:, :1], 9, 1, 4)[:, 0] > 0).long()
    out = FusedExecutor(model)(x, training=False)
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
    print(f'eval size {size} batch {batch} warm {warm}: logits fused {cos(out, o32):.4f} bf16 {cos(o16, o32):.4f} | '
          f'grads mean fused {sum(cf) / len(cf):.4f} bf16 {sum(cb) / len(cb):.4f} | min fused {min(cf):.4f} '
          f'bf16 {min(cb):.4f}', flush=True)
