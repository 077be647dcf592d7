"""Dev: per-parameter gradient cosine of the fused executor vs fp32 eager (and bf16 autocast vs fp32)."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from medical_segmentation_pytorch_amd.models import smp  # noqa: E402
from medical_segmentation_pytorch_amd.runtime.fused_model import FusedExecutor  # noqa: E402


def cos(a, b):
    return F.cosine_similarity(a.flatten().float(), b.flatten().float(), dim=0).item()


arch = sys.argv[1] if len(sys.argv) > 1 else 'DeepLabV3'
enc = sys.argv[2] if len(sys.argv) > 2 else 'resnet18'
gpu = torch.device('cuda', 0)
torch.manual_seed(0)
model = getattr(smp, arch)(encoder_name=enc, encoder_weights=None, in_channels=3, classes=2).to(gpu).train()
for m in model.modules():
    if isinstance(m, torch.nn.modules.dropout._DropoutNd):
        m.p = 0.0
ref, ref16 = copy.deepcopy(model), copy.deepcopy(model)
x = torch.randn(4, 3, 64, 64, device=gpu)
tgt = torch.randint(0, 2, (4, 64, 64), device=gpu)
out = FusedExecutor(model)(x, training=True)
F.cross_entropy(out, tgt).backward()
F.cross_entropy(ref(x), tgt).backward()
with torch.autocast('cuda', dtype=torch.bfloat16):
    o16 = ref16(x).float()
F.cross_entropy(o16, tgt).backward()
rows = []
for (n, p), q, r in zip(model.named_parameters(), ref.parameters(), ref16.parameters()):
    if q.grad is None or q.grad.abs().sum() == 0:
        continue
    rows.append((cos(p.grad, q.grad), cos(r.grad, q.grad), n, tuple(p.shape), q.grad.norm().item()))
rows.sort()
for c, cb, n, sh, gn in rows[:25]:
    print(f'{c:.4f} bf16 {cb:.4f}  {n} {sh} |g|={gn:.3e}')
print('mean fused', sum(r[0] for r in rows) / len(rows), 'bf16', sum(r[1] for r in rows) / len(rows))
