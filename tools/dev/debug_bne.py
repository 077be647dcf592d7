"""Dev diagnostics: BN-epilogue on/off and deferred-BN numerics on a small DuckNet (GPU)."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from medical_segmentation_pytorch_amd.models.ducknet import DuckNet  # noqa: E402
from medical_segmentation_pytorch_amd.runtime import fused_model  # noqa: E402
from medical_segmentation_pytorch_amd.runtime.fused_model import FusedExecutor  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


dev = torch.device('cuda', 0)
torch.manual_seed(0)
base = DuckNet(2, 3, 17).to(dev).train()
x = torch.randn(2, 3, 64, 64, device=dev)
tgt = torch.randint(0, 2, (2, 64, 64), device=dev)
runs = {}
for tag, on in (('off', False), ('off2', False), ('on', True)):
    fused_model._BN_EPILOGUE = on
    m = copy.deepcopy(base)
    out = FusedExecutor(m)(x, training=True)
    F.cross_entropy(out, tgt).backward()
    runs[tag] = {n: p.grad.clone() for n, p in m.named_parameters()}
ref = copy.deepcopy(base)
F.cross_entropy(ref(x), tgt).backward()
fp32 = {n: p.grad.clone() for n, p in ref.named_parameters()}
rows = []
for n in runs['off']:
    rows.append((rel(runs['on'][n], runs['off'][n]), rel(runs['off2'][n], runs['off'][n]),
                 rel(runs['off'][n], fp32[n]), rel(runs['on'][n], fp32[n]), n))
rows.sort(reverse=True)
print('on-vs-off  off-vs-off  off-vs-fp32  on-vs-fp32  param')
for r in rows[:25]:
    print(f'{r[0]:.2e}  {r[1]:.2e}  {r[2]:.2e}  {r[3]:.2e}  {r[4]}')
print('median on-vs-off', sorted(r[0] for r in rows)[len(rows) // 2])
