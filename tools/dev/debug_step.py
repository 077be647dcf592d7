"""Dev: FusedStep sanity -- grads vs eager fp32, memory growth per step, graph vs no graph."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from medical_segmentation_pytorch_amd.runtime.trainer_engine import FusedStep, make_model  # noqa: E402

dev = torch.device('cuda', 0)
graph = int(sys.argv[1]) if len(sys.argv) > 1 else 0
torch.manual_seed(0)
model = make_model('ducknet', 17).to(dev).train()
ref = copy.deepcopy(model)
x = torch.randn(4, 3, 128, 128, device=dev)
t = torch.randint(0, 2, (4, 128, 128), device=dev)
step = FusedStep(model, x.clone(), t.clone(), lr=0.0, use_graph=bool(graph), total_steps=10)
F.cross_entropy(ref(x), t).backward()
for it in range(6):
    loss = step()
    torch.cuda.synchronize()
    cos = []
    nonfin = []
    for (n, p), q in zip(model.named_parameters(), ref.parameters()):
        g = p.grad
        if not torch.isfinite(g).all():
            nonfin.append(n)
        if q.grad.abs().sum() > 0:
            cos.append((F.cosine_similarity(g.flatten(), q.grad.flatten(), 0).item(), n))
    cos.sort()
    print(f'graph={graph} it={it} loss={float(loss):.5f} mem={torch.cuda.memory_allocated() / 2**30:.2f}GiB '
          f'nonfinite={len(nonfin)} {nonfin[:3]} worst-cos={cos[:3]} median-cos={cos[len(cos) // 2][0]:.4f}', flush=True)
