"""Dev: graph vs eager FusedStep from the same state; list params whose grads disagree per step."""
import copy
import sys

import torch

sys.path.insert(0, '.')
from medical_segmentation_pytorch_amd.runtime.bench_step import synthetic_batch  # noqa: E402
from medical_segmentation_pytorch_amd.runtime.trainer_engine import FusedStep, make_model  # noqa: E402

dev = torch.device('cuda', 0)
torch.manual_seed(1)
base = make_model('ducknet', 17).to(dev).train()
x, t = synthetic_batch(8, 128, dev)
steps = [FusedStep(copy.deepcopy(base), x.clone(), t.clone(), lr=1e-3, use_graph=g, total_steps=600) for g in (False, True)]
for it in range(1, 5):
    losses = [float(s()) for s in steps]
    torch.cuda.synchronize()
    bad = []
    for (n, p), q in zip(steps[0].model.named_parameters(), steps[1].model.parameters()):
        a, b = p.grad, q.grad
        rel = float((a - b).norm() / (a.norm() + 1e-20))
        if rel > 0.5:
            bad.append((rel, n, float(a.abs().max()), float(b.abs().max())))
    bad.sort(reverse=True)
    print(f'it={it} losses={losses} n_bad={len(bad)}', flush=True)
    for r in bad[:12]:
        print('   ', r, flush=True)
