"""Dev: per-step trajectory of the fused step (loss, grad/param magnitudes) to find a divergence."""
import argparse
import sys

import torch

sys.path.insert(0, '.')
import bench as B  # noqa: E402
from medical_segmentation_pytorch_amd.runtime.bench_step import build_bench_step  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--graph', type=int, default=1)
ap.add_argument('--steps', type=int, default=12)
ap.add_argument('--batch', type=int, default=16)
ap.add_argument('--size', type=int, default=352)
ap.add_argument('--impl', default='fused')
a = ap.parse_args()
dev = torch.device('cuda', 0)
args = argparse.Namespace(train_images=64, size=a.size, batch=a.batch)
feed = B.make_feed(args, dev, seed=1)
step = build_bench_step(impl=a.impl, batch=a.batch, size=a.size, base_channel=17, device=dev, feed=feed,
                        total_steps=600, lr=1e-3, use_graph=bool(a.graph))
model = step.model if a.impl == 'fused' else step.model_ref
for it in range(1, a.steps + 1):
    loss = step()
    torch.cuda.synchronize()
    gmax, gname = max((float(p.grad.abs().max()), n) for n, p in model.named_parameters() if p.grad is not None)
    pmax, pname = max((float(p.detach().abs().max()), n) for n, p in model.named_parameters())
    rv = [b for n, b in model.named_buffers() if n.endswith('running_var')]
    rvmax = max(float(b.max()) for b in rv)
    print(f'{a.impl} g={a.graph} it={it} loss={float(loss):.4f} gmax={gmax:.3e} ({gname}) pmax={pmax:.3e} ({pname}) '
          f'rvmax={rvmax:.3e}', flush=True)
