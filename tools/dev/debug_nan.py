"""Dev: find where NaN parameters appear in fused training (which param, which step)."""
import argparse
import sys

import torch

sys.path.insert(0, '.')
import bench as B  # noqa: E402
from medical_segmentation_pytorch_amd.runtime.bench_step import build_bench_step  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--graph', type=int, default=1)
ap.add_argument('--steps', type=int, default=120)
ap.add_argument('--batch', type=int, default=16)
ap.add_argument('--size', type=int, default=352)
ap.add_argument('--feed', type=int, default=1)
a = ap.parse_args()
dev = torch.device('cuda', 0)
args = argparse.Namespace(train_images=64, size=a.size, batch=a.batch)
feed = B.make_feed(args, dev, seed=1) if a.feed else None
step = build_bench_step(impl='fused', batch=a.batch, size=a.size, base_channel=17, device=dev, feed=feed,
                        total_steps=600, lr=1e-3, use_graph=bool(a.graph))
names = {id(p): n for n, p in step.model.named_parameters()}
for it in range(1, a.steps + 1):
    loss = step()
    torch.cuda.synchronize()
    bad = [n for n, p in step.model.named_parameters() if not torch.isfinite(p).all()]
    gbad = [n for n, p in step.model.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
    mx = max(float(p.detach().abs().max()) for p in step.model.parameters())
    if bad or gbad or it % 10 == 0:
        print(it, 'loss', float(loss), 'maxabs', mx, 'nan params', bad[:8], len(bad), 'nan grads', gbad[:8], len(gbad),
              flush=True)
    if bad:
        for n, p in step.model.named_parameters():
            if n in bad[:3]:
                print(n, p.shape, p.detach().flatten()[:8], p.grad.flatten()[:8] if p.grad is not None else None)
        bufbad = [n for n, b in step.model.named_buffers() if b.is_floating_point() and not torch.isfinite(b).all()]
        print('nan buffers', bufbad[:8], len(bufbad))
        h = step.opt.hyper.cpu().tolist()
        print('hyper', h)
        break
