#!/usr/bin/env python3
"""Accuracy run on the synthetic polyp task (no dataset download is possible): trains a model with the
reference protocol pieces that matter for accuracy -- MyConfig augmentation (randscale [-0.5, 1.0],
colour jitter 0.5 + hue 0.2, flips 0.5; reference datasets/polyp.py:38-47), Adam lr 1e-3
(0.1 * base_lr), per-iteration OneCycle (cos, 3/400 warmup; reference utils/scheduler.py), CE loss,
EMA-free validation of the live weights (MyConfig use_ema=False) -- and validates periodically on a
held-out split with the reference metric: torchmetrics-style macro Dice over both classes from one
confusion matrix (reference utils/metrics.py:4-13), plus foreground Dice (the paper's convention).

    python tools/train_synthetic.py --impl fused --steps 6000 --batch 16 --size 352
    python tools/train_synthetic.py --impl eager ...   (stock PyTorch-ROCm, bf16 autocast: the comparison)

Validation runs twice per checkpoint: fp32 eager module forward (what the reference does,
core/seg_trainer.py:114) and, for the fused engine, its bf16 eval executor -- the gap is reported.
Prints one JSON line per validation and a final summary line (``"final": true``).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def confmat_dice(cm):
    tp = cm.diag()
    dice = 2 * tp / (cm.sum(0) + cm.sum(1)).clamp(min=1)
    iou = tp / (cm.sum(0) + cm.sum(1) - tp).clamp(min=1)
    return float(dice.mean()), float(dice[1]), float(iou.mean())


@torch.no_grad()
def evaluate(forward, imgs, msks, device, bs=16):
    from medical_segmentation_pytorch_amd.utils.transforms import normalize_to_tensor
    cm = torch.zeros(2, 2, dtype=torch.float64)
    for i in range(0, len(imgs), bs):
        x = torch.stack([normalize_to_tensor(im) for im in imgs[i:i + bs]]).to(device)
        t = torch.stack([torch.from_numpy(m.astype('int64')) for m in msks[i:i + bs]]).to(device)
        p = forward(x).float().argmax(1)
        cm += torch.bincount((t * 2 + p).flatten(), minlength=4).view(2, 2).double().cpu()
    return confmat_dice(cm)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--impl', choices=['fused', 'eager'], default='fused')
    ap.add_argument('--model', default='ducknet')
    ap.add_argument('--base-channel', type=int, default=17)
    ap.add_argument('--steps', type=int, default=6000)
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--size', type=int, default=352)
    ap.add_argument('--train-images', type=int, default=880, help='Kvasir-SEG train split size')
    ap.add_argument('--val-images', type=int, default=100)
    ap.add_argument('--val-every', type=int, default=500)
    ap.add_argument('--lr', type=float, default=1e-3)
    ap.add_argument('--seed', type=int, default=1)
    ap.add_argument('--out', default='')
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench as B
    from medical_segmentation_pytorch_amd.runtime.bench_step import build_bench_step
    dev = torch.device('cuda', 0)
    t0 = time.time()
    args = argparse.Namespace(train_images=a.train_images, size=a.size, batch=a.batch)
    feed = B.make_feed(args, dev, seed=a.seed)
    vi, vm = B.synthetic_split(a.val_images, a.size, seed=10_000 + a.seed)
    print(f'[train] data ready in {time.time() - t0:.1f}s', file=sys.stderr, flush=True)
    step = build_bench_step(impl=a.impl, batch=a.batch, size=a.size, base_channel=a.base_channel, device=dev,
                            model_name=a.model, feed=feed, total_steps=a.steps, lr=a.lr)
    model = step.model if a.impl == 'fused' else step.model_ref
    best = {'dice': -1.0}
    hist = []
    t_train = 0.0
    for it in range(1, a.steps + 1):
        ts = time.perf_counter()
        loss = step()
        if it % a.val_every == 0 or it == a.steps:
            torch.cuda.synchronize()
            t_train += time.perf_counter() - ts
            lval = float(loss.detach().float())
            wn = float(sum(float(p.detach().float().norm()) ** 2 for p in model.parameters()) ** 0.5)
            model.eval()
            d32, fg32, iou32 = evaluate(lambda x: model(x), vi, vm, dev)
            rec = {'step': it, 'dice_fp32': round(d32, 4), 'fg_dice_fp32': round(fg32, 4), 'miou_fp32': round(iou32, 4)}
            if a.impl == 'fused':
                from medical_segmentation_pytorch_amd.runtime.fused_model import FusedExecutor
                ex = FusedExecutor(model)
                d16, fg16, iou16 = evaluate(lambda x: ex(x, training=False), vi, vm, dev)
                rec.update(dice_bf16_fused=round(d16, 4), fg_dice_bf16_fused=round(fg16, 4))
            model.train()
            rec['train_s'] = round(t_train, 1)
            rec['loss'] = round(lval, 5)
            rec['weight_norm'] = round(wn, 3)
            hist.append(rec)
            print(json.dumps(rec), flush=True)
            if d32 > best['dice']:
                best = {'dice': d32, 'step': it, **rec}
        else:
            t_train += time.perf_counter() - ts
    summary = {'final': True, 'impl': a.impl, 'model': f'{a.model}-{a.base_channel}', 'steps': a.steps,
               'batch': a.batch, 'size': a.size, 'train_images': a.train_images, 'val_images': a.val_images,
               'best': best, 'last': hist[-1], 'train_s': round(t_train, 1),
               'data': 'synthetic polyp frames (datasets/synthetic.py), MyConfig augmentation on the GPU'}
    print(json.dumps(summary), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump({'summary': summary, 'history': hist}, f, indent=1)


if __name__ == '__main__':
    main()
