#!/usr/bin/env python3
"""Accuracy through the reference's entry point: runs ``python main.py`` (MyConfig + CLI overrides ->
SegTrainer.run: train, validate every ``--val-every`` epochs, save best.pth, val_best on it -- reference
``main.py:8-21``, ``core/base_trainer.py:78-127``) on the synthetic 352x352 polyp split (no dataset can be
downloaded; datasets/synthetic.py), then summarises ``save_dir/val_history.json``: best / val_best macro
Dice (the reference metric), foreground Dice (2 IoU_fg / (1 + IoU_fg)), mIoU, and the time and
iterations to the first validation at macro Dice >= ``--target``.

    python tools/accuracy_main.py --batch 320 --epochs 300 --out profiles/r03/accuracy_main_bs320.json
    python tools/accuracy_main.py --batch 16 --epochs 55 --val-fp32 ...
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def summarise(hist, target):
    h = json.load(open(hist))
    rows = [r for r in h['history'] if not r['val_best']]
    best = max(rows, key=lambda r: r['score']) if rows else None
    final = [r for r in h['history'] if r['val_best']]

    def fg(r):
        j = r['iou'][-1] if 'iou' in r else None
        return None if j is None else round(2 * j / (1 + j), 4)

    hit = next((r for r in rows if r['score'] >= target), None)
    return {
        'best_score': round(h['best_score'], 4),
        'best': None if best is None else {'epoch': best['epoch'], 'train_itrs': best['train_itrs'],
                                           'elapsed_s': best['elapsed_s'], 'macro_dice': round(best['score'], 4),
                                           'fg_dice': fg(best), 'miou': round(sum(best['iou']) / len(best['iou']), 4)
                                           if 'iou' in best else None},
        # val_best runs on the val split, then (MyConfig use_test_set) on the held-out test split
        **{name: None if len(final) <= i else {'macro_dice': round(final[i]['score'], 4), 'fg_dice': fg(final[i]),
                                                'miou': round(sum(final[i]['iou']) / len(final[i]['iou']), 4)
                                                if 'iou' in final[i] else None, 'fp32': final[i]['fp32']}
           for i, name in enumerate(('val_best', 'test_best'))},
        f'time_to_macro_dice_{target}': None if hit is None else {'elapsed_s': hit['elapsed_s'],
                                                                  'train_itrs': hit['train_itrs'],
                                                                  'epoch': hit['epoch']},
        'wall_s': h['wall_s'], 'iters_per_epoch': h['iters_per_epoch'], 'train_bs': h['train_bs'],
        'history': [{'epoch': r['epoch'], 'itrs': r['train_itrs'], 's': r['elapsed_s'], 'dice': round(r['score'], 4),
                     'fg_dice': fg(r)} for r in rows],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=320)
    ap.add_argument('--accum', type=int, default=1, help='gradient accumulation micro-batches (config.accum_steps)')
    ap.add_argument('--epochs', type=int, default=300)
    ap.add_argument('--val-every', type=int, default=10)
    ap.add_argument('--size', type=int, default=352)
    ap.add_argument('--train-images', type=int, default=880, help='Kvasir-SEG train split size')
    ap.add_argument('--val-images', type=int, default=100)
    ap.add_argument('--base-lr', type=float, default=0.01, help='reference rule: adam lr = 0.1 * base_lr * gpu_num')
    ap.add_argument('--lr-scale', default='reference', choices=['reference', 'sqrt', 'linear'],
                    help='large-batch lr rule (utils/optimizer.lr_batch_factor)')
    ap.add_argument('--begin-val', type=int, default=0, help='first validated epoch')
    ap.add_argument('--model', default='ducknet')
    ap.add_argument('--base-channel', type=int, default=17)
    ap.add_argument('--val-fp32', action='store_true', help='validate the EMA model in fp32 eager (reference protocol)')
    ap.add_argument('--target', type=float, default=0.98)
    ap.add_argument('--save-dir', default='')
    ap.add_argument('--out', default='')
    ap.add_argument('--extra', nargs=argparse.REMAINDER, default=[])
    a = ap.parse_args()
    save = a.save_dir or tempfile.mkdtemp(prefix='msp_acc_')
    cmd = [sys.executable, '-u', os.path.join(ROOT, 'main.py'), '--dataset', 'synthetic', '--model', a.model,
           '--base_channel', str(a.base_channel), '--crop_size', str(a.size), '--synthetic_size', str(a.size),
           '--synthetic_num', str(a.train_images), str(a.val_images), str(a.val_images), '--train_bs', str(a.batch),
           '--total_epoch', str(a.epochs), '--val_interval', str(a.val_every), '--begin_val_epoch', str(a.begin_val),
           '--lr_scale', a.lr_scale, '--accum_steps', str(a.accum),
           '--val_bs', '16', '--save_dir', save, '--base_lr', str(a.base_lr), '--use_tb', '--load_ckpt',
           '--no_progress_bar', '--log_interval', '1000'] + (['--val_fp32'] if a.val_fp32 else []) + a.extra
    print('[acc]', ' '.join(cmd), file=sys.stderr, flush=True)
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT)
    if r.returncode != 0:
        sys.exit(r.returncode)
    out = {'entry': 'python main.py (SegTrainer.run -> val_best on best.pth)', 'model': f'{a.model}-{a.base_channel}',
           'batch': a.batch, 'accum_steps': a.accum, 'global_batch': a.batch * a.accum, 'epochs': a.epochs, 'size': a.size, 'train_images': a.train_images,
           'val_images': a.val_images, 'lr_scale': a.lr_scale,
           'adam_lr': json.load(open(os.path.join(save, 'config.json'))).get('lr', 0.1 * a.base_lr),
           'val_fp32': a.val_fp32,
           'data': 'synthetic polyp frames (datasets/synthetic.py), MyConfig augmentation on the GPU (DeviceAugLoader)',
           'process_wall_s': round(time.time() - t0, 1),
           **summarise(os.path.join(save, 'val_history.json'), a.target)}
    print(json.dumps({k: v for k, v in out.items() if k != 'history'}), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(out, f, indent=1)
    if not a.save_dir:
        shutil.rmtree(save, ignore_errors=True)


if __name__ == '__main__':
    main()
