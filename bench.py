#!/usr/bin/env python3
"""Headline benchmark: DUCKNet-17 training images/sec at 352x352, bf16, 1..N MI355X (weak scaling).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is launched under
``torch.distributed.run`` with one rank per GPU (RCCL).  Each step is a full reference training
iteration (``core/seg_trainer.py:24-95`` semantics): zero_grad, forward, CE loss, backward (DDP
bucketed all-reduce + SyncBN), optimizer step (Adam, MyConfig default), OneCycle scheduler step and
EMA update.  W untimed warmup steps, then K steps bracketed by barrier + synchronize; the MAX
elapsed over ranks is reported.  Data: synthetic 352x352 polyp images/masks, random-init weights.

Per-GPU micro-batch defaults to 320 images on the fused engine: the north star sizes micro-batches to
fill the 288 GB of HBM3E (measured on one MI355X: 434 img/s at 128 / 67 GiB, 445 at 256 / 134 GiB, 459.5
at 384 / 229 GiB -- the small deep layers fill the chip better); 320 (~191 GiB allocated) keeps
headroom for the caching allocator and the RCCL / DDP buffers of the multi-GPU runs at a cost of well
under 1 % (``--batch 384`` for the last bit).  The eager engine defaults to 128 (its NCHW step needs ~103 GiB there).  At the reference's
16 the step is dominated by fixed-cost launches and, under DDP, SyncBN exchanges; ``--batch 16``
reproduces MyConfig's per-process batch.

``--impl fused`` (default) runs the MI355X-native engine (HIP kernels + hipGraph); ``--impl eager``
runs the same step with stock PyTorch-ROCm (MIOpen convs, torch DDP/SyncBN) = the in-house
"reference speed" of BASELINE.md.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--batch', type=int, default=None,
                   help='per-GPU micro-batch (images); default 320 fused (~191 GiB of the 288 GB HBM3E; 384: 229 GiB), 128 eager')
    p.add_argument('--size', type=int, default=352)
    p.add_argument('--base-channel', type=int, default=17)
    p.add_argument('--impl', choices=['fused', 'eager'], default='fused')
    p.add_argument('--model', default='ducknet',
                   help="ducknet | unet | smp-<resnet encoder> (e.g. smp-resnet101, BASELINE config #3)")
    p.add_argument('--teacher', default=None,
                   help='KD teacher (e.g. smp-resnet101; BASELINE config #4 = --base-channel 34 --teacher smp-resnet101)')
    p.add_argument('--channels-last', action='store_true')
    p.add_argument('--no-graph', action='store_true')
    p.add_argument('--graph-ddp', choices=['auto', 'on', 'off'], default='auto',
                   help='capture the multi-rank step (bucket all-reduces + SyncBN RCCL calls) in the hipGraph: '
                        'auto = on at per-GPU batch <= 64, where host launches would be exposed; at the bench batch '
                        'the step is GPU-bound and runs uncaptured, so the comm evidence pass (eager per-bucket '
                        'RCCL timings and knock-outs) can run')
    p.add_argument('--ddp', action='store_true',
                   help='run the distributed code path (process group, RCCL gradient buckets) even at WORLD_SIZE=1')
    p.add_argument('--data', choices=['augment', 'fixed'], default='augment',
                   help='augment (default): every step draws a fresh MyConfig-augmented batch from an HBM-resident '
                        'synthetic polyp split (GPU augmentation kernels, inside the timed loop); fixed: replay one '
                        'resident batch (isolates the model step)')
    p.add_argument('--train-images', type=int, default=128,
                   help='synthetic train split size (per rank; a larger --batch spans several epochs of it)')
    p.add_argument('--val-images', type=int, default=32, help='held-out synthetic val split for the Dice (0 = skip)')
    p.add_argument('--lr', type=float, default=1e-3, help='Adam lr per GPU (reference: 0.1 * base_lr * gpu_num)')
    p.add_argument('--seed', type=int, default=1, help='trainer random_seed (model init, data order; MyConfig: 1)')
    p.add_argument('--comm-steps', type=int, default=3,
                   help='multi-GPU evidence pass after the timed region (0 = off): per-bucket RCCL timings, SyncBN '
                        'exchange count/time, and the step time with every collective knocked out')
    a = p.parse_args(argv)
    if a.batch is None:
        a.batch = 320 if a.impl == 'fused' and a.model == 'ducknet' and a.base_channel == 17 else 128
    return a


def synthetic_split(n, size, seed):
    """n synthetic polyp frames (HWC uint8) + masks (HW {0,1} uint8), reference-like content."""
    import numpy as np
    from medical_segmentation_pytorch_amd.datasets.synthetic import make_sample
    rng = np.random.default_rng(seed)
    pairs = [make_sample(size, rng) for _ in range(n)]
    return [p[0] for p in pairs], [p[1] for p in pairs]


def make_feed(args, device, seed):
    """The timed loop's data pipeline: HBM-resident split + the reference train augmentation
    (MyConfig: randscale [-0.5, 1.0], colour jitter 0.5 (+ hue 0.2), flips 0.5; crop = bench size) on the
    GPU kernels, one fresh batch per step written into the step's static input buffers."""
    from medical_segmentation_pytorch_amd.datasets.device_loader import DeviceAugLoader, DeviceDataset
    from medical_segmentation_pytorch_amd.utils.transforms import SegAugment
    imgs, msks = synthetic_split(args.train_images, args.size, seed)
    data = DeviceDataset.from_arrays(imgs, msks, device)
    aug = SegAugment(args.size, args.size, randscale=[-0.5, 1.0], brightness=0.5, contrast=0.5, saturation=0.5,
                     h_flip=0.5, v_flip=0.5)
    loader = DeviceAugLoader(None, args.batch, device, seed=seed, data=data, aug=aug)
    order = loader.stream()

    def feed(images, masks):
        loader.batch(next(order), out=(images, masks))
    return feed


def val_dice(model, args, device, seed):
    """Reference validation metric (torchmetrics Dice, average='macro' over both classes, from one
    confusion matrix -- reference utils/metrics.py:4-13) + foreground Dice, on a held-out synthetic split,
    evaluated by the fused executor in eval mode (running BN statistics)."""
    from medical_segmentation_pytorch_amd.runtime.fused_model import FusedExecutor
    from medical_segmentation_pytorch_amd.utils.transforms import normalize_to_tensor
    imgs, msks = synthetic_split(args.val_images, args.size, seed)
    ex = FusedExecutor(model)
    model.eval()
    cm = torch.zeros(2, 2, dtype=torch.float64)
    with torch.no_grad():
        for i in range(0, len(imgs), 16):
            x = torch.stack([normalize_to_tensor(im) for im in imgs[i:i + 16]]).to(device)
            t = torch.stack([torch.from_numpy(m.astype('int64')) for m in msks[i:i + 16]]).to(device)
            p = ex(x, training=False).argmax(1)
            cm += torch.bincount((t * 2 + p).flatten(), minlength=4).view(2, 2).double().cpu()
    model.train()
    tp = cm.diag()
    dice = 2 * tp / (cm.sum(0) + cm.sum(1)).clamp(min=1)
    return float(dice.mean()), float(dice[1])


def comm_evidence(step, args, dist, step_ms, device):
    """Multi-GPU evidence, measured AFTER the timed region (and after the Dice): (1) ``comm_steps``
    instrumented steps -- per gradient bucket its size, RCCL on-stream time, how long before the end of
    backward it was issued (the compute it can hide under) and whether it only left at finish(); every
    SyncBN exchange's RCCL time; (2) ``comm_steps`` steps with EVERY collective knocked out (local BN
    statistics, no gradient averaging: a timing probe that leaves the ranks' weights diverged, hence last)
    -> exposed communication = step time - that.  Reference comm pattern: utils/parallel.py:35-39."""
    import statistics
    from medical_segmentation_pytorch_amd.ops import bn as bnmod
    bk = getattr(step, 'bucketer', None)
    n = args.comm_steps
    world = dist.get_world_size()
    cuda = device.type == 'cuda'

    def sync():
        if cuda:
            torch.cuda.synchronize(device)
    out = {'world_size': world, 'backend': dist.get_backend(),
           'rccl_version': '.'.join(str(v) for v in torch.cuda.nccl.version()) if cuda else None,
           'timed_step_ms': round(step_ms, 3)}
    if bk is not None:
        bk.instrument = True
    bnmod.COMM['instrument'] = True
    bnmod.COMM['works'] = []
    ex0 = bnmod.EXCHANGES[0]
    from medical_segmentation_pytorch_amd.runtime import comm as ipc_comm
    ipc_comm.wait_stats(reset=True)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    sync()
    out['instrumented_step_ms'] = round((time.perf_counter() - t0) / n * 1e3, 3)
    out['syncbn_exchanges_per_step'] = (bnmod.EXCHANGES[0] - ex0) / n
    out['syncbn_exchange_path'] = ipc_comm.describe()
    # IPC path: per exchange, the spin before the last peer's flag (rank skew) vs the rest (transport)
    out['syncbn_ipc_wait'] = ipc_comm.wait_stats(reset=True) or None
    durs = []
    for _, w in bnmod.COMM['works']:
        try:
            durs.append(float(w._get_duration()))
        except Exception:
            pass
    out['syncbn_exchange_ms_per_step'] = round(sum(durs) / n, 3) if durs else None
    out['syncbn_bytes_per_step'] = sum(b for b, _ in bnmod.COMM['works']) / n
    bnmod.COMM['instrument'] = False
    bnmod.COMM['works'] = []
    if bk is not None:
        recs = bk.collect()
        bk.instrument = False
        per = {}
        for r in recs:
            per.setdefault(r['bucket'], []).append(r)
        out['buckets'] = [{'bucket': b, 'mib': rs[0]['mib'],
                           'rccl_ms': (round(statistics.median([r['rccl_ms'] for r in rs if r['rccl_ms'] is not None]), 3)
                                       if any(r['rccl_ms'] is not None for r in rs) else None),
                           'issue_to_bwd_end_ms': round(statistics.median([r['issue_to_bwd_end_ms'] for r in rs]), 3),
                           'late': any(r['late'] for r in rs)} for b, rs in sorted(per.items())]
        ro = list(dict.fromkeys(bk.ready_order))
        out['buckets_rebuilt_in_ready_order'] = bool(bk.rebuilt) and bk.bucket_order()[:len(ro)] == ro
        out['grad_ready_order_is_reverse_registration'] = ro == sorted(ro, reverse=True)
    # knock-out pass
    if bk is not None:
        bk.enabled = False
    bnmod.COMM['enabled'] = False
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    sync()
    t = torch.tensor([(time.perf_counter() - t0) / n * 1e3], device=device, dtype=torch.float64)
    bnmod.COMM['enabled'] = True
    if bk is not None:
        bk.enabled = True
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out['step_ms_comm_off'] = round(t.item(), 3)
    out['exposed_comm_ms'] = round(step_ms - t.item(), 3)
    return out


def model_label(args):
    if args.model == 'ducknet':
        name = f'DUCKNet-{args.base_channel}'
    elif args.model == 'unet':
        name = f'UNet-{args.base_channel}'
    else:
        parts = args.model.split('-')   # smp-<encoder> | smp-<decoder>-<encoder>
        name = f'smp-{parts[1]}({parts[2]})' if len(parts) == 3 else f'smp-Unet({args.model[4:]})'
    return name + (f' + KD teacher {args.teacher}' if args.teacher else '')


# In-house reference speed: the reference's training step in eager PyTorch-ROCm on one
# MI355X at its best measured config, DUCKNet-17 352x352 -- channels-last bs128, 158.37 img/s (round-3
# sweep over bs 16/32/64/128: 120.3 / 141.6 / 152.3 / 158.4; profiles/eager_reference_speed.json, kept
# here too because the profiles directory does not travel to the GPU boxes).
EAGER_REFERENCE_IMG_S_PER_GPU = 158.37
# The same protocol for the other BASELINE configs at 352x352 (eager channels-last, one measured batch each,
# round 3: profiles/r03/eager_{r101_cl_bs64,kd_cl_bs32}.json): (model, base channel, teacher) -> img/s/GPU
EAGER_REFERENCE_CONFIGS = {
    ('ducknet', 17, None): EAGER_REFERENCE_IMG_S_PER_GPU,
    ('smp-resnet101', None, None): 877.91,        # config #3: smp-Unet(ResNet-101), bs64
    ('ducknet', 34, 'smp-resnet101'): 54.09,      # config #4: DUCKNet-34 + ResNet-101-Unet KD teacher, bs32
}


def self_launch(args, argv=None):
    """``python bench.py --gpus N`` (N > 1) without a launcher: start N rank processes (torchrun
    environment, one per GPU) BEFORE this process makes any GPU call, supervise them (the first failing
    rank stops the rest) and return the job's exit code.  Returns None when this process is a rank."""
    if args.gpus <= 1 or os.environ.get('WORLD_SIZE') is not None:
        return None
    from medical_segmentation_pytorch_amd.utils.launch import spawn_ranks
    rest = list(sys.argv[1:] if argv is None else argv)
    print(f'[bench] no WORLD_SIZE in the environment: starting {args.gpus} ranks (one per GPU)', file=sys.stderr,
          flush=True)
    return spawn_ranks(args.gpus, [os.path.abspath(__file__)] + rest)


def main(argv=None):
    args = parse_args(argv)
    rc = self_launch(args, argv)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))

    dist = None
    cuda = torch.cuda.is_available()   # (first GPU call of this process: after the self-launch decision)
    # test hooks: BENCH_DIST_BACKEND=gloo + BENCH_SAME_DEVICE=1 rehearse the N-rank path on one GPU
    # (RCCL refuses two ranks per device); the driver's runs use RCCL, one rank per GPU.  Without a GPU the
    # whole contract runs on the CPU over gloo (the trainer's eager engine): the CPU test tier's rehearsal.
    dev_index = 0 if os.environ.get('BENCH_SAME_DEVICE') == '1' else local_rank
    ddp = world > 1 or args.ddp
    if ddp:
        import torch.distributed as dist
        if cuda:
            torch.cuda.set_device(dev_index)
        backend = os.environ.get('BENCH_DIST_BACKEND', 'nccl' if cuda else 'gloo')
        # per-collective on-stream durations for the evidence pass (Work._get_duration; captured works
        # carry timing events too: tools/dev/graph_rccl_probe.py runs with it set)
        os.environ.setdefault('TORCH_NCCL_ENABLE_TIMING', '1')
        kw = {'device_id': torch.device('cuda', dev_index)} if backend == 'nccl' else {}
        dist.init_process_group(backend, **kw)
        world, rank = dist.get_world_size(), dist.get_rank()   # the process group's own view (n_gpus)
    if world != args.gpus:
        # a bench that silently ran a different job size would report a wrong n_gpus / scaling point
        print(f'[bench] error: --gpus {args.gpus} but the job has {world} rank(s)', file=sys.stderr, flush=True)
        sys.exit(3)
    device = torch.device('cuda', dev_index) if cuda else torch.device('cpu')

    def sync():
        if cuda:
            torch.cuda.synchronize()

    impl = args.impl
    # multi-rank steps: the RCCL collectives are captured with the rest of the step when --graph-ddp is on
    # (auto: per-GPU batch <= 64, where the ~2k host launches per step would be exposed); at the bench
    # batch the step is GPU-bound (profiles/r06/ddp_graph: graph vs no graph within noise), so it runs
    # uncaptured and the per-bucket RCCL evidence pass below can run
    graph_ddp = args.graph_ddp == 'on' or (args.graph_ddp == 'auto' and args.batch <= 64)
    if ddp and dist.get_backend() != 'nccl':   # gloo collectives run on the host: never captured
        graph_ddp = False
    use_graph = cuda and not args.no_graph and (not ddp or graph_ddp)
    total_steps = args.warmup + args.steps + 2 * args.comm_steps + 2
    save_dir = None
    if impl == 'fused':
        # the benched step IS the trainer's: SegTrainer.train_step on its own DeviceAugLoader batches
        import tempfile
        from medical_segmentation_pytorch_amd.runtime.bench_step import TrainerStep, bench_config
        save_dir = os.environ.get('BENCH_SAVE_DIR') or os.path.join(
            tempfile.gettempdir(), f'msp_bench_{os.getuid()}_{os.environ.get("MASTER_PORT", os.getpid())}')
        same_dev = os.environ.get('BENCH_SAME_DEVICE') == '1'
        cfg = bench_config(args.model, args.base_channel, args.batch, args.size, args.lr, total_steps,
                           args.train_images, args.val_images, save_dir,
                           device_index=dev_index if (not ddp or same_dev) else None, teacher_name=args.teacher,
                           use_graph=use_graph, dist_backend=os.environ.get('BENCH_DIST_BACKEND') if ddp else None,
                           world=world, dist_world1_bucketer=ddp)
        cfg.random_seed = args.seed
        if not cuda:
            cfg.base_workers = 0   # CPU rehearsal: batches built in-process
        step = TrainerStep(cfg, fixed=args.data == 'fixed')
    else:
        from medical_segmentation_pytorch_amd.runtime.bench_step import build_bench_step
        feed = make_feed(args, device, seed=1000 + rank) if args.data == 'augment' else None
        step = build_bench_step(impl=impl, batch=args.batch, size=args.size,
                                base_channel=args.base_channel, device=device,
                                channels_last=args.channels_last, use_graph=use_graph,
                                distributed=ddp, model_name=args.model, teacher_name=args.teacher,
                                feed=feed, total_steps=total_steps, lr=args.lr * world)

    t_w = time.perf_counter()
    if rank == 0:   # heartbeat: MIOpen's first-call kernel search (eager impl) can be silent for minutes
        import threading

        def _beat():
            while True:
                time.sleep(30)
                print(f'[bench] alive {time.perf_counter() - t_w:.0f}s', file=sys.stderr, flush=True)
        threading.Thread(target=_beat, daemon=True).start()
    for i in range(args.warmup):
        step()
        if rank == 0:   # progress on stderr (first eager steps can spend minutes in MIOpen's kernel search)
            sync()
            print(f'[bench] warmup {i + 1}/{args.warmup} done at {time.perf_counter() - t_w:.1f}s', file=sys.stderr,
                  flush=True)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    ms = elapsed / args.steps * 1e3
    global_batch = args.batch * world
    value = global_batch * args.steps / elapsed
    dice = fg_dice = None
    if args.val_images > 0 and hasattr(step, 'validate') and args.model in ('ducknet', 'unet'):
        # the trainer's own validation (EMA model = live weights with use_ema=False, MyConfig) after this
        # run's W+K steps; every rank takes part (the confusion matrix is all-reduced)
        dice, fg_dice = step.validate()
    elif args.val_images > 0 and rank == 0 and args.model in ('ducknet', 'unet') and hasattr(step, 'ema_model'):
        dice, fg_dice = val_dice(step.ema_model, args, device, seed=99)
    # The reference publishes no throughput; the baseline is the in-house "reference speed"
    # of BASELINE.md's protocol: the same step in eager PyTorch-ROCm on one MI355X at its best measured
    # config (profiles/eager_reference_speed.json), times the GPU count (weak scaling; generous to the
    # eager side, whose DDP+SyncBN would scale sub-linearly).
    comm = None
    if dist is not None and args.comm_steps > 0 and impl == 'fused' and not use_graph:
        comm = comm_evidence(step, args, dist, ms, device)
    baseline = None
    here = os.path.dirname(os.path.abspath(__file__))
    try:
        with open(os.path.join(here, 'BASELINE.json')) as f:
            baseline = (json.load(f).get('published') or {}).get('images_per_sec')
    except Exception:
        pass
    ref_key = (args.model, args.base_channel if args.model == 'ducknet' else None, args.teacher or None)
    if baseline is None and args.size == 352 and ref_key in EAGER_REFERENCE_CONFIGS:
        per_gpu = EAGER_REFERENCE_CONFIGS[ref_key]
        if ref_key == ('ducknet', 17, None):
            try:   # a re-measured value, where the profiles directory is present
                with open(os.path.join(here, 'profiles', 'eager_reference_speed.json')) as f:
                    per_gpu = json.load(f)['images_per_sec_per_gpu']
            except Exception:
                pass
        baseline = per_gpu * world
    if rank == 0:
        print(json.dumps({
            'metric': ('images/sec (whole node) + val Dice, DUCKNet-17 352x352 at 1/2/4/8 MI355X'
                       if args.model == 'ducknet' and args.base_channel == 17 and not args.teacher and args.size == 352
                       else f'images/sec (whole node), {model_label(args)} {args.size}x{args.size}'),
            'value': round(value, 2), 'unit': 'images/sec', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': round(value / baseline, 3) if baseline else None,
            'dtype': 'bf16' if cuda else 'fp32',
            'data': (f'synthetic {args.size}x{args.size} polyp images/masks, random-init weights; ' +
                     ('CPU rehearsal (no GPU): host DataLoader, eager engine over gloo' if not cuda else
                      ('fresh batch per step from the trainer\'s DeviceAugLoader (HBM-resident split, MyConfig '
                       'augmentation on the GPU) inside the timed loop' if impl == 'fused' else
                       'fresh GPU-augmented batch per step (MyConfig aug) inside the timed loop')
                      if args.data == 'augment' else 'one resident batch replayed')),
            'val_dice': None if dice is None else round(dice, 4),
            'val_dice_fg': None if fg_dice is None else round(fg_dice, 4),
            'val_dice_note': (f'macro Dice (reference metric) on {args.val_images} held-out synthetic images after '
                              f'this run\'s {args.warmup + args.steps} training steps, by SegTrainer.validate (EMA model); '
                              'converged accuracy: tools/train_synthetic.py') if dice is not None else None,
            **({'comm': comm} if comm is not None else {}),
            'config': {'model': model_label(args), 'global_batch': global_batch,
                       'per_gpu_batch': args.batch, 'seq_len': args.size * args.size,
                       'step': 'SegTrainer.train_step' if impl == 'fused' else 'eager reference step',
                       'image_size': args.size, 'parallelism': f'dp{world}', 'impl': impl,
                       'optimizer': 'adam', 'loss': 'ce', 'syncbn': world > 1, 'hipgraph': use_graph,
                       'peak_mem_gib': round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)
                       if torch.cuda.is_available() else None,
                       'peak_reserved_gib': round(torch.cuda.max_memory_reserved() / 2 ** 30, 1)
                       if torch.cuda.is_available() else None},
        }), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if save_dir is not None and rank == 0 and not os.environ.get('BENCH_SAVE_DIR'):
        import shutil
        shutil.rmtree(save_dir, ignore_errors=True)


if __name__ == '__main__':
    main()
