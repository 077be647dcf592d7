"""Typed command-line overrides -- reference ``configs/parser.py:4-195``.

Same flag names and the same ``store_true`` / ``store_false`` semantics as the reference.  Fixed
(SURVEY Appendix E.4): list/tuple flags take space-separated values instead of being split into
characters, ``--reduction`` is a string, assignment is ``setattr`` (no ``exec``), ``--dataroot`` also
sets ``data_root``, and ``load_parser`` re-runs the derived-field pass so ``--crop_size`` propagates.
"""
from __future__ import annotations

import argparse


def _flag(parser, name, **kw):
    parser.add_argument(f'--{name}', default=None, **kw)


def get_parser():
    p = argparse.ArgumentParser(description='MI355X-native medical segmentation trainer')
    # Dataset
    _flag(p, 'dataset', type=str, choices=['polyp', 'synthetic'])
    _flag(p, 'subset', type=str)
    _flag(p, 'dataroot', type=str)
    _flag(p, 'data_root', type=str)
    _flag(p, 'num_class', type=int)
    _flag(p, 'ignore_index', type=int)
    _flag(p, 'num_channel', type=int)
    _flag(p, 'use_test_set', action='store_true')
    # Model
    _flag(p, 'model', type=str, choices=['unet', 'ducknet', 'smp'])
    _flag(p, 'encoder', type=str)
    _flag(p, 'decoder', type=str, choices=['deeplabv3', 'deeplabv3p', 'fpn', 'linknet', 'manet',
                                           'pan', 'pspnet', 'unet', 'unetpp'])
    _flag(p, 'encoder_weights', type=str)
    _flag(p, 'base_channel', type=int)
    # Training
    _flag(p, 'total_epoch', type=int)
    _flag(p, 'base_lr', type=float)
    _flag(p, 'train_bs', type=int)
    _flag(p, 'use_aux', action='store_true')
    _flag(p, 'aux_coef', type=float, nargs='+')
    # Validating
    _flag(p, 'metrics', type=str, nargs='+')
    _flag(p, 'val_bs', type=int)
    _flag(p, 'begin_val_epoch', type=int)
    _flag(p, 'val_interval', type=int)
    _flag(p, 'val_img_stride', type=int)
    # Testing
    _flag(p, 'is_testing', action='store_true')
    _flag(p, 'test_bs', type=int)
    _flag(p, 'test_data_folder', type=str)
    _flag(p, 'colormap', type=str, choices=['random', 'custom'])
    _flag(p, 'colormap_path', type=str)
    _flag(p, 'save_mask', action='store_false')
    _flag(p, 'blend_prediction', action='store_false')
    _flag(p, 'blend_alpha', type=float)
    # Loss
    _flag(p, 'loss_type', type=str, choices=['ce', 'ohem', 'bce', 'dice', 'bce_dice', 'ce_dice'])
    _flag(p, 'class_weights', type=float, nargs='+')
    _flag(p, 'ohem_thrs', type=float)
    _flag(p, 'reduction', type=str, choices=['mean', 'sum', 'none'])
    # Scheduler
    _flag(p, 'lr_policy', type=str, choices=['cos_warmup', 'linear', 'step'])
    _flag(p, 'warmup_epochs', type=int)
    _flag(p, 'step_size', type=int)
    # Optimizer
    _flag(p, 'optimizer_type', type=str, choices=['sgd', 'adam', 'adamw'])
    _flag(p, 'momentum', type=float)
    _flag(p, 'weight_decay', type=float)
    # Monitoring
    _flag(p, 'save_ckpt', action='store_false')
    _flag(p, 'save_dir', type=str)
    _flag(p, 'use_tb', action='store_false')
    _flag(p, 'tb_log_dir', type=str)
    _flag(p, 'ckpt_name', type=str)
    # Training setting
    _flag(p, 'amp_training', action='store_true')
    _flag(p, 'resume_training', action='store_false')
    _flag(p, 'load_ckpt', action='store_false')
    _flag(p, 'load_ckpt_path', type=str)
    _flag(p, 'base_workers', type=int)
    _flag(p, 'random_seed', type=int)
    _flag(p, 'use_ema', action='store_true')
    # Augmentation
    _flag(p, 'crop_size', type=int)
    _flag(p, 'crop_h', type=int)
    _flag(p, 'crop_w', type=int)
    _flag(p, 'scale', type=float)
    _flag(p, 'randscale', type=float, nargs='+')
    _flag(p, 'brightness', type=float)
    _flag(p, 'contrast', type=float)
    _flag(p, 'saturation', type=float)
    _flag(p, 'h_flip', type=float)
    _flag(p, 'v_flip', type=float)
    # DDP
    _flag(p, 'synBN', action='store_false')
    _flag(p, 'destroy_ddp_process', action='store_false')
    _flag(p, 'local_rank', type=int)
    # Knowledge distillation
    _flag(p, 'kd_training', action='store_true')
    _flag(p, 'teacher_ckpt', type=str)
    _flag(p, 'teacher_model', type=str)
    _flag(p, 'teacher_encoder', type=str)
    _flag(p, 'teacher_decoder', type=str)
    _flag(p, 'kd_loss_type', type=str, choices=['kl_div', 'mse'])
    _flag(p, 'kd_loss_coefficient', type=float)
    _flag(p, 'kd_temperature', type=float)
    # MI355X engine
    _flag(p, 'engine', type=str, choices=['auto', 'fused', 'eager'])
    _flag(p, 'amp_dtype', type=str, choices=['bf16', 'fp16'])
    _flag(p, 'use_graph', action='store_false')
    _flag(p, 'bucket_cap_mb', type=float)
    _flag(p, 'grad_compress', type=str, choices=['bf16'])
    _flag(p, 'synthetic_data', action='store_true')
    _flag(p, 'synthetic_num', type=int, nargs=3)
    _flag(p, 'synthetic_size', type=int)
    _flag(p, 'bucketer_world1', action='store_true')
    _flag(p, 'no_graph_collectives', action='store_false', dest='graph_collectives')
    _flag(p, 'syncbn_comm', type=str, choices=['auto', 'ipc', 'rccl'])
    _flag(p, 'lr_scale', type=str, choices=['reference', 'sqrt', 'linear'])
    _flag(p, 'lr_ref_batch', type=int)
    _flag(p, 'accum_steps', type=int)
    _flag(p, 'val_fp32', action='store_true')
    _flag(p, 'gpu_augment', action='store_false')
    _flag(p, 'trace', action='store_true')
    _flag(p, 'watchdog_timeout_s', type=float)
    _flag(p, 'dist_timeout_min', type=float)
    _flag(p, 'graph_warmup', type=int)
    _flag(p, 'log_interval', type=int)
    _flag(p, 'no_progress_bar', action='store_true')
    _flag(p, 'dist_backend', type=str, choices=['nccl', 'gloo'])
    _flag(p, 'num_workers_cap', action='store_false', dest='cap_workers')
    return p


def load_parser(config, argv=None):
    args, _unknown = get_parser().parse_known_args(argv)
    for key, value in vars(args).items():
        if value is None:
            continue
        if key in ('aux_coef', 'class_weights', 'randscale') and isinstance(value, list):
            value = value if len(value) > 1 or key != 'randscale' else value[0]
        setattr(config, key, value)
        if key == 'dataroot':
            config.data_root = value
        if key == 'crop_size':
            config.crop_h = config.crop_w = value
        if key == 'no_progress_bar':
            config.progress_bar = not value
        if key == 'synthetic_num':
            config.synthetic_num = tuple(value)
    if getattr(config, 'dataset', None) == 'synthetic':
        config.dataset, config.synthetic_data = 'polyp', True
    return config.init_dependent_config()
