"""Configuration object with the reference's field names -- ``configs/base_config.py:5-123``.

Every default of the reference ``BaseConfig`` is kept (Appendix A of SURVEY.md).  Additions are the
MI355X engine knobs at the bottom (``engine``, ``use_graph``, ``bucket_cap_mb`` ...) which old
configs simply do not set.  ``init_dependent_config`` derives the same fields as the reference
(``base_config.py:106-123``) and, unlike it, may be re-run after CLI overrides
(SURVEY Appendix E.4): derived fields are only filled when still unset.
"""
from __future__ import annotations

import os


class BaseConfig:
    def __init__(self):
        # Dataset
        self.dataset = None
        self.subset = None
        self.dataroot = None
        self.data_root = None          # field read by the polyp dataset (reference polyp.py:14)
        self.num_class = -1
        self.ignore_index = 255
        self.num_channel = None
        self.use_test_set = False

        # Model
        self.model = None
        self.encoder = None
        self.decoder = None
        self.encoder_weights = 'imagenet'
        self.base_channel = None

        # Training
        self.total_epoch = 200
        self.base_lr = 0.01
        self.train_bs = 16             # per GPU
        self.use_aux = False
        self.aux_coef = None

        # Validating
        self.metrics = ['dice']        # the first one drives best-checkpoint selection
        self.val_bs = 16
        self.begin_val_epoch = 0
        self.val_interval = 1
        self.val_img_stride = 1

        # Testing
        self.is_testing = False
        self.test_bs = 16
        self.test_data_folder = None
        self.colormap = 'random'
        self.colormap_path = None
        self.save_mask = True
        self.blend_prediction = True
        self.blend_alpha = 0.3

        # Loss
        self.loss_type = 'ce'
        self.class_weights = None
        self.ohem_thrs = 0.7
        self.reduction = 'mean'

        # Scheduler
        self.lr_policy = 'cos_warmup'
        self.warmup_epochs = 3
        self.step_size = None          # reference StepLR needs it but never defines it (Appendix E.3)

        # Optimizer
        self.optimizer_type = 'sgd'
        self.momentum = 0.9
        self.weight_decay = 1e-4

        # Monitoring
        self.save_ckpt = True
        self.save_dir = 'save'
        self.use_tb = True
        self.tb_log_dir = None
        self.ckpt_name = None
        self.logger_name = None

        # Training setting
        self.amp_training = False
        self.resume_training = True
        self.load_ckpt = True
        self.load_ckpt_path = None
        self.base_workers = 8
        self.random_seed = 1
        self.use_ema = False

        # Augmentation
        self.crop_size = 512
        self.crop_h = None
        self.crop_w = None
        self.scale = 1.0
        self.randscale = 0.0
        self.brightness = 0.0
        self.contrast = 0.0
        self.saturation = 0.0
        self.h_flip = 0.0
        self.v_flip = 0.0

        # DDP
        self.synBN = True
        self.destroy_ddp_process = True
        self.local_rank = int(os.getenv('LOCAL_RANK', -1))
        self.main_rank = self.local_rank in [-1, 0]

        # Knowledge distillation
        self.kd_training = False
        self.teacher_ckpt = ''
        self.teacher_model = 'smp'
        self.teacher_encoder = None
        self.teacher_decoder = None
        self.kd_loss_type = 'kl_div'
        self.kd_loss_coefficient = 1.0
        self.kd_temperature = 4.0

        # ---- MI355X engine knobs (new; absent from the reference) ----
        self.engine = 'auto'           # 'auto' | 'fused' (HIP kernels) | 'eager' (stock torch ops)
        self.amp_dtype = 'bf16'        # CDNA4 autocast dtype when amp_training: 'bf16' | 'fp16'
        self.use_graph = True          # capture the static-shape train step in a hipGraph
        self.eager_channels_last = True   # eager engine on a GPU: channels-last activations (MIOpen NHWC
                                          # kernels; 1.8x the NCHW step on MI355X, profiles/r02/eager_sweep)
        self.bucket_cap_mb = 64        # gradient bucket size for the RCCL all-reduce
        self.grad_compress = None      # None | 'bf16' all-reduce compression
        self.lr_scale = 'reference'    # lr vs batch: 'reference' (x gpu_num) | 'sqrt' | 'linear' in
                                       # global_batch / lr_ref_batch (utils/optimizer.lr_batch_factor)
        self.lr_ref_batch = 16         # the batch base_lr is tuned for (MyConfig train_bs)
        self.accum_steps = 1           # gradient accumulation: micro-batches per optimizer step (DDP averaging
                                       # semantics: global batch = train_bs x gpu_num x accum_steps; BN
                                       # statistics per micro-batch, as torch DDP + no_sync)
        self.syncbn_comm = 'rccl'      # SyncBN statistic exchange: 'rccl' | 'auto' (IPC peer-memory kernel on one
                                       # node after a self-test, RCCL otherwise) | 'ipc'  (env MSP_SYNCBN_COMM
                                       # overrides; IPC is opt-in until a cross-GPU run of it is recorded)
        self.gpu_augment = True        # run augmentation on the GPU over an HBM-resident dataset
        self.dist_backend = None       # None -> 'nccl' (RCCL) on GPU, 'gloo' on CPU
        self.log_interval = 50         # device-side loss accumulation, host sync every N iters
        self.ckpt_extra_state = True   # also save scaler/EMA/RNG (extra keys; old readers ignore)
        self.synthetic_data = False    # generate a synthetic polyp set when data_root is missing
        self.synthetic_num = (64, 16, 16)
        self.synthetic_size = 352
        self.cap_workers = True        # cap DataLoader workers at the host CPU count (ref: gpu_num*base_workers)
        self.teacher_base_channel = None
        self.graph_warmup = 3          # eager iterations before the hipGraph capture
        self.bucketer_world1 = False   # attach the RCCL gradient bucketer at world size 1 too (bench --ddp)
        self.graph_collectives = True  # capture a step that issues torch.distributed collectives (gradient
                                       # buckets, SyncBN over RCCL) in the hipGraph too (RCCL calls are graph
                                       # nodes; tools/dev/graph_rccl_probe.py); False: such steps run eagerly
        self.val_fp32 = False          # validate the EMA model in fp32 eager PyTorch exactly as the reference
                                       # (core/seg_trainer.py:114); False: the bf16 fused executor (fast)
        self.progress_bar = True
        self.trace = False             # roctx ranges around step phases + per-phase HIP-event timing
        self.watchdog_timeout_s = 0    # >0: dump stacks + exit(75) after this long without a step
        self.dist_timeout_min = 30     # process-group timeout (a dead peer errors instead of hanging)
        self.dist_group = None         # process sub-group (concurrent HPO trials); None = WORLD
        self.device_index = None       # explicit GPU index: single-device run without DataParallel scaling
                                       # (bench.py), or every DDP rank on that one device (gloo rehearsal)

    # ------------------------------------------------------------------
    def init_dependent_config(self):
        """Derive dependent fields (reference base_config.py:106-123).  Fields this pass derived
        itself are re-derived on a later call (after CLI overrides); user-set values are kept."""
        assert len(self.metrics) > 0
        auto = getattr(self, '_auto_derived', set())

        def derive(name, value, cond):
            if getattr(self, name) is None or name in auto:
                if cond:
                    setattr(self, name, value)
                    auto.add(name)

        derive('load_ckpt_path', f'{self.save_dir}/last.pth', not self.is_testing)
        derive('tb_log_dir', f'{self.save_dir}/tb_logs/', True)
        derive('crop_h', self.crop_size, True)
        derive('crop_w', self.crop_size, True)
        if self.data_root is None and self.dataroot is not None:
            self.data_root = self.dataroot
        if self.dataroot is None and self.data_root is not None:
            self.dataroot = self.data_root
        if self.logger_name is None:
            self.logger_name = 'seg_trainer'
        if self.dataset in ('polyp', 'synthetic'):
            self.num_class = 2 if self.num_class == -1 else self.num_class
            self.num_channel = 3 if self.num_channel is None else self.num_channel
        self._auto_derived = auto
        return self

    def to_dict(self):
        return {k: v for k, v in vars(self).items() if not k.startswith('_')}
