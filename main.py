"""Train / predict entry point -- reference ``main.py:8-21``.

    python main.py                                   # 1 GPU / CPU: one process; N GPUs: N workers, one per
                                                     # GPU, with DataParallel's global batch and lr
                                                     # (utils/launch.py; reference utils/parallel.py:24-42)
    torchrun --nproc_per_node=8 main.py              # one process per MI355X (RCCL over xGMI)
    python main.py --model ducknet --base_channel 17 --dataset synthetic --crop_size 352 ...

Command-line overrides are ON here (the reference ships them commented out, ``main.py:14``).
"""
import warnings

from medical_segmentation_pytorch_amd.configs import MyConfig, load_parser
from medical_segmentation_pytorch_amd.core import SegTrainer
from medical_segmentation_pytorch_amd.utils.launch import apply_dp_semantics, maybe_spawn_workers

warnings.filterwarnings('ignore')

if __name__ == '__main__':
    config = MyConfig()
    config.init_dependent_config()
    config = load_parser(config)
    if not config.is_testing:   # predict is single-process (reference core/seg_trainer.py:149-150)
        maybe_spawn_workers()   # launcher-less multi-GPU run: one worker per GPU (no GPU call made yet)
    apply_dp_semantics(config)
    trainer = SegTrainer(config)
    if config.is_testing:
        trainer.predict(config)
    else:
        trainer.run(config)
