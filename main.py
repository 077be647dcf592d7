"""Train / predict entry point -- reference ``main.py:8-21``.

    python main.py                                   # single process (1 GPU, or CPU)
    torchrun --nproc_per_node=8 main.py              # one process per MI355X (RCCL over xGMI)
    python main.py --model ducknet --base_channel 17 --dataset synthetic --crop_size 352 ...

Command-line overrides are ON here (the reference ships them commented out, ``main.py:14``).
"""
import warnings

from medical_segmentation_pytorch_amd.configs import MyConfig, load_parser
from medical_segmentation_pytorch_amd.core import SegTrainer

warnings.filterwarnings('ignore')

if __name__ == '__main__':
    config = MyConfig()
    config.init_dependent_config()
    config = load_parser(config)
    trainer = SegTrainer(config)
    if config.is_testing:
        trainer.predict(config)
    else:
        trainer.run(config)
