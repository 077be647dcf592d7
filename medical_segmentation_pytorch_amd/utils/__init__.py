"""Runtime glue (reference ``utils/__init__.py:1-7`` star-exports)."""
from .metrics import Dice, JaccardIndex, get_seg_metrics  # noqa: F401
from .model_ema import ModelEmaV2, get_ema_model  # noqa: F401
from .optimizer import FusedOptimizer, get_optimizer  # noqa: F401
from .parallel import (FusedModel, de_parallel, destroy_ddp_process, is_parallel, parallel_model,  # noqa: F401
                       sampler_set_epoch, set_device, use_fused)
from .scheduler import get_scheduler  # noqa: F401
from .transforms import Scale, SegAugment, normalize_to_tensor  # noqa: F401
from .utils import (get_colormap, get_logger, get_writer, log_config, mkdir, save_config,  # noqa: F401
                    set_seed)
