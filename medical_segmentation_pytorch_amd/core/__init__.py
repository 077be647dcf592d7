from .base_trainer import BaseTrainer  # noqa: F401
from .loss import get_loss_fn, kd_loss_fn  # noqa: F401
from .seg_trainer import SegTrainer  # noqa: F401
