"""User config -- mirrors reference ``configs/my_config.py:4-40``.

One deliberate change: the reference ships ``num_class = 1`` together with
``loss_type = 'ce'``, which crashes on the first polyp pixel.  Here ``num_class = 2`` (the value the
published numbers were trained with, ``base_config.py:121-122``); ``num_class = 1`` is still
supported and selects the sigmoid/BCE(+Dice) path.
"""
from .base_config import BaseConfig


class MyConfig(BaseConfig):
    def __init__(self):
        super().__init__()
        # Dataset
        self.dataset = 'polyp'
        self.subset = 'kvasir'
        self.data_root = '/path/to/your/dataset'
        self.use_test_set = True
        self.num_channel = 3
        self.num_class = 2

        # Model
        self.model = 'unet'
        self.base_channel = 32
        self.model_path = 'save/best.pth'   # used by app.py

        # Training
        self.total_epoch = 400
        self.train_bs = 16
        self.loss_type = 'ce'
        self.optimizer_type = 'adam'

        # Validating
        self.metrics = ['dice', 'iou']
        self.val_bs = 1

        # Training setting
        self.use_ema = False
        self.logger_name = 'medseg_trainer'

        # Augmentation
        self.crop_size = 320
        self.randscale = [-0.5, 1.0]
        self.brightness = 0.5
        self.contrast = 0.5
        self.saturation = 0.5
        self.h_flip = 0.5
        self.v_flip = 0.5
