import pytest
from medical_segmentation_pytorch_amd.configs import BaseConfig, MyConfig, OptunaConfig, load_parser


def test_defaults_match_reference():
    c = BaseConfig()
    assert (c.total_epoch, c.base_lr, c.train_bs, c.val_bs) == (200, 0.01, 16, 16)
    assert (c.loss_type, c.ohem_thrs, c.lr_policy, c.warmup_epochs) == ('ce', 0.7, 'cos_warmup', 3)
    assert (c.optimizer_type, c.momentum, c.weight_decay) == ('sgd', 0.9, 1e-4)
    assert c.synBN and c.resume_training and c.load_ckpt and not c.use_ema and c.ignore_index == 255
    assert (c.kd_loss_type, c.kd_loss_coefficient, c.kd_temperature) == ('kl_div', 1.0, 4.0)


def test_dependent_fields():
    c = MyConfig().init_dependent_config()
    assert c.load_ckpt_path == 'save/last.pth' and c.tb_log_dir == 'save/tb_logs/'
    assert c.crop_h == c.crop_w == 320 and c.num_class == 2 and c.num_channel == 3


def test_parser_overrides_and_rederive():
    c = MyConfig().init_dependent_config()
    c = load_parser(c, ['--save_dir', 'runs/x', '--crop_size', '352', '--randscale', '-0.5', '1.0',
                        '--metrics', 'dice', 'iou', '--reduction', 'mean', '--use_tb', '--model', 'ducknet',
                        '--base_channel', '17', '--class_weights', '1', '2'])
    assert c.save_dir == 'runs/x' and c.load_ckpt_path == 'runs/x/last.pth' and c.tb_log_dir == 'runs/x/tb_logs/'
    assert c.crop_h == c.crop_w == 352
    assert c.randscale == [-0.5, 1.0] and c.metrics == ['dice', 'iou'] and c.reduction == 'mean'
    assert c.use_tb is False            # store_false flips a default-True boolean (reference semantics)
    assert c.model == 'ducknet' and c.base_channel == 17 and c.class_weights == [1.0, 2.0]


def test_user_set_paths_are_kept():
    c = MyConfig()
    c.load_ckpt_path = 'mine.pth'
    c.init_dependent_config()
    c = load_parser(c, ['--save_dir', 'other'])
    assert c.load_ckpt_path == 'mine.pth'


class _Trial:
    def suggest_categorical(self, name, choices):
        return choices[-1]

    def suggest_float(self, name, lo, hi, log=False):
        return hi

    def suggest_int(self, name, lo, hi):
        return hi


def test_optuna_trial_params():
    c = OptunaConfig().init_dependent_config()
    c.get_trial_params(_Trial())
    assert c.randscale[0] <= 0 <= c.randscale[1]
    assert c.optimizer_type in ('sgd', 'adam', 'adamw') and c.loss_type in ('ohem', 'ce')


@pytest.mark.parametrize('name,key', [('smp-resnet101', 'unet'), ('smp-fpn-resnet101', 'fpn'),
                                      ('smp-deeplabv3plus-resnet101', 'deeplabv3p'),
                                      ('smp-UnetPlusPlus-resnet34', 'unetpp'), ('smp-pspnet-resnet18', 'pspnet')])
def test_bench_config_smp_decoder_keys(tmp_path, name, key):
    """bench.py's ``smp-<decoder>-<encoder>`` names map onto the reference hub's decoder keys
    (models/__init__.py decoder_hub: DeepLabV3Plus is 'deeplabv3p', UnetPlusPlus 'unetpp')."""
    from medical_segmentation_pytorch_amd.models import decoder_hub
    from medical_segmentation_pytorch_amd.runtime.bench_step import bench_config
    cfg = bench_config(name, 17, 2, 64, 1e-3, 10, 4, 1, str(tmp_path))
    assert cfg.model == 'smp' and cfg.decoder == key and cfg.decoder in decoder_hub
    assert cfg.encoder == name.split('-')[-1]
