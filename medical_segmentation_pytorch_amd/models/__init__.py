"""Model factory -- reference ``models/__init__.py:8-62``.

``model='unet'|'ducknet'`` -> the native models (fused MI355X executor on GPU);
``model='smp'`` -> ``decoder_hub[decoder](encoder_name, encoder_weights, in_channels, classes)`` from
the native smp re-implementation (:mod:`.smp`).  ``get_teacher_model`` builds the KD teacher
(smp, ``encoder_weights=None``) and loads ``teacher_ckpt['state_dict']`` with ``weights_only=True``.
"""
from __future__ import annotations

import os

import torch

from . import smp
from .ducknet import DuckNet
from .unet import UNet

decoder_hub = {'deeplabv3': smp.DeepLabV3, 'deeplabv3p': smp.DeepLabV3Plus, 'fpn': smp.FPN,
               'linknet': smp.Linknet, 'manet': smp.MAnet, 'pan': smp.PAN, 'pspnet': smp.PSPNet,
               'unet': smp.Unet, 'unetpp': smp.UnetPlusPlus}
model_hub = {'unet': UNet, 'ducknet': DuckNet}
aux_models = []


def get_model(config):
    if config.model == 'smp':
        if config.decoder not in decoder_hub:
            raise ValueError(f'Unsupported decoder type: {config.decoder}')
        return decoder_hub[config.decoder](encoder_name=config.encoder, encoder_weights=config.encoder_weights,
                                           in_channels=config.num_channel, classes=config.num_class)
    if config.model in model_hub:
        if config.use_aux:
            raise ValueError(f'Model {config.model} does not support auxiliary heads.\n')
        return model_hub[config.model](num_class=config.num_class, n_channel=config.num_channel,
                                       base_channel=config.base_channel)
    raise NotImplementedError(f'Unsupport model type: {config.model}')


def get_teacher_model(config, device):
    if not config.kd_training:
        return None
    if not os.path.isfile(config.teacher_ckpt):
        raise ValueError(f'Could not find teacher checkpoint at path {config.teacher_ckpt}.')
    if config.teacher_model == 'smp':
        if config.teacher_decoder not in decoder_hub:
            raise ValueError(f'Unsupported teacher decoder type: {config.teacher_decoder}')
        model = decoder_hub[config.teacher_decoder](encoder_name=config.teacher_encoder, encoder_weights=None,
                                                    in_channels=config.num_channel, classes=config.num_class)
    elif config.teacher_model in model_hub:
        model = model_hub[config.teacher_model](num_class=config.num_class, n_channel=config.num_channel,
                                                base_channel=config.teacher_base_channel or config.base_channel)
    else:
        raise ValueError(f'Unsupported teacher model: {config.teacher_model}')
    ckpt = torch.load(config.teacher_ckpt, map_location='cpu', weights_only=True)
    model.load_state_dict(ckpt['state_dict'])
    del ckpt
    return model.to(device).eval()


def count_params(model):
    return sum(p.numel() for p in model.parameters())
