#!/usr/bin/env python3
"""Parameter count (and FLOPs) -- reference ``tools/get_model_infos.py:9-36``.  ``ptflops`` is not
available, so FLOPs are counted natively with forward hooks (conv / transposed conv / linear MACs x 2).
"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from medical_segmentation_pytorch_amd.configs import MyConfig, load_parser  # noqa: E402
from medical_segmentation_pytorch_amd.models import get_model  # noqa: E402


def count_flops(model, size=(352, 352), in_ch=3):
    flops = [0]

    def conv_hook(m, inp, out):
        k = m.kernel_size[0] * m.kernel_size[1] * (m.in_channels // m.groups)
        if isinstance(m, nn.ConvTranspose2d):   # every input pixel scatters Cout*kh*kw MACs
            flops[0] += 2 * inp[0][0].numel() * m.out_channels * m.kernel_size[0] * m.kernel_size[1] // m.groups
        else:
            flops[0] += 2 * out[0].numel() * k

    def lin_hook(m, inp, out):
        flops[0] += 2 * out[0].numel() * m.in_features

    hooks = []
    for m in model.modules():
        if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            hooks.append(m.register_forward_hook(conv_hook))
        elif isinstance(m, nn.Linear):
            hooks.append(m.register_forward_hook(lin_hook))
    model.eval()
    with torch.no_grad():
        model(torch.zeros(1, in_ch, *size))
    for h in hooks:
        h.remove()
    return flops[0]


def cal_model_params(config, imgw=352, imgh=352):
    model = get_model(config)
    print(f'\nModel: {config.model}\nEncoder: {config.encoder}\nDecoder: {config.decoder}')
    params = sum(p.numel() for p in model.parameters())
    print(f'Number of parameters: {params / 1e6:.2f}M')
    gflops = count_flops(model, (imgh, imgw), config.num_channel) / 1e9
    print(f'FLOPs @ {imgh}x{imgw}: {gflops:.2f} GFLOP/img (forward)\n')
    return params, gflops


if __name__ == '__main__':
    config = MyConfig()
    config.init_dependent_config()
    config = load_parser(config)
    cal_model_params(config)
