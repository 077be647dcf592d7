"""U-Net (Ronneberger et al.) with the reference's layer plan -- ``models/unet.py:14-77``.

Encoder stage = ConvBlock (2 x 3x3 ConvBNAct) + MaxPool2d(3, 2, 1) (``unet.py:45-55``); decoder stage =
DeConvBNAct (3x3/s2 transposed conv, bias) -> concat skip -> ConvBlock (``unet.py:58-69``); bias-free
1x1 head.  H and W must be divisible by 16.  ``base_channel=32`` -> 8.634M params.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .modules import ConvBNAct, DeConvBNAct, conv1x1


class ConvBlock(nn.Sequential):
    def __init__(self, in_channels, out_channels, act_type='relu'):
        super().__init__(ConvBNAct(in_channels, out_channels, 3, act_type=act_type, inplace=True),
                         ConvBNAct(out_channels, out_channels, 3, act_type=act_type, inplace=True))


class DownsampleBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type='relu'):
        super().__init__()
        self.conv = ConvBlock(in_channels, out_channels, act_type)
        self.pool = nn.MaxPool2d(3, 2, 1)

    def forward(self, x):
        feat = self.conv(x)
        return self.pool(feat), feat


class UpsampleBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type='relu'):
        super().__init__()
        self.up = DeConvBNAct(in_channels, out_channels, act_type=act_type)
        self.conv = ConvBlock(in_channels, out_channels, act_type)

    def forward(self, x, residual):
        return self.conv(torch.cat([self.up(x), residual], dim=1))


class UNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, base_channel=64, act_type='relu'):
        super().__init__()
        b = base_channel
        self.base_channel = b
        self.num_class = num_class
        widths = [n_channel, b, 2 * b, 4 * b, 8 * b]
        for i in range(1, 5):
            setattr(self, f'down_stage{i}', DownsampleBlock(widths[i - 1], widths[i], act_type))
        self.mid_stage = ConvBlock(8 * b, 16 * b, act_type)
        for i in range(4, 0, -1):
            setattr(self, f'up_stage{i}', UpsampleBlock(2 * widths[i], widths[i], act_type))
        self.seg_head = conv1x1(b, num_class)

    def forward(self, x):
        skips = []
        for i in range(1, 5):
            x, feat = getattr(self, f'down_stage{i}')(x)
            skips.append(feat)
        x = self.mid_stage(x)
        for i in range(4, 0, -1):
            x = getattr(self, f'up_stage{i}')(x, skips[i - 1])
        return self.seg_head(x)
