"""DUCK-Net (Dumitru et al., arXiv:2311.02239) with the reference's layer plan.

Reference parity: ``models/ducknet.py:15-179``.
  * encoder: 5 ``DownsampleBlock`` (DUCK -> 3x3/s2 ConvBNAct, plus a 2x2/s2 ConvBNAct path on the
    previous down-sampled tensor, combined by addition) ``ducknet.py:37-43,55-72``
  * bottleneck: 4 ``ResidualBlock`` ``ducknet.py:24-29``
  * decoder: 5 ``UpsampleBlock`` (nearest x2 -> + skip -> DUCK) ``ducknet.py:75-87``
  * head: bias-free 1x1 conv ``ducknet.py:35``
  * DUCK = in_bn -> 6 parallel branches on one tensor -> 6-way sum -> out_bn ``ducknet.py:113-154``;
    the separated branch uses a 1x7 / 7x1 pair (``filter_size = 6 + 1``, ``ducknet.py:114-117``).

Inputs must have H and W divisible by 32.  ``base_channel`` 17 -> 40.102M params, 34 -> 160.284M.

This module is the reference-semantics graph (CPU path, parity tests, eager baseline).  The fused
MI355X executor (:mod:`medical_segmentation_pytorch_amd.runtime.ducknet_exec`) walks the same
module tree and drives the HIP kernels with these parameters.
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F

from .modules import Activation, ConvBNAct, conv1x1


def _bn_act(channels, act_type):
    return nn.Sequential(nn.BatchNorm2d(channels), Activation(act_type))


class ResidualBlock(nn.Module):
    """``BN-act(conv1x1(x) + CBA3x3(CBA3x3(x)))`` -- ``ducknet.py:90-110``."""

    def __init__(self, in_channels, out_channels, act_type='relu'):
        super().__init__()
        self.upper_branch = conv1x1(in_channels, out_channels)
        self.lower_branch = nn.Sequential(ConvBNAct(in_channels, out_channels, 3, act_type=act_type),
                                          ConvBNAct(out_channels, out_channels, 3, act_type=act_type))
        self.bn = _bn_act(out_channels, act_type)

    def forward(self, x):
        return self.bn(self.upper_branch(x) + self.lower_branch(x))


def _chain(in_channels, out_channels, act_type, specs):
    """A Sequential of ConvBNActs; ``specs`` = [(kernel, dilation), ...]."""
    layers, c = [], in_channels
    for k, d in specs:
        layers.append(ConvBNAct(c, out_channels, k, dilation=d, act_type=act_type))
        c = out_channels
    return nn.Sequential(*layers)


def _residual_stack(in_channels, out_channels, depth, act_type):
    return nn.Sequential(*[ResidualBlock(in_channels if i == 0 else out_channels, out_channels, act_type)
                           for i in range(depth)])


class DUCK(nn.Module):
    """Six-branch multi-scale block (``ducknet.py:113-154``)."""

    def __init__(self, in_channels, out_channels, act_type='relu', filter_size=7):
        super().__init__()
        self.in_bn = _bn_act(in_channels, act_type)
        self.branch1 = _chain(in_channels, out_channels, act_type, [(3, 1), (3, 2), (3, 3)])   # widescope
        self.branch2 = _chain(in_channels, out_channels, act_type, [(3, 1), (3, 2)])           # midscope
        self.branch3 = ResidualBlock(in_channels, out_channels, act_type)
        self.branch4 = _residual_stack(in_channels, out_channels, 2, act_type)
        self.branch5 = _residual_stack(in_channels, out_channels, 3, act_type)
        self.branch6 = _chain(in_channels, out_channels, act_type,                               # separated
                              [((1, filter_size), 1), ((filter_size, 1), 1)])
        self.out_bn = _bn_act(out_channels, act_type)

    def branches(self):
        return (self.branch1, self.branch2, self.branch3, self.branch4, self.branch5, self.branch6)

    def forward(self, x):
        x = self.in_bn(x)
        total = None
        for branch in self.branches():
            y = branch(x)
            total = y if total is None else total + y
        return self.out_bn(total)


class DownsampleBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type='relu', fuse_channels=None):
        super().__init__()
        fuse_channels = in_channels if fuse_channels is None else fuse_channels
        self.duck = DUCK(in_channels, fuse_channels, act_type)
        self.conv1 = ConvBNAct(fuse_channels, out_channels, 3, 2, act_type=act_type)
        self.conv2 = ConvBNAct(in_channels, out_channels, 2, 2, act_type=act_type)

    def forward(self, x1, x2=None):
        """Returns (down-sampled DUCK path, skip, down-sampled shortcut path)."""
        shortcut = self.conv2(x1 if x2 is None else x2)
        skip = self.duck(x1)
        return self.conv1(skip), skip, shortcut


class UpsampleBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type='relu'):
        super().__init__()
        self.duck = DUCK(in_channels, out_channels, act_type)

    def forward(self, x, residual):
        x = F.interpolate(x, residual.shape[2:], mode='nearest') + residual
        return self.duck(x)


class DuckNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, base_channel=17, act_type='relu'):
        super().__init__()
        b = base_channel
        self.base_channel = b
        self.num_class = num_class
        self.down_stage1 = DownsampleBlock(n_channel, 2 * b, act_type, fuse_channels=b)
        self.down_stage2 = DownsampleBlock(2 * b, 4 * b, act_type)
        self.down_stage3 = DownsampleBlock(4 * b, 8 * b, act_type)
        self.down_stage4 = DownsampleBlock(8 * b, 16 * b, act_type)
        self.down_stage5 = DownsampleBlock(16 * b, 32 * b, act_type)
        self.mid_stage = nn.Sequential(ResidualBlock(32 * b, 32 * b, act_type),
                                       ResidualBlock(32 * b, 32 * b, act_type),
                                       ResidualBlock(32 * b, 16 * b, act_type),
                                       ResidualBlock(16 * b, 16 * b, act_type))
        self.up_stage5 = UpsampleBlock(16 * b, 8 * b, act_type)
        self.up_stage4 = UpsampleBlock(8 * b, 4 * b, act_type)
        self.up_stage3 = UpsampleBlock(4 * b, 2 * b, act_type)
        self.up_stage2 = UpsampleBlock(2 * b, b, act_type)
        self.up_stage1 = UpsampleBlock(b, b, act_type)
        self.seg_head = conv1x1(b, num_class)

    def down_stages(self):
        return [self.down_stage1, self.down_stage2, self.down_stage3, self.down_stage4, self.down_stage5]

    def up_stages(self):
        return [self.up_stage5, self.up_stage4, self.up_stage3, self.up_stage2, self.up_stage1]

    def forward(self, x):
        skips = []
        down, skip, shortcut = self.down_stage1(x)
        skips.append(skip)
        for stage in self.down_stages()[1:]:
            down, skip, shortcut = stage(down + shortcut, shortcut)
            skips.append(skip)
        x = self.mid_stage(down + shortcut)
        for stage, skip in zip(self.up_stages(), reversed(skips)):
            x = stage(x, skip)
        return self.seg_head(x)
