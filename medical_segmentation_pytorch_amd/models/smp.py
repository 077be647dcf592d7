"""Native replacement of ``segmentation_models_pytorch`` 0.3.2 as used by the reference
(``models/__init__.py:8-39``: ``decoder_hub`` x ``encoder_name``; SURVEY §2.4 "smp-UNet").

smp is not installable here, so the architectures are re-implemented with smp's module layout so
that ``state_dict`` keys are smp's (``encoder.*``, ``decoder.blocks.N.conv1.0.weight``,
``segmentation_head.0.{weight,bias}`` -- the keys ``app.py:107`` greps) and the ResNet-18 U-Net has
smp's 14.328M parameters (README ``:113``).  Encoders: torchvision-layout ResNet-18/34/50/101/152,
ResNeXt-50/101 and MobileNetV2 (the reference's dead ``models/backbone.py`` family).  ImageNet
weights cannot be downloaded: ``encoder_weights='imagenet'`` warns and keeps the random init unless
``encoder_weights`` is a path to a local state_dict (loaded with ``weights_only=True``).

Parity note: decoders other than U-Net are faithful re-implementations whose parameter counts are
"parity unpinned" (no smp install or fixture in the reference to compare against).
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------- common modules
class Conv2dReLU(nn.Sequential):
    def __init__(self, in_channels, out_channels, kernel_size, padding=0, stride=1, use_batchnorm=True):
        conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                         bias=not use_batchnorm)
        bn = nn.BatchNorm2d(out_channels) if use_batchnorm else nn.Identity()
        super().__init__(conv, bn, nn.ReLU(inplace=True))


class SegmentationHead(nn.Sequential):
    def __init__(self, in_channels, out_channels, kernel_size=3, upsampling=1):
        conv = nn.Conv2d(in_channels, out_channels, kernel_size=kernel_size, padding=kernel_size // 2)
        up = nn.UpsamplingBilinear2d(scale_factor=upsampling) if upsampling > 1 else nn.Identity()
        super().__init__(conv, up, nn.Identity())


class SeparableConv2d(nn.Sequential):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, bias=True):
        dw = nn.Conv2d(in_channels, in_channels, kernel_size, stride=stride, padding=padding, dilation=dilation,
                       groups=in_channels, bias=False)
        pw = nn.Conv2d(in_channels, out_channels, kernel_size=1, bias=bias)
        super().__init__(dw, pw)


# ----------------------------------------------------------------------------- encoders
class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = nn.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, groups=groups, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


class ResNetEncoder(nn.Module):
    """torchvision ResNet without avgpool/fc; ``forward`` returns the 6 smp feature maps."""

    def __init__(self, block, layers, out_channels, depth=5, in_channels=3, groups=1, width_per_group=64):
        super().__init__()
        self._out_channels = out_channels
        self._depth = depth
        self.inplanes = 64
        self.groups, self.base_width = groups, width_per_group
        self.conv1 = nn.Conv2d(in_channels, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], 2)
        self.layer3 = self._make_layer(block, 256, layers[2], 2)
        self.layer4 = self._make_layer(block, 512, layers[3], 2)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')

    def _make_layer(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                 nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, down, self.groups, self.base_width)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes, groups=self.groups, base_width=self.base_width)
                   for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    @property
    def out_channels(self):
        return self._out_channels[:self._depth + 1]

    def get_stages(self):
        return [nn.Identity(), nn.Sequential(self.conv1, self.bn1, self.relu),
                nn.Sequential(self.maxpool, self.layer1), self.layer2, self.layer3, self.layer4]

    def forward(self, x):
        feats = []
        for stage in self.get_stages()[:self._depth + 1]:
            x = stage(x)
            feats.append(x)
        return feats

    def make_dilated(self, output_stride):
        """smp ``make_dilated``: replace strides of the last stage(s) by dilation."""
        if output_stride == 16:
            stages, rates = [self.layer4], [2]
        elif output_stride == 8:
            stages, rates = [self.layer3, self.layer4], [2, 4]
        else:
            raise ValueError(f'output stride should be 16 or 8, got {output_stride}')
        for stage, rate in zip(stages, rates):
            for m in stage.modules():
                if isinstance(m, nn.Conv2d):
                    m.stride = (1, 1)
                    m.dilation = (rate, rate)
                    kh, kw = m.kernel_size
                    m.padding = ((kh // 2) * rate, (kw // 2) * rate)


def _inverted_residual(inp, oup, stride, expand):
    hidden = int(round(inp * expand))
    layers = []
    if expand != 1:
        layers += [nn.Conv2d(inp, hidden, 1, bias=False), nn.BatchNorm2d(hidden), nn.ReLU6(inplace=True)]
    layers += [nn.Conv2d(hidden, hidden, 3, stride, 1, groups=hidden, bias=False), nn.BatchNorm2d(hidden),
               nn.ReLU6(inplace=True), nn.Conv2d(hidden, oup, 1, bias=False), nn.BatchNorm2d(oup)]
    return nn.Sequential(*layers)


class _InvRes(nn.Module):
    def __init__(self, inp, oup, stride, expand):
        super().__init__()
        self.conv = _inverted_residual(inp, oup, stride, expand)
        self.use_res = stride == 1 and inp == oup

    def forward(self, x):
        return x + self.conv(x) if self.use_res else self.conv(x)


class MobileNetV2Encoder(nn.Module):
    """torchvision MobileNetV2 ``features`` split into the smp stages (reference models/backbone.py:39-57)."""

    def __init__(self, depth=5, in_channels=3):
        super().__init__()
        self._depth = depth
        self._out_channels = (in_channels, 16, 24, 32, 96, 1280)
        cfg = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
               (6, 320, 1, 1)]
        feats = [nn.Sequential(nn.Conv2d(in_channels, 32, 3, 2, 1, bias=False), nn.BatchNorm2d(32),
                               nn.ReLU6(inplace=True))]
        c = 32
        for t, ch, n, s in cfg:
            for i in range(n):
                feats.append(_InvRes(c, ch, s if i == 0 else 1, t))
                c = ch
        feats.append(nn.Sequential(nn.Conv2d(c, 1280, 1, bias=False), nn.BatchNorm2d(1280), nn.ReLU6(inplace=True)))
        self.features = nn.Sequential(*feats)

    @property
    def out_channels(self):
        return self._out_channels[:self._depth + 1]

    def get_stages(self):
        f = self.features
        return [nn.Identity(), f[:2], f[2:4], f[4:7], f[7:14], f[14:]]

    def forward(self, x):
        out = []
        for stage in self.get_stages()[:self._depth + 1]:
            x = stage(x)
            out.append(x)
        return out

    def make_dilated(self, output_stride):
        """smp ``replace_strides_with_dilation`` over the last stage(s) (DeepLabV3/V3+, PAN)."""
        stages = self.get_stages()
        if output_stride == 16:
            plan = [(stages[5], 2)]
        elif output_stride == 8:
            plan = [(stages[4], 2), (stages[5], 4)]
        else:
            raise ValueError(f'output stride should be 16 or 8, got {output_stride}')
        for stage, rate in plan:
            for m in stage.modules():
                if isinstance(m, nn.Conv2d):
                    m.stride = (1, 1)
                    m.dilation = (rate, rate)
                    kh, kw = m.kernel_size
                    m.padding = ((kh // 2) * rate, (kw // 2) * rate)


ENCODERS = {
    'resnet18': (BasicBlock, [2, 2, 2, 2], (3, 64, 64, 128, 256, 512), {}),
    'resnet34': (BasicBlock, [3, 4, 6, 3], (3, 64, 64, 128, 256, 512), {}),
    'resnet50': (Bottleneck, [3, 4, 6, 3], (3, 64, 256, 512, 1024, 2048), {}),
    'resnet101': (Bottleneck, [3, 4, 23, 3], (3, 64, 256, 512, 1024, 2048), {}),
    'resnet152': (Bottleneck, [3, 8, 36, 3], (3, 64, 256, 512, 1024, 2048), {}),
    'resnext50_32x4d': (Bottleneck, [3, 4, 6, 3], (3, 64, 256, 512, 1024, 2048),
                        {'groups': 32, 'width_per_group': 4}),
    'resnext101_32x8d': (Bottleneck, [3, 4, 23, 3], (3, 64, 256, 512, 1024, 2048),
                         {'groups': 32, 'width_per_group': 8}),
}


def get_encoder(name, in_channels=3, depth=5, weights=None, output_stride=32):
    if name == 'mobilenet_v2':
        enc = MobileNetV2Encoder(depth, in_channels)
    elif name in ENCODERS:
        block, layers, oc, kw = ENCODERS[name]
        oc = (in_channels,) + tuple(oc[1:])
        enc = ResNetEncoder(block, layers, oc, depth, in_channels, **kw)
    else:
        raise KeyError(f'Wrong encoder name `{name}`, supported: {sorted(list(ENCODERS) + ["mobilenet_v2"])}')
    if weights is not None:
        if isinstance(weights, str) and os.path.isfile(weights):
            sd = torch.load(weights, map_location='cpu', weights_only=True)
            sd = sd.get('state_dict', sd)
            sd = {k: v for k, v in sd.items() if not k.startswith('fc.')}
            enc.load_state_dict(sd, strict=False)
        else:
            warnings.warn(f'encoder_weights={weights!r}: no network access to download pretrained weights; '
                          'the encoder keeps its random initialisation (pass a local .pth path to load).')
    if output_stride != 32:
        enc.make_dilated(output_stride)
    return enc


# ----------------------------------------------------------------------------- decoders
class UnetDecoderBlock(nn.Module):
    def __init__(self, in_channels, skip_channels, out_channels, use_batchnorm=True):
        super().__init__()
        self.conv1 = Conv2dReLU(in_channels + skip_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm)
        self.attention1 = nn.Identity()
        self.conv2 = Conv2dReLU(out_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm)
        self.attention2 = nn.Identity()

    def forward(self, x, skip=None):
        x = F.interpolate(x, scale_factor=2, mode='nearest')
        if skip is not None:
            x = self.attention1(torch.cat([x, skip], dim=1))
        return self.attention2(self.conv2(self.conv1(x)))


class UnetDecoder(nn.Module):
    def __init__(self, encoder_channels, decoder_channels=(256, 128, 64, 32, 16), use_batchnorm=True):
        super().__init__()
        enc = list(encoder_channels[1:])[::-1]
        in_ch = [enc[0]] + list(decoder_channels[:-1])
        skip_ch = enc[1:] + [0]
        self.center = nn.Identity()
        self.blocks = nn.ModuleList([UnetDecoderBlock(i, s, o, use_batchnorm)
                                     for i, s, o in zip(in_ch, skip_ch, decoder_channels)])

    def forward(self, *features):
        feats = features[1:][::-1]
        x = self.center(feats[0])
        skips = feats[1:]
        for i, block in enumerate(self.blocks):
            x = block(x, skips[i] if i < len(skips) else None)
        return x


class UnetPlusPlusDecoder(nn.Module):
    def __init__(self, encoder_channels, decoder_channels=(256, 128, 64, 32, 16), use_batchnorm=True):
        super().__init__()
        enc = list(encoder_channels[1:])[::-1]
        self.in_channels = [enc[0]] + list(decoder_channels[:-1])
        self.skip_channels = enc[1:] + [0]
        self.out_channels = list(decoder_channels)
        self.center = nn.Identity()
        blocks = {}
        for layer_idx in range(len(self.in_channels) - 1):
            for depth_idx in range(layer_idx + 1):
                if depth_idx == 0:
                    in_ch = self.in_channels[layer_idx]
                    skip_ch = self.skip_channels[layer_idx] * (layer_idx + 1)
                    out_ch = self.out_channels[layer_idx]
                else:
                    out_ch = self.skip_channels[layer_idx]
                    skip_ch = self.skip_channels[layer_idx] * (layer_idx + 1 - depth_idx)
                    in_ch = self.skip_channels[layer_idx - 1]
                blocks[f'x_{depth_idx}_{layer_idx}'] = UnetDecoderBlock(in_ch, skip_ch, out_ch, use_batchnorm)
        last = len(self.in_channels) - 1
        blocks[f'x_0_{last}'] = UnetDecoderBlock(self.in_channels[-1], 0, self.out_channels[-1], use_batchnorm)
        self.blocks = nn.ModuleDict(blocks)
        self.depth = last

    def forward(self, *features):
        feats = features[1:][::-1]
        dense = {}
        for layer_idx in range(len(self.in_channels) - 1):
            for depth_idx in range(self.depth - layer_idx):
                if layer_idx == 0:
                    dense[f'x_{depth_idx}_{depth_idx}'] = self.blocks[f'x_{depth_idx}_{depth_idx}'](
                        feats[depth_idx], feats[depth_idx + 1])
                else:
                    li = depth_idx + layer_idx
                    cat = [dense[f'x_{i}_{li}'] for i in range(depth_idx + 1, li + 1)]
                    cat = torch.cat(cat + [feats[li + 1]], dim=1)
                    dense[f'x_{depth_idx}_{li}'] = self.blocks[f'x_{depth_idx}_{li}'](dense[f'x_{depth_idx}_{li - 1}'],
                                                                                        cat)
        return self.blocks[f'x_0_{self.depth}'](dense[f'x_0_{self.depth - 1}'])


class Conv3x3GNReLU(nn.Module):
    def __init__(self, in_channels, out_channels, upsample=False):
        super().__init__()
        self.upsample = upsample
        self.block = nn.Sequential(nn.Conv2d(in_channels, out_channels, 3, padding=1, bias=False),
                                   nn.GroupNorm(32, out_channels), nn.ReLU(inplace=True))

    def forward(self, x):
        x = self.block(x)
        return F.interpolate(x, scale_factor=2, mode='bilinear', align_corners=True) if self.upsample else x


class FPNBlock(nn.Module):
    def __init__(self, pyramid_channels, skip_channels):
        super().__init__()
        self.skip_conv = nn.Conv2d(skip_channels, pyramid_channels, kernel_size=1)

    def forward(self, x, skip):
        return F.interpolate(x, scale_factor=2, mode='nearest') + self.skip_conv(skip)


class SegmentationBlock(nn.Module):
    def __init__(self, in_channels, out_channels, n_upsamples=0):
        super().__init__()
        blocks = [Conv3x3GNReLU(in_channels, out_channels, upsample=bool(n_upsamples))]
        blocks += [Conv3x3GNReLU(out_channels, out_channels, upsample=True) for _ in range(1, n_upsamples)]
        self.block = nn.Sequential(*blocks)

    def forward(self, x):
        return self.block(x)


class FPNDecoder(nn.Module):
    def __init__(self, encoder_channels, pyramid_channels=256, segmentation_channels=128, dropout=0.2,
                 merge_policy='add'):
        super().__init__()
        self.out_channels = segmentation_channels if merge_policy == 'add' else segmentation_channels * 4
        ec = list(encoder_channels)[::-1]
        self.p5 = nn.Conv2d(ec[0], pyramid_channels, kernel_size=1)
        self.p4 = FPNBlock(pyramid_channels, ec[1])
        self.p3 = FPNBlock(pyramid_channels, ec[2])
        self.p2 = FPNBlock(pyramid_channels, ec[3])
        self.seg_blocks = nn.ModuleList([SegmentationBlock(pyramid_channels, segmentation_channels, n)
                                         for n in [3, 2, 1, 0]])
        self.merge_policy = merge_policy
        self.dropout = nn.Dropout2d(p=dropout, inplace=True)

    def forward(self, *features):
        c2, c3, c4, c5 = features[-4:]
        p5 = self.p5(c5)
        p4 = self.p4(p5, c4)
        p3 = self.p3(p4, c3)
        p2 = self.p2(p3, c2)
        pyr = [blk(p) for blk, p in zip(self.seg_blocks, [p5, p4, p3, p2])]
        x = sum(pyr) if self.merge_policy == 'add' else torch.cat(pyr, dim=1)
        return self.dropout(x)


class TransposeX2(nn.Sequential):
    def __init__(self, in_channels, out_channels, use_batchnorm=True):
        layers = [nn.ConvTranspose2d(in_channels, out_channels, kernel_size=4, stride=2, padding=1)]
        if use_batchnorm:
            layers.append(nn.BatchNorm2d(out_channels))
        layers.append(nn.ReLU(inplace=True))
        super().__init__(*layers)


class LinknetDecoderBlock(nn.Module):
    def __init__(self, in_channels, out_channels, use_batchnorm=True):
        super().__init__()
        self.block = nn.Sequential(Conv2dReLU(in_channels, in_channels // 4, 1, use_batchnorm=use_batchnorm),
                                   TransposeX2(in_channels // 4, in_channels // 4, use_batchnorm),
                                   Conv2dReLU(in_channels // 4, out_channels, 1, use_batchnorm=use_batchnorm))

    def forward(self, x, skip=None):
        x = self.block(x)
        return x + skip if skip is not None else x


class LinknetDecoder(nn.Module):
    def __init__(self, encoder_channels, prefinal_channels=32, n_blocks=5, use_batchnorm=True):
        super().__init__()
        ec = list(encoder_channels[1:])[::-1]
        ch = ec + [prefinal_channels]
        self.blocks = nn.ModuleList([LinknetDecoderBlock(ch[i], ch[i + 1], use_batchnorm) for i in range(n_blocks)])

    def forward(self, *features):
        feats = features[1:][::-1]
        x, skips = feats[0], feats[1:]
        for i, block in enumerate(self.blocks):
            x = block(x, skips[i] if i < len(skips) else None)
        return x


class PSPBlock(nn.Module):
    def __init__(self, in_channels, out_channels, pool_size, use_bathcnorm=True):
        super().__init__()
        if pool_size == 1:
            use_bathcnorm = False
        self.pool = nn.Sequential(nn.AdaptiveAvgPool2d((pool_size, pool_size)),
                                  Conv2dReLU(in_channels, out_channels, (1, 1), use_batchnorm=use_bathcnorm))

    def forward(self, x):
        h, w = x.shape[2:]
        return F.interpolate(self.pool(x), size=(h, w), mode='bilinear', align_corners=True)


class PSPModule(nn.Module):
    def __init__(self, in_channels, sizes=(1, 2, 3, 6), use_bathcnorm=True):
        super().__init__()
        self.blocks = nn.ModuleList([PSPBlock(in_channels, in_channels // len(sizes), s, use_bathcnorm) for s in sizes])

    def forward(self, x):
        return torch.cat([b(x) for b in self.blocks] + [x], dim=1)


class PSPDecoder(nn.Module):
    def __init__(self, encoder_channels, use_batchnorm=True, out_channels=512, dropout=0.2):
        super().__init__()
        self.psp = PSPModule(encoder_channels[-1], (1, 2, 3, 6), use_batchnorm)
        self.conv = Conv2dReLU(encoder_channels[-1] * 2, out_channels, 1, use_batchnorm=use_batchnorm)
        self.dropout = nn.Dropout2d(p=dropout)

    def forward(self, *features):
        return self.dropout(self.conv(self.psp(features[-1])))


class ASPPConv(nn.Sequential):
    def __init__(self, in_channels, out_channels, dilation):
        super().__init__(nn.Conv2d(in_channels, out_channels, 3, padding=dilation, dilation=dilation, bias=False),
                         nn.BatchNorm2d(out_channels), nn.ReLU())


class ASPPSeparableConv(nn.Sequential):
    def __init__(self, in_channels, out_channels, dilation):
        super().__init__(SeparableConv2d(in_channels, out_channels, 3, padding=dilation, dilation=dilation, bias=False),
                         nn.BatchNorm2d(out_channels), nn.ReLU())


class ASPPPooling(nn.Sequential):
    def __init__(self, in_channels, out_channels):
        super().__init__(nn.AdaptiveAvgPool2d(1), nn.Conv2d(in_channels, out_channels, 1, bias=False),
                         nn.BatchNorm2d(out_channels), nn.ReLU())

    def forward(self, x):
        size = x.shape[-2:]
        for m in self:
            x = m(x)
        return F.interpolate(x, size=size, mode='bilinear', align_corners=False)


class ASPP(nn.Module):
    def __init__(self, in_channels, out_channels, atrous_rates, separable=False):
        super().__init__()
        mods = [nn.Sequential(nn.Conv2d(in_channels, out_channels, 1, bias=False), nn.BatchNorm2d(out_channels),
                              nn.ReLU())]
        conv = ASPPSeparableConv if separable else ASPPConv
        mods += [conv(in_channels, out_channels, r) for r in atrous_rates]
        mods.append(ASPPPooling(in_channels, out_channels))
        self.convs = nn.ModuleList(mods)
        self.project = nn.Sequential(nn.Conv2d(5 * out_channels, out_channels, 1, bias=False),
                                     nn.BatchNorm2d(out_channels), nn.ReLU(), nn.Dropout(0.5))

    def forward(self, x):
        return self.project(torch.cat([c(x) for c in self.convs], dim=1))


class DeepLabV3Decoder(nn.Sequential):
    def __init__(self, in_channels, out_channels=256, atrous_rates=(12, 24, 36)):
        super().__init__(ASPP(in_channels, out_channels, atrous_rates),
                         nn.Conv2d(out_channels, out_channels, 3, padding=1, bias=False),
                         nn.BatchNorm2d(out_channels), nn.ReLU())
        self.out_channels = out_channels

    def forward(self, *features):
        return super().forward(features[-1])


class DeepLabV3PlusDecoder(nn.Module):
    def __init__(self, encoder_channels, out_channels=256, atrous_rates=(12, 24, 36), output_stride=16):
        super().__init__()
        self.out_channels = out_channels
        self.aspp = nn.Sequential(ASPP(encoder_channels[-1], out_channels, atrous_rates, separable=True),
                                  SeparableConv2d(out_channels, out_channels, 3, padding=1, bias=False),
                                  nn.BatchNorm2d(out_channels), nn.ReLU())
        self.up = nn.UpsamplingBilinear2d(scale_factor=2 if output_stride == 8 else 4)
        hi = encoder_channels[-4]
        self.block1 = nn.Sequential(nn.Conv2d(hi, 48, 1, bias=False), nn.BatchNorm2d(48), nn.ReLU())
        self.block2 = nn.Sequential(SeparableConv2d(48 + out_channels, out_channels, 3, padding=1, bias=False),
                                    nn.BatchNorm2d(out_channels), nn.ReLU())

    def forward(self, *features):
        a = self.up(self.aspp(features[-1]))
        return self.block2(torch.cat([a, self.block1(features[-4])], dim=1))


class ConvBnRelu(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1, bias=True,
                 add_relu=True, interpolate=False):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)
        self.add_relu, self.interpolate = add_relu, interpolate
        self.bn = nn.BatchNorm2d(out_channels)
        self.activation = nn.ReLU(inplace=True)

    def forward(self, x):
        x = self.bn(self.conv(x))
        if self.add_relu:
            x = self.activation(x)
        if self.interpolate:
            x = F.interpolate(x, scale_factor=2, mode='bilinear', align_corners=True)
        return x


class FPABlock(nn.Module):
    def __init__(self, in_channels, out_channels, upscale_mode='bilinear'):
        super().__init__()
        self.upscale_mode = upscale_mode
        self.align_corners = True if upscale_mode == 'bilinear' else None
        self.branch1 = nn.Sequential(nn.AdaptiveAvgPool2d(1), ConvBnRelu(in_channels, out_channels, 1))
        self.mid = nn.Sequential(ConvBnRelu(in_channels, out_channels, 1))
        self.down1 = nn.Sequential(nn.MaxPool2d(2, 2), ConvBnRelu(in_channels, 1, 7, 1, 3))
        self.down2 = nn.Sequential(nn.MaxPool2d(2, 2), ConvBnRelu(1, 1, 5, 1, 2))
        self.down3 = nn.Sequential(nn.MaxPool2d(2, 2), ConvBnRelu(1, 1, 3, 1, 1), ConvBnRelu(1, 1, 3, 1, 1))
        self.conv2 = ConvBnRelu(1, 1, 5, 1, 2)
        self.conv1 = ConvBnRelu(1, 1, 7, 1, 3)

    def forward(self, x):
        h, w = x.shape[2:]
        up = dict(mode=self.upscale_mode, align_corners=self.align_corners)
        b1 = F.interpolate(self.branch1(x), size=(h, w), **up)
        mid = self.mid(x)
        x1 = self.down1(x)
        x2 = self.down2(x1)
        x3 = F.interpolate(self.down3(x2), size=(h // 4, w // 4), **up)
        x = F.interpolate(self.conv2(x2) + x3, size=(h // 2, w // 2), **up)
        x = F.interpolate(x + self.conv1(x1), size=(h, w), **up)
        return x * mid + b1


class GAUBlock(nn.Module):
    def __init__(self, in_channels, out_channels, upscale_mode='bilinear'):
        super().__init__()
        self.upscale_mode = upscale_mode
        self.align_corners = True if upscale_mode == 'bilinear' else None
        self.conv1 = nn.Sequential(nn.AdaptiveAvgPool2d(1), ConvBnRelu(out_channels, out_channels, 1, add_relu=False),
                                   nn.Sigmoid())
        self.conv2 = ConvBnRelu(in_channels, out_channels, 3, 1, 1)

    def forward(self, x, y):
        h, w = x.shape[2:]
        y_up = F.interpolate(y, size=(h, w), mode=self.upscale_mode, align_corners=self.align_corners)
        return y_up + self.conv2(x) * self.conv1(y)


class PANDecoder(nn.Module):
    def __init__(self, encoder_channels, decoder_channels=32, upscale_mode='bilinear'):
        super().__init__()
        self.fpa = FPABlock(encoder_channels[-1], decoder_channels)
        self.gau3 = GAUBlock(encoder_channels[-2], decoder_channels, upscale_mode)
        self.gau2 = GAUBlock(encoder_channels[-3], decoder_channels, upscale_mode)
        self.gau1 = GAUBlock(encoder_channels[-4], decoder_channels, upscale_mode)

    def forward(self, *features):
        x5 = self.fpa(features[-1])
        x4 = self.gau3(features[-2], x5)
        x3 = self.gau2(features[-3], x4)
        return self.gau1(features[-4], x3)


class PABBlock(nn.Module):
    def __init__(self, in_channels, pab_channels=64):
        super().__init__()
        self.pab_channels, self.in_channels = pab_channels, in_channels
        self.top_conv = nn.Conv2d(in_channels, pab_channels, 1)
        self.center_conv = nn.Conv2d(in_channels, pab_channels, 1)
        self.bottom_conv = nn.Conv2d(in_channels, in_channels, 3, padding=1)
        self.map_softmax = nn.Softmax(dim=1)
        self.out_conv = nn.Conv2d(in_channels, in_channels, 3, padding=1)

    def forward(self, x):
        b, _, h, w = x.shape
        top = self.top_conv(x).flatten(2)
        center = self.center_conv(x).flatten(2).transpose(1, 2)
        bottom = self.bottom_conv(x).flatten(2).transpose(1, 2)
        sp = self.map_softmax(torch.matmul(center, top).view(b, -1)).view(b, h * w, h * w)
        sp = torch.matmul(sp, bottom).reshape(b, self.in_channels, h, w)
        return self.out_conv(x + sp)


class MFABBlock(nn.Module):
    def __init__(self, in_channels, skip_channels, out_channels, use_batchnorm=True, reduction=16):
        super().__init__()
        red = max(1, skip_channels // reduction)
        self.hl_conv = nn.Sequential(Conv2dReLU(in_channels, in_channels, 3, padding=1, use_batchnorm=use_batchnorm),
                                     Conv2dReLU(in_channels, skip_channels, 1, use_batchnorm=use_batchnorm))
        self.SE_ll = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(skip_channels, red, 1), nn.ReLU(inplace=True),
                                   nn.Conv2d(red, skip_channels, 1), nn.Sigmoid())
        self.SE_hl = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(skip_channels, red, 1), nn.ReLU(inplace=True),
                                   nn.Conv2d(red, skip_channels, 1), nn.Sigmoid())
        self.conv1 = Conv2dReLU(2 * skip_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm)
        self.conv2 = Conv2dReLU(out_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm)

    def forward(self, x, skip=None):
        x = F.interpolate(self.hl_conv(x), scale_factor=2, mode='nearest')
        att = self.SE_hl(x)
        if skip is not None:
            att = att + self.SE_ll(skip)
            x = torch.cat([x * att, skip], dim=1)
        return self.conv2(self.conv1(x))


class MAnetDecoder(nn.Module):
    def __init__(self, encoder_channels, decoder_channels=(256, 128, 64, 32, 16), reduction=16, use_batchnorm=True,
                 pab_channels=64):
        super().__init__()
        enc = list(encoder_channels[1:])[::-1]
        in_ch = [enc[0]] + list(decoder_channels[:-1])
        skip_ch = enc[1:] + [0]
        self.center = PABBlock(enc[0], pab_channels=pab_channels)
        self.blocks = nn.ModuleList([
            MFABBlock(i, s, o, use_batchnorm, reduction) if s > 0 else UnetDecoderBlock(i, s, o, use_batchnorm)
            for i, s, o in zip(in_ch, skip_ch, decoder_channels)])

    def forward(self, *features):
        feats = features[1:][::-1]
        x = self.center(feats[0])
        skips = feats[1:]
        for i, block in enumerate(self.blocks):
            x = block(x, skips[i] if i < len(skips) else None)
        return x


# ----------------------------------------------------------------------------- models
class SegmentationModel(nn.Module):
    def forward(self, x):
        features = self.encoder(x)
        return self.segmentation_head(self.decoder(*features))

    @torch.no_grad()
    def predict(self, x):
        if self.training:
            self.eval()
        return self.forward(x)


def _make(decoder_fn, head_in, head_k=3, head_up=1, depth=5, output_stride=32):
    def ctor(encoder_name='resnet34', encoder_weights='imagenet', in_channels=3, classes=1, **kw):
        m = SegmentationModel()
        m.encoder = get_encoder(encoder_name, in_channels, depth, encoder_weights, output_stride)
        m.decoder = decoder_fn(m.encoder.out_channels, **kw)
        hin = head_in(m.decoder) if callable(head_in) else head_in
        m.segmentation_head = SegmentationHead(hin, classes, head_k, head_up)
        m.name = f'{decoder_fn.__name__.replace("Decoder", "").lower()}-{encoder_name}'
        return m
    return ctor


Unet = _make(UnetDecoder, 16)
UnetPlusPlus = _make(UnetPlusPlusDecoder, 16)
FPN = _make(FPNDecoder, lambda d: d.out_channels, head_k=1, head_up=4)
Linknet = _make(LinknetDecoder, 32, head_k=1)
MAnet = _make(MAnetDecoder, 16)
PAN = _make(PANDecoder, 32, head_k=3, head_up=4, output_stride=16)
PSPNet = _make(PSPDecoder, 512, head_k=3, head_up=8, depth=3)
DeepLabV3 = _make(DeepLabV3Decoder, 256, head_k=1, head_up=8, output_stride=8)
DeepLabV3Plus = _make(DeepLabV3PlusDecoder, 256, head_k=1, head_up=4, output_stride=16)


def _v3_decoder(enc_channels, **kw):
    return DeepLabV3Decoder(enc_channels[-1], **kw)


DeepLabV3 = _make(_v3_decoder, 256, head_k=1, head_up=8, output_stride=8)
