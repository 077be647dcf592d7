"""Feature-extractor backbones -- reference ``models/backbone.py:4-57`` (``ResNet``, ``Mobilenetv2``).

The reference wraps torchvision (not installed here, and no weights can be downloaded); these are
built from the native torchvision-layout encoders of :mod:`.smp`, so attribute names
(``conv1/bn1/relu/maxpool/layer1..4``; ``layer1..4`` slices of the MobileNetV2 ``features``) and
state_dict keys match torchvision's.  ``pretrained=True`` accepts a local state_dict path via
``weights=`` (loaded with ``weights_only=True``); otherwise it warns and keeps the random init.
Both return the 4x/8x/16x/32x feature maps ``(x1, x2, x3, x4)``.
"""
from __future__ import annotations

import warnings

import torch
import torch.nn as nn

from .smp import ENCODERS, MobileNetV2Encoder, ResNetEncoder

_RESNETS = ('resnet18', 'resnet34', 'resnet50', 'resnet101', 'resnet152')


def _load(module, pretrained, weights):
    if weights is not None:
        sd = torch.load(weights, map_location='cpu', weights_only=True)
        sd = sd.get('state_dict', sd)
        module.load_state_dict({k: v for k, v in sd.items() if not k.startswith(('fc.', 'classifier.'))},
                               strict=False)
    elif pretrained:
        warnings.warn('pretrained=True: ImageNet weights cannot be downloaded here; random init kept '
                      '(pass weights=<local .pth> to load them).')


class ResNet(nn.Module):
    def __init__(self, resnet_type, pretrained=True, weights=None):
        super().__init__()
        if resnet_type not in _RESNETS:
            raise ValueError(f'Unsupported ResNet type: {resnet_type}.\n')
        block, layers, oc, kw = ENCODERS[resnet_type]
        enc = ResNetEncoder(block, layers, oc, **kw)
        _load(enc, pretrained, weights)
        self.conv1, self.bn1, self.relu, self.maxpool = enc.conv1, enc.bn1, enc.relu, enc.maxpool
        self.layer1, self.layer2, self.layer3, self.layer4 = enc.layer1, enc.layer2, enc.layer3, enc.layer4

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))    # 4x down
        x1 = self.layer1(x)
        x2 = self.layer2(x1)                                     # 8x
        x3 = self.layer3(x2)                                     # 16x
        x4 = self.layer4(x3)                                     # 32x
        return x1, x2, x3, x4


class Mobilenetv2(nn.Module):
    def __init__(self, pretrained=True, weights=None):
        super().__init__()
        enc = MobileNetV2Encoder()
        _load(enc, pretrained, weights)
        f = enc.features
        self.layer1, self.layer2, self.layer3, self.layer4 = f[:4], f[4:7], f[7:14], f[14:18]

    def forward(self, x):
        x1 = self.layer1(x)      # 4x down
        x2 = self.layer2(x1)     # 8x
        x3 = self.layer3(x2)     # 16x
        x4 = self.layer4(x3)     # 32x
        return x1, x2, x3, x4
