"""Building blocks shared by every model family.

Parity notes (reference ``models/modules.py``):
  * ``conv1x1`` / ``conv3x3``            -> ``modules.py:7,13``  (bias-free convs)
  * ``ConvBNAct``                        -> ``modules.py:73-85`` (padding = (k-1)//2 * dilation)
  * ``DeConvBNAct``                      -> ``modules.py:89-108`` (k = 2s-1, output_padding = s-1)
  * ``Activation`` (16-entry hub)        -> ``modules.py:111-131``
  * ``DSConvBNAct``/``DWConvBNAct``/``PWConvBNAct``/``PyramidPoolingModule``/``SegHead``/
    ``channel_shuffle``                  -> ``modules.py:18-69,134-166`` (unused by the reference
    models, kept so user code importing them keeps working)

Module *names* are part of the checkpoint contract (``Sequential`` index 0 = conv, 1 = BN, 2 = act),
so ``state_dict`` keys match the reference exactly.  The modules here are the plain-PyTorch
(reference-semantics) path used on CPU and for numerics checks; the MI355X training path lowers
the same parameters onto the fused HIP kernels in :mod:`medical_segmentation_pytorch_amd.runtime`.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

_ACTIVATIONS = {
    'relu': nn.ReLU, 'relu6': nn.ReLU6, 'leakyrelu': nn.LeakyReLU, 'prelu': nn.PReLU,
    'celu': nn.CELU, 'elu': nn.ELU, 'hardswish': nn.Hardswish, 'hardtanh': nn.Hardtanh,
    'gelu': nn.GELU, 'glu': nn.GLU, 'selu': nn.SELU, 'silu': nn.SiLU,
    'sigmoid': nn.Sigmoid, 'softmax': nn.Softmax, 'tanh': nn.Tanh, 'none': nn.Identity,
}


def _same_padding(kernel_size, dilation=1):
    if isinstance(kernel_size, (list, tuple)):
        return tuple((k - 1) // 2 * dilation for k in kernel_size)
    return (kernel_size - 1) // 2 * dilation


def conv3x3(in_channels, out_channels, stride=1, bias=False):
    return nn.Conv2d(in_channels, out_channels, 3, stride=stride, padding=1, bias=bias)


def conv1x1(in_channels, out_channels, stride=1, bias=False):
    return nn.Conv2d(in_channels, out_channels, 1, stride=stride, padding=0, bias=bias)


def channel_shuffle(x, groups=2):
    n, c, h, w = x.shape
    return x.reshape(n, groups, c // groups, h, w).transpose(1, 2).reshape(n, c, h, w)


class Activation(nn.Module):
    """Name -> activation module.  The wrapped module lives under ``.activation``."""

    def __init__(self, act_type, **kwargs):
        super().__init__()
        key = act_type.lower()
        if key not in _ACTIVATIONS:
            raise NotImplementedError(f'Unsupport activation type: {act_type}')
        self.act_type = key
        self.activation = _ACTIVATIONS[key](**kwargs)

    def forward(self, x):
        return self.activation(x)


class ConvBNAct(nn.Sequential):
    """conv (no bias) -> BatchNorm2d -> activation; children '0', '1', '2'."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, dilation=1, groups=1,
                 bias=False, act_type='relu', **kwargs):
        conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride,
                         _same_padding(kernel_size, dilation), dilation, groups, bias)
        super().__init__(conv, nn.BatchNorm2d(out_channels), Activation(act_type, **kwargs))


class DWConvBNAct(nn.Sequential):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, dilation=1,
                 act_type='relu', **kwargs):
        conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride,
                         _same_padding(kernel_size, dilation), dilation=dilation,
                         groups=in_channels, bias=False)
        super().__init__(conv, nn.BatchNorm2d(out_channels), Activation(act_type, **kwargs))


class PWConvBNAct(nn.Sequential):
    def __init__(self, in_channels, out_channels, act_type='relu', bias=True, **kwargs):
        super().__init__(nn.Conv2d(in_channels, out_channels, 1, bias=bias),
                         nn.BatchNorm2d(out_channels), Activation(act_type, **kwargs))


class DSConvBNAct(nn.Sequential):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, dilation=1,
                 act_type='relu', **kwargs):
        super().__init__(
            DWConvBNAct(in_channels, in_channels, kernel_size, stride, dilation, act_type, **kwargs),
            PWConvBNAct(in_channels, out_channels, act_type, **kwargs))


class DeConvBNAct(nn.Module):
    """Transposed conv (+bias) -> BN -> act, held in ``self.up_conv`` (keys ``up_conv.{0,1}``)."""

    def __init__(self, in_channels, out_channels, scale_factor=2, kernel_size=None, padding=None,
                 act_type='relu', **kwargs):
        super().__init__()
        kernel_size = 2 * scale_factor - 1 if kernel_size is None else kernel_size
        padding = (kernel_size - 1) // 2 if padding is None else padding
        self.up_conv = nn.Sequential(
            nn.ConvTranspose2d(in_channels, out_channels, kernel_size=kernel_size,
                               stride=scale_factor, padding=padding,
                               output_padding=scale_factor - 1),
            nn.BatchNorm2d(out_channels),
            Activation(act_type, **kwargs))

    def forward(self, x):
        return self.up_conv(x)


class PyramidPoolingModule(nn.Module):
    def __init__(self, in_channels, out_channels, act_type, pool_sizes=(1, 2, 4, 6), bias=False):
        super().__init__()
        assert len(pool_sizes) == 4, 'Length of pool size should be 4.\n'
        hid = in_channels // 4
        for i, p in enumerate(pool_sizes, 1):
            setattr(self, f'stage{i}', nn.Sequential(nn.AdaptiveAvgPool2d(p), conv1x1(in_channels, hid)))
        self.conv = PWConvBNAct(2 * in_channels, out_channels, act_type=act_type, bias=bias)

    def forward(self, x):
        size = x.shape[2:]
        feats = [x] + [F.interpolate(getattr(self, f'stage{i}')(x), size, mode='bilinear',
                                     align_corners=True) for i in range(1, 5)]
        return self.conv(torch.cat(feats, dim=1))


class SegHead(nn.Sequential):
    def __init__(self, in_channels, num_class, act_type, hid_channels=128):
        super().__init__(ConvBNAct(in_channels, hid_channels, 3, act_type=act_type),
                         conv1x1(hid_channels, num_class))
