"""Decoder-hub HIP kernels (csrc/decoder.hip) vs plain PyTorch fp32 references of the same ops:
bilinear resize (both align modes, up / down / from 1x1), GroupNorm(+ReLU), adaptive average pooling
(PSPNet bins, global) and depthwise conv -- forward values and every gradient."""
import os
import sys

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

pytestmark = pytest.mark.gpu


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize('case', [((11, 13), (22, 26), True), ((11, 13), (22, 26), False), ((6, 6), (44, 44), True),
                                  ((1, 1), (17, 9), False), ((44, 44), (88, 88), True), ((20, 20), (7, 5), False)])
def test_resize_bilinear(gpu, case):
    from medical_segmentation_pytorch_amd.ops.decoder import resize_bilinear
    (h, w), (oh, ow), align = case
    torch.manual_seed(0)
    x = torch.randn(2, 24, h, w, device=gpu)
    xr = x.clone().requires_grad_(True)
    ref = F.interpolate(xr, size=(oh, ow), mode='bilinear', align_corners=align)
    g = torch.randn_like(ref)
    ref.backward(g)
    xb = _nhwc(x).to(torch.bfloat16).requires_grad_(True)
    y = resize_bilinear(xb, size=(oh, ow), align_corners=align)
    y.backward(_nhwc(g).to(torch.bfloat16))
    assert _rel(y, _nhwc(ref)) < 1e-2
    assert _rel(xb.grad, _nhwc(xr.grad)) < 1e-2


def test_resize_accumulate(gpu):
    from medical_segmentation_pytorch_amd.ops.decoder import resize_bilinear
    x = torch.randn(2, 8, 8, 16, device=gpu).to(torch.bfloat16)
    base = torch.randn(2, 16, 16, 16, device=gpu).to(torch.bfloat16)
    out = base.clone()
    resize_bilinear(x, scale_factor=2, align_corners=True, out=out)
    ref = base.float() + resize_bilinear(x, scale_factor=2, align_corners=True).float()
    assert _rel(out, ref) < 1e-2


@pytest.mark.parametrize('relu', [True, False])
def test_group_norm_act(gpu, relu):
    from medical_segmentation_pytorch_amd.ops.decoder import group_norm_act
    torch.manual_seed(0)
    gn = nn.GroupNorm(32, 128).to(gpu)
    with torch.no_grad():
        gn.weight.uniform_(0.5, 1.5)
        gn.bias.uniform_(-0.2, 0.2)
    x = torch.randn(2, 128, 23, 17, device=gpu) * 2 + 0.5
    xr = x.clone().requires_grad_(True)
    ref = F.group_norm(xr, 32, gn.weight, gn.bias, gn.eps)
    if relu:
        ref = torch.relu(ref)
    g = torch.randn_like(ref)
    gw, gb = torch.autograd.grad(ref, (gn.weight, gn.bias), g, retain_graph=True)
    ref.backward(g)
    xb = _nhwc(x).to(torch.bfloat16).requires_grad_(True)
    y = group_norm_act(xb, gn, relu)
    dw, db = torch.autograd.grad(y, (gn.weight, gn.bias), _nhwc(g).to(torch.bfloat16), retain_graph=True)
    y.backward(_nhwc(g).to(torch.bfloat16))
    assert _rel(y, _nhwc(ref)) < 1e-2
    assert _rel(xb.grad, _nhwc(xr.grad)) < 3e-2
    assert _rel(dw, gw) < 2e-2 and _rel(db, gb) < 2e-2


@pytest.mark.parametrize('out_hw', [1, 2, 3, 6, (5, 7)])
def test_adaptive_avgpool(gpu, out_hw):
    from medical_segmentation_pytorch_amd.ops.decoder import adaptive_avgpool
    torch.manual_seed(0)
    x = torch.randn(2, 40, 22, 19, device=gpu)
    xr = x.clone().requires_grad_(True)
    ref = F.adaptive_avg_pool2d(xr, out_hw)
    g = torch.randn_like(ref)
    ref.backward(g)
    xb = _nhwc(x).to(torch.bfloat16).requires_grad_(True)
    y = adaptive_avgpool(xb, out_hw)
    y.backward(_nhwc(g).to(torch.bfloat16))
    assert _rel(y, _nhwc(ref)) < 1e-2
    assert _rel(xb.grad, _nhwc(xr.grad)) < 1e-2


@pytest.mark.parametrize('dil,bias', [(1, False), (12, False), (2, True)])
def test_dwconv(gpu, dil, bias):
    from medical_segmentation_pytorch_amd.ops.decoder import dwconv
    torch.manual_seed(0)
    conv = nn.Conv2d(64, 64, 3, padding=dil, dilation=dil, groups=64, bias=bias).to(gpu)
    x = torch.randn(2, 64, 30, 26, device=gpu)
    xr = x.clone().requires_grad_(True)
    ref = conv(xr)
    g = torch.randn_like(ref)
    grads = torch.autograd.grad(ref, [conv.weight] + ([conv.bias] if bias else []), g, retain_graph=True)
    ref.backward(g)
    xb = _nhwc(x).to(torch.bfloat16).requires_grad_(True)
    y = dwconv(xb, conv)
    mine = torch.autograd.grad(y, [conv.weight] + ([conv.bias] if bias else []), _nhwc(g).to(torch.bfloat16),
                               retain_graph=True)
    y.backward(_nhwc(g).to(torch.bfloat16))
    assert _rel(y, _nhwc(ref)) < 1e-2
    assert _rel(xb.grad, _nhwc(xr.grad)) < 1e-2
    for a, b in zip(mine, grads):
        assert _rel(a, b) < 1e-2
