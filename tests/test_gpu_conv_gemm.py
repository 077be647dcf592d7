"""The LDS-tiled implicit-GEMM conv kernel (csrc/conv_gemm.hip) vs fp32 PyTorch, over every tile
configuration: forward (+ bias, multi-group outputs, stride 2, asymmetric / dilated taps, ragged pixel
tails, K tails), the stride-1 data-gradient it also runs, the BN-statistics epilogue, the
accumulating epilogue and the BN-backward epilogue (MI355X only)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from medical_segmentation_pytorch_amd.ops.conv import Branch, ConvPlan, conv
from medical_segmentation_pytorch_amd.ops.fm import cpad, from_fm_reference, to_fm_reference

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.fixture
def ext():
    from medical_segmentation_pytorch_amd.ops import _ext
    C = _ext.require()
    yield C
    C.conv_gemm_force_cfg(-1)
    C.conv_set_gemm(True)
    C.conv_set_wgrad_gemm(1)


GEMM_CASES = [
    # N, H, W, Cin, Cout, (kh, kw), stride, pad, dil, groups, bias
    (2, 11, 13, 72, 72, (3, 3), 1, (1, 1), (1, 1), 1, False),      # K = 648 -> Kp 672 (a 32-wide K tail)
    (2, 9, 9, 136, 136, (3, 3), 1, (3, 3), (3, 3), 1, False),      # dilation 3
    (1, 7, 19, 64, 40, (1, 7), 1, (0, 3), (1, 1), 1, True),        # 1x7 + bias, 40 output channels
    (2, 10, 6, 136, 72, (7, 1), 1, (3, 0), (1, 1), 3, False),      # 7x1, three output groups
    (3, 6, 6, 272, 272, (3, 3), 2, (1, 1), (1, 1), 1, False),      # stride 2, M tail (27 pixels)
    (2, 8, 8, 72, 144, (2, 2), 2, (0, 0), (1, 1), 1, False),       # 2x2 s2 (DUCKNet shortcut)
    (2, 5, 7, 544, 96, (1, 1), 1, (0, 0), (1, 1), 2, False),       # 1x1, wide K, two groups
    (2, 7, 5, 272, 24, (3, 3), 1, (1, 1), (1, 1), 1, True),        # bias, narrow output (one co tile)
    (4, 16, 16, 256, 256, (3, 3), 1, (2, 2), (2, 2), 1, False),    # DeepLabV3 (output stride 8) layer3
    (4, 16, 16, 512, 512, (3, 3), 1, (4, 4), (4, 4), 1, False),    # ... layer4: dilation 4 on a 16x16 map
]


@pytest.mark.parametrize('cfg', [-1, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize('case', GEMM_CASES)
def test_gemm_conv_fwd_bwd(gpu, ext, case, cfg):
    n, h, w, ci, co, (kh, kw), s, pad, dil, groups, bias = case
    ext.conv_gemm_force_cfg(cfg)
    torch.manual_seed(0)
    ms = [nn.Conv2d(ci, co, (kh, kw), s, pad, dil, bias=bias).to(gpu) for _ in range(groups)]
    br = [Branch(m.weight, g, 0, kh * kw) for g, m in enumerate(ms)]
    plan = ConvPlan(kh, kw, ci, co, br, stride=s, padding=pad, dilation=dil, Go=groups,
                    bias=ms[0].bias if bias else None)
    x = _bf(torch.randn(n, ci, h, w, device=gpu))
    xf = to_fm_reference(x).requires_grad_(True)
    oh, ow = plan.out_hw(h, w)
    assert ext.conv_uses_gemm(plan.fwd_dims(n, h, w, oh, ow), [t[0] for t in plan.taps_fwd],
                              [t[1] for t in plan.taps_fwd], False)
    ys, part = conv(plan, [xf], want_stats=not bias)
    xr = x.clone().requires_grad_(True)
    wrs = [_bf(m.weight.detach()).requires_grad_(True) for m in ms]
    brf = ms[0].bias.detach().float() if bias else None
    refs = [F.conv2d(xr, wr, brf, s, pad, dil) for wr in wrs]
    for y, r in zip(ys, refs):
        assert y.shape == (n, r.shape[2], r.shape[3], cpad(co))
        assert _rel(from_fm_reference(y, co), r) < 1e-2
        if co < cpad(co):
            assert y[..., co:].abs().max().item() == 0.0
    if not bias:   # BN partials == channel sums of the stored (bf16) outputs
        tot = part.sum(0)
        yv = torch.cat([y.float().reshape(-1, cpad(co)) for y in ys], 1)
        assert ((tot[0] - yv.sum(0)).abs() / yv.abs().sum(0).clamp_min(1e-6)).max() < 1e-4
        assert _rel(tot[1], (yv * yv).sum(0)) < 1e-4
    gs = [_bf(torch.randn_like(r)) for r in refs]
    torch.autograd.backward(refs, gs)
    torch.autograd.backward(ys, [to_fm_reference(g) for g in gs])
    assert _rel(from_fm_reference(xf.grad, ci), xr.grad) < 2e-2
    for m, wr in zip(ms, wrs):
        assert _rel(m.weight.grad, wr.grad) < 2e-2


def test_gemm_matches_gather_kernel(gpu, ext):
    """Same launch on the GEMM kernel and on the register-direct gather kernel: both within bf16
    rounding of each other (different fp32 summation orders)."""
    torch.manual_seed(3)
    m = nn.Conv2d(136, 272, 3, 1, 1, bias=False).to(gpu)
    plan = ConvPlan(3, 3, 136, 272, [Branch(m.weight)], padding=(1, 1))
    xf = to_fm_reference(_bf(torch.randn(4, 136, 12, 12, device=gpu)))
    (y1,), p1 = conv(plan, [xf], want_stats=True)
    ext.conv_set_gemm(False)
    (y0,), p0 = conv(plan, [xf], want_stats=True)
    assert _rel(y1, y0) < 4e-3
    assert _rel(p1.sum(0), p0.sum(0)) < 1e-3


def test_gemm_accumulate_and_bn_epilogue(gpu, ext):
    """conv_fwd(accumulate=True) adds into the stored bf16 output; conv_fwd_bn emits the BN-backward
    partials (sum g, sum g*(y - mean)), g = dz * relu'(y*scale + shift), of the data-gradient it stores."""
    C = ext
    torch.manual_seed(5)
    n, h, w, ci, co = 2, 9, 11, 72, 136
    m = nn.Conv2d(ci, co, 3, 1, 1, bias=False).to(gpu)
    plan = ConvPlan(3, 3, ci, co, [Branch(m.weight)], padding=(1, 1))
    x = to_fm_reference(_bf(torch.randn(n, ci, h, w, device=gpu)))
    wp = plan.pack_fwd(gpu)
    dims = plan.fwd_dims(n, h, w, h, w)
    dy = [t[0] for t in plan.taps_fwd]
    dx = [t[1] for t in plan.taps_fwd]
    assert C.conv_uses_gemm(dims, dy, dx, False)
    base = to_fm_reference(_bf(torch.randn(n, co, h, w, device=gpu)))
    y = base.clone()
    C.conv_fwd([x], wp, [y], None, None, dims, dy, dx, False, accumulate=True)
    yr = F.conv2d(from_fm_reference(x, ci), _bf(m.weight.detach()), None, 1, 1)
    assert _rel(from_fm_reference(y, co), yr + from_fm_reference(base, co)) < 1e-2
    # BN-backward epilogue: treat the conv output as dL/dz of a BN(+ReLU) over y_bn
    y_bn = to_fm_reference(_bf(torch.randn(n, co, h, w, device=gpu)))
    coef = torch.zeros(3, cpad(co), device=gpu)
    coef[0, :co] = torch.rand(co, device=gpu) + 0.5
    coef[1, :co] = torch.randn(co, device=gpu) * 0.2
    coef[2, :co] = torch.randn(co, device=gpu) * 0.1
    out = torch.empty_like(y_bn)
    nblk = C.conv_stat_blocks(dims, dy, dx)
    part = torch.empty(nblk, 2, cpad(co), device=gpu)
    C.conv_fwd_bn([x], wp, [out], part, dims, dy, dx, y_bn, coef, True)
    dz = out.float()
    yb = y_bn.float()
    gmask = (yb * coef[0] + coef[1]) > 0
    g = torch.where(gmask, dz, torch.zeros_like(dz)).reshape(-1, cpad(co))
    s_ref = g.sum(0)
    q_ref = (g * (yb.reshape(-1, cpad(co)) - coef[2])).sum(0)
    tot = part.sum(0)
    assert _rel(tot[0], s_ref) < 1e-4 and _rel(tot[1], q_ref) < 1e-4
    assert _rel(from_fm_reference(out, co), yr) < 1e-2


WGRAD_CASES = [
    # N, H, W, Cin, Cout, (kh, kw), stride, pad, dil, groups
    (2, 17, 19, 24, 24, (3, 3), 1, (1, 1), (1, 1), 1),     # L1-like narrow rows
    (2, 12, 11, 40, 40, (1, 7), 1, (0, 3), (1, 1), 5),     # fused 5 groups, ragged pixel stages
    (1, 9, 9, 72, 136, (3, 3), 1, (3, 3), (3, 3), 1),      # dilated
    (2, 8, 10, 136, 272, (3, 3), 2, (1, 1), (1, 1), 1),    # strided (3x3 s2 downsample)
    (3, 6, 6, 272, 96, (1, 1), 1, (0, 0), (1, 1), 2),      # 1x1, K < tile
    (2, 10, 10, 24, 48, (2, 2), 2, (0, 0), (1, 1), 1),     # 2x2 s2 shortcut
]


@pytest.mark.parametrize('cfg', [-1, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize('prologue', [False, True])
@pytest.mark.parametrize('case', WGRAD_CASES)
def test_wgrad_gemm(gpu, ext, case, prologue, cfg):
    """Weight gradient on the LDS-tiled GEMM kernel vs fp32 torch, every tile configuration, with and
    without the deferred-BN(+ReLU) prologue on x (re-normalised in LDS; zero padding stays zero)."""
    C = ext
    n, h, w, ci, co, (kh, kw), s, pad, dil, groups = case
    C.conv_wgrad_gemm_force_cfg(cfg)
    C.conv_set_wgrad_gemm(2)   # the GEMM kernel for every eligible shape (the planner keeps narrow ones on halo)
    try:
        torch.manual_seed(7)
        ms = [nn.Conv2d(ci, co, (kh, kw), s, pad, dil, bias=False).to(gpu) for _ in range(groups)]
        plan = ConvPlan(kh, kw, ci, co, [Branch(m.weight, g, 0, kh * kw) for g, m in enumerate(ms)], stride=s,
                        padding=pad, dilation=dil, Go=groups)
        x = _bf(torch.randn(n, ci, h, w, device=gpu))
        xf = to_fm_reference(x)
        oh, ow = plan.out_hw(h, w)
        dims = plan.fwd_dims(n, h, w, oh, ow)
        dy = [t[0] for t in plan.taps_fwd]
        dx = [t[1] for t in plan.taps_fwd]
        assert C.conv_uses_wgrad_gemm(dims, dy, dx, False)
        gys = [to_fm_reference(_bf(torch.randn(n, co, oh, ow, device=gpu))) for _ in range(groups)]
        xc, xr = [], 0
        z = x
        if prologue:
            st = torch.zeros(4, plan.Cgi, device=gpu)
            st[0, :ci] = torch.rand(ci, device=gpu) + 0.5
            st[1, :ci] = torch.randn(ci, device=gpu) * 0.3
            xc, xr = [st], 1
            z = _bf(torch.relu(x * st[0, :ci].view(1, -1, 1, 1) + st[1, :ci].view(1, -1, 1, 1)))
        KT = plan.T * plan.Cip
        nrep = C.conv_wgrad_replicas(dims, dy, dx, False, False, bool(xc))
        dwp = torch.empty(nrep * plan.rows * KT, device=gpu)
        C.conv_wgrad(gys, [xf], dwp, dims, dy, dx, False, xc, xr)
        tot = dwp.view(nrep, plan.rows, KT).sum(0)          # [rows][t*Cip + c]
        for g_, m in enumerate(ms):
            zr = z.clone().requires_grad_(False)
            wr = m.weight.detach().clone().requires_grad_(True)
            yr = F.conv2d(zr, wr, None, s, pad, dil)
            yr.backward(from_fm_reference(gys[g_], co))
            got = tot[g_ * plan.Cgo:g_ * plan.Cgo + co].view(co, plan.T, plan.Cip)[:, :, :ci].permute(0, 2, 1)
            assert _rel(got.reshape(co, ci, kh, kw), wr.grad) < 1e-2, g_
    finally:
        C.conv_wgrad_gemm_force_cfg(-1)
