"""The halo-staged implicit-GEMM conv (csrc/conv_gemm.hip conv_hgemm_kernel) vs fp32 PyTorch at the odd
geometries it has to get right: widths that are not a multiple of the tile (prime widths: one strip of
the whole width), dilation 3 at 11x11 / 22x22 (halo boxes that cross image boundaries, masked taps),
1x7 / 7x1 channel tails at 136 / 272 / 544 input channels, 72-channel inputs (a 16-wide tail chunk with
8 real channels), multi-group inputs (UNet concat) and outputs (fused sibling convs), bias, the
BN-statistics epilogue, the data-gradient (flipped taps: the same kernel), the accumulating and the
BN-backward epilogues -- over every tile configuration (MI355X only)."""
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
    C.conv_hgemm_force_cfg(-1)
    C.conv_set_hgemm(True)


HG_CASES = [
    # N, H, W, Cin, Cout, (kh, kw), pad, dil, Gi, Go, bias
    (2, 11, 11, 136, 136, (3, 3), (3, 3), (3, 3), 1, 1, False),   # dilation 3 at 11x11
    (2, 22, 22, 72, 72, (3, 3), (3, 3), (3, 3), 1, 1, False),     # dilation 3 at 22x22, 72-ch tail chunk
    (3, 13, 17, 72, 144, (3, 3), (1, 1), (1, 1), 1, 1, False),    # prime width 17 (one strip), 3 images
    (2, 9, 20, 136, 136, (1, 7), (0, 3), (1, 1), 1, 1, True),     # 1x7 + bias, width 20 (strips of 10/20)
    (2, 20, 6, 272, 72, (7, 1), (3, 0), (1, 1), 1, 3, False),     # 7x1, three output groups, 272 channels
    (1, 11, 11, 544, 96, (1, 7), (0, 3), (1, 1), 1, 1, False),    # 1x7 at 544 channels
    (1, 11, 11, 544, 64, (7, 1), (3, 0), (1, 1), 1, 2, False),    # 7x1 at 544 channels, two output groups
    (2, 16, 16, 256, 256, (3, 3), (2, 2), (2, 2), 1, 1, False),   # dilation 2 (DeepLabV3 output stride 8)
    (2, 44, 44, 64, 40, (3, 3), (1, 1), (1, 1), 1, 1, True),      # 44x44 strips, one 64-ch chunk, bias
    (2, 12, 12, 72, 136, (3, 3), (1, 1), (1, 1), 2, 1, False),    # two input groups (concat), 2 x 72 ch
]


def _plan(gpu, case):
    n, h, w, ci, co, (kh, kw), pad, dil, gi, go, bias = case
    ms = [nn.Conv2d(gi * ci, co, (kh, kw), 1, pad, dil, bias=bias).to(gpu) for _ in range(go)]
    br = [Branch(m.weight, g, 0, kh * kw) for g, m in enumerate(ms)]
    plan = ConvPlan(kh, kw, ci, co, br, stride=1, padding=pad, dilation=dil, Gi=gi, Go=go,
                    bias=ms[0].bias if bias else None)
    return ms, plan


@pytest.mark.parametrize('cfg', [-1, 0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize('case', HG_CASES)
def test_hgemm_conv_fwd_bwd(gpu, ext, case, cfg):
    n, h, w, ci, co, (kh, kw), pad, dil, gi, go, bias = case
    ext.conv_hgemm_force_cfg(cfg)
    torch.manual_seed(0)
    ms, plan = _plan(gpu, case)
    dims = plan.fwd_dims(n, h, w, h, w)
    fy, fx = [t[0] for t in plan.taps_fwd], [t[1] for t in plan.taps_fwd]
    if not ext.conv_uses_hgemm(dims, fy, fx):
        pytest.skip('configuration does not fit this geometry')
    xs = [_bf(torch.randn(n, ci, h, w, device=gpu)) for _ in range(gi)]
    xfs = [to_fm_reference(x).requires_grad_(True) for x in xs]
    ys, part = conv(plan, xfs, want_stats=not bias)
    xr = torch.cat(xs, 1).requires_grad_(True)
    wrs = [_bf(m.weight.detach()).requires_grad_(True) for m in ms]
    brf = ms[0].bias.detach().float() if bias else None
    refs = [F.conv2d(xr, wr, brf, 1, pad, dil) for wr in wrs]
    for y, r in zip(ys, refs):
        assert y.shape == (n, h, w, cpad(co))
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
    dref = xr.grad
    for i, xf in enumerate(xfs):
        assert _rel(from_fm_reference(xf.grad, ci), dref[:, i * ci:(i + 1) * ci]) < 2e-2
    for m, wr in zip(ms, wrs):
        assert _rel(m.weight.grad, wr.grad) < 2e-2


def test_hgemm_dgrad_runs_halo_path(gpu, ext):
    """The data-gradient launch of a wide 3x3 (flipped taps) is planned on the halo kernel too."""
    _, plan = _plan(gpu, (4, 22, 22, 136, 136, (3, 3), (1, 1), (1, 1), 1, 1, False))
    dims_d = [4, 22, 22, plan.Go, plan.Cgo, 22, 22, 1, plan.Cgi, 136, plan.T, plan.Kp, 1]
    assert ext.conv_uses_hgemm(dims_d, [t[0] for t in plan.taps_bwd], [t[1] for t in plan.taps_bwd])


def test_hgemm_matches_im2col_kernel(gpu, ext):
    """Same launch on the halo kernel and on the im2col LDS-DMA kernel: within bf16 rounding of each other."""
    torch.manual_seed(3)
    m = nn.Conv2d(136, 272, 3, 1, 3, 3, bias=False).to(gpu)
    plan = ConvPlan(3, 3, 136, 272, [Branch(m.weight)], padding=(3, 3), dilation=(3, 3))
    xf = to_fm_reference(_bf(torch.randn(4, 136, 22, 22, device=gpu)))
    (y1,), p1 = conv(plan, [xf], want_stats=True)
    ext.conv_set_hgemm(False)
    (y0,), p0 = conv(plan, [xf], want_stats=True)
    assert _rel(y1, y0) < 4e-3
    assert _rel(p1.sum(0), p0.sum(0)) < 1e-3


def test_hgemm_accumulate_and_bn_epilogue(gpu, ext):
    """accumulate=True adds into the stored bf16 output; conv_fwd_bn emits the BN-backward partials
    (sum g, sum g*(y - mean)), g = dz * relu'(y*scale + shift), of the data-gradient it stores."""
    C = ext
    torch.manual_seed(5)
    n, h, w, ci, co = 2, 11, 11, 72, 136
    m = nn.Conv2d(ci, co, 3, 1, 1, bias=False).to(gpu)
    plan = ConvPlan(3, 3, ci, co, [Branch(m.weight)], padding=(1, 1))
    x = to_fm_reference(_bf(torch.randn(n, ci, h, w, device=gpu)))
    wp = plan.pack_fwd(gpu)
    dims = plan.fwd_dims(n, h, w, h, w)
    dy = [t[0] for t in plan.taps_fwd]
    dx = [t[1] for t in plan.taps_fwd]
    assert C.conv_uses_hgemm(dims, dy, dx)
    base = to_fm_reference(_bf(torch.randn(n, co, h, w, device=gpu)))
    y = base.clone()
    C.conv_fwd([x], wp, [y], None, None, dims, dy, dx, False, accumulate=True)
    yr = F.conv2d(from_fm_reference(x, ci), _bf(m.weight.detach()), None, 1, 1)
    assert _rel(from_fm_reference(y, co), yr + from_fm_reference(base, co)) < 1e-2
    # BN-backward epilogue: data-gradient of a conv whose input z = relu(bn(yb)): out = dL/dz (stored),
    # partials of g = dz * [scale*yb + shift > 0]
    wd, kpd = plan.pack_dgrad(gpu)
    dims_d = [n, h, w, 1, plan.Cgo, h, w, 1, plan.Cgi, ci, plan.T, kpd, 1]
    bdy, bdx = [t[0] for t in plan.taps_bwd], [t[1] for t in plan.taps_bwd]
    assert C.conv_uses_hgemm(dims_d, bdy, bdx)
    gz = to_fm_reference(_bf(torch.randn(n, co, h, w, device=gpu)))
    yb = to_fm_reference(_bf(torch.randn(n, ci, h, w, device=gpu)))
    coef = torch.zeros(3, plan.Cgi, device=gpu)
    coef[0, :ci] = torch.rand(ci, device=gpu) + 0.5
    coef[1, :ci] = torch.randn(ci, device=gpu) * 0.2
    coef[2, :ci] = torch.randn(ci, device=gpu) * 0.1
    nblk = C.conv_stat_blocks(dims_d, bdy, bdx, False, False, True)
    part = torch.empty(nblk, 2, plan.Cgi, device=gpu)
    dz = torch.empty_like(yb)
    C.conv_fwd_bn([gz], wd, [dz], part, dims_d, bdy, bdx, yb, coef, True)
    dzr = torch.nn.grad.conv2d_input((n, ci, h, w), _bf(m.weight.detach()), from_fm_reference(gz, co), 1, 1)
    assert _rel(from_fm_reference(dz, ci), dzr) < 1e-2
    dzs = dz.float().reshape(-1, plan.Cgi)
    ybs = yb.float().reshape(-1, plan.Cgi)
    gmask = (ybs * coef[0] + coef[1]) > 0
    g = torch.where(gmask, dzs, torch.zeros_like(dzs))
    tot = part.sum(0)
    assert _rel(tot[0, :ci], g.sum(0)[:ci]) < 1e-4
    assert _rel(tot[1, :ci], (g * (ybs - coef[2])).sum(0)[:ci]) < 1e-4
