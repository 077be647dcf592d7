"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same op (MI355X only)."""
import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from medical_segmentation_pytorch_amd.ops.bn import BNState, bn_act, bn_act_reference
from medical_segmentation_pytorch_amd.ops.conv import Branch, ConvPlan, conv, conv_reference
from medical_segmentation_pytorch_amd.ops.fm import cpad, from_fm_reference, to_fm_reference

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _bf(t):
    return t.to(torch.bfloat16).float()


CONV_CASES = [
    # N, H, W, Cin, Cout, (kh, kw), stride, pad, dil
    (2, 16, 16, 17, 17, (3, 3), 1, (1, 1), (1, 1)),
    (2, 16, 16, 17, 34, (3, 3), 1, (2, 2), (2, 2)),
    (2, 16, 16, 34, 34, (3, 3), 1, (3, 3), (3, 3)),
    (2, 12, 20, 3, 17, (1, 7), 1, (0, 3), (1, 1)),
    (2, 12, 20, 17, 17, (7, 1), 1, (3, 0), (1, 1)),
    (2, 16, 16, 17, 34, (2, 2), 2, (0, 0), (1, 1)),
    (2, 16, 16, 17, 34, (3, 3), 2, (1, 1), (1, 1)),
    (2, 8, 8, 136, 68, (1, 1), 1, (0, 0), (1, 1)),
    (1, 11, 11, 272, 544, (3, 3), 1, (1, 1), (1, 1)),
    (3, 9, 7, 40, 72, (3, 3), 1, (1, 1), (1, 1)),
    (2, 17, 15, 17, 34, (3, 3), 2, (1, 1), (1, 1)),    # odd sizes: uneven output phases in the dgrad
    (2, 16, 16, 64, 128, (1, 1), 2, (0, 0), (1, 1)),   # ResNet downsample: 3 of 4 dgrad phases are empty
    (2, 32, 32, 3, 64, (7, 7), 2, (3, 3), (1, 1)),     # ResNet stem: 49 taps
    (2, 20, 20, 136, 136, (3, 3), 1, (1, 1), (1, 1)),  # 136 ch: too wide for a 256-px halo tile
    (2, 13, 19, 136, 72, (3, 3), 1, (2, 2), (2, 2)),   # the same, dilated, ragged tiles
]


@pytest.mark.parametrize('case', CONV_CASES)
def test_conv_fwd_bwd(gpu, case):
    n, h, w, ci, co, (kh, kw), s, pad, dil = case
    torch.manual_seed(0)
    m = nn.Conv2d(ci, co, (kh, kw), s, pad, dil, bias=False).to(gpu)
    plan = ConvPlan(kh, kw, ci, co, [Branch(m.weight)], stride=s, padding=pad, dilation=dil)
    x = _bf(torch.randn(n, ci, h, w, device=gpu))
    xf = to_fm_reference(x).requires_grad_(True)
    (y,), part = conv(plan, [xf], want_stats=True)
    # reference with the same bf16-rounded operands
    xr = x.clone().requires_grad_(True)
    wr = _bf(m.weight.detach()).requires_grad_(True)
    yr = F.conv2d(xr, wr, None, s, pad, dil)
    assert y.shape == (n, yr.shape[2], yr.shape[3], cpad(co))
    assert _rel(from_fm_reference(y, co), yr) < 1e-2
    if co < cpad(co):
        assert y[..., co:].abs().max().item() == 0.0      # padded channels stay zero
    # conv-epilogue BN partials == channel sums of the stored output
    tot = part.sum(0)
    yv = y.float().reshape(-1, cpad(co))
    # (bias-free epilogues sum the fp32 accumulators: the stored values' sums up to bf16 rounding
    # noise, measured against the sum of magnitudes because the channel sums cancel)
    assert ((tot[0] - yv.sum(0)).abs() / yv.abs().sum(0).clamp_min(1e-6)).max() < 1e-3
    assert _rel(tot[1], (yv * yv).sum(0)) < 1e-2
    # backward
    g = _bf(torch.randn_like(yr))
    yr.backward(g)
    gf = to_fm_reference(g)
    y.backward(gf)
    assert _rel(from_fm_reference(xf.grad, ci), xr.grad) < 2e-2
    assert _rel(m.weight.grad, wr.grad) < 2e-2


def test_conv_groups_fused_siblings(gpu):
    """DUCK-style horizontal fusion: 3x3 convs + 1x1 convs (centre tap) in one launch."""
    torch.manual_seed(1)
    n, h, w, ci, co = 2, 16, 16, 17, 17
    c3 = [nn.Conv2d(ci, co, 3, 1, 1, bias=False).to(gpu) for _ in range(2)]
    c1 = [nn.Conv2d(ci, co, 1, bias=False).to(gpu) for _ in range(2)]
    br = [Branch(c.weight, g, 0, 9) for g, c in enumerate(c3)] + [Branch(c.weight, 2 + g, 4, 1) for g, c in enumerate(c1)]
    plan = ConvPlan(3, 3, ci, co, br, padding=(1, 1), Go=4)
    x = _bf(torch.randn(n, ci, h, w, device=gpu))
    xf = to_fm_reference(x).requires_grad_(True)
    ys, part = conv(plan, [xf], want_stats=True)
    refs = [F.conv2d(x, _bf(c.weight.detach()), None, 1, 1) for c in c3] + [F.conv2d(x, _bf(c.weight.detach())) for c in c1]
    for y, r in zip(ys, refs):
        assert _rel(from_fm_reference(y, co), r) < 1e-2
    # backward: input grad = sum of the four branches' dgrads
    gs = [_bf(torch.randn_like(r)) for r in refs]
    xr = x.clone().requires_grad_(True)
    ws = [_bf(c.weight.detach()).requires_grad_(True) for c in c3 + c1]
    out = sum((F.conv2d(xr, wv, None, 1, 1 if i < 2 else 0) * gg).sum() for i, (wv, gg) in enumerate(zip(ws, gs)))
    out.backward()
    torch.autograd.backward(ys, [to_fm_reference(gg) for gg in gs])
    assert _rel(from_fm_reference(xf.grad, ci), xr.grad) < 2e-2
    for c, wv in zip(c3 + c1, ws):
        assert _rel(c.weight.grad, wv.grad) < 2e-2


@pytest.mark.parametrize('c,deferred', [(17, False), (72, True)])
def test_conv_multi_accumulates_dgrad(gpu, c, deferred):
    """Sibling launches on one input as one node (ops.conv.conv_multi, the DUCK split): outputs, weight
    grads and the input gradient (later plans' dgrads accumulate in the epilogue) vs separate launches."""
    from medical_segmentation_pytorch_amd.ops.bn import Deferred
    from medical_segmentation_pytorch_amd.ops.conv import conv_multi
    torch.manual_seed(7)
    n, h, w = 2, 20, 24
    c3 = [nn.Conv2d(c, c, 3, 1, 1, bias=False).to(gpu) for _ in range(3)]
    c1 = [nn.Conv2d(c, c, 1, bias=False).to(gpu) for _ in range(2)]
    x0 = to_fm_reference(_bf(torch.randn(n, c, h, w, device=gpu)))
    stats = torch.zeros(4, x0.shape[-1], device=gpu)
    stats[0, :c] = torch.rand(c, device=gpu) + 0.5
    stats[1, :c] = torch.randn(c, device=gpu) * 0.1
    res = []
    for multi in (False, True):
        for m in c3 + c1:
            m.weight.grad = None
        p3 = ConvPlan(3, 3, c, c, [Branch(m.weight, g, 0, 9) for g, m in enumerate(c3)], padding=(1, 1), Go=3)
        p1 = ConvPlan(1, 1, c, c, [Branch(m.weight, g, 0, 1) for g, m in enumerate(c1)], Go=2)
        xt = x0.clone().requires_grad_(True)
        x = Deferred(xt, stats, True) if deferred else xt
        if multi:
            (ya, _), (yb, _) = conv_multi([p3, p1], x)
        else:
            ya, _ = conv(p3, [x])
            yb, _ = conv(p1, [x])
        outs = list(ya) + list(yb)
        gs = [to_fm_reference(_bf(torch.randn(n, c, h, w, device=gpu, generator=torch.Generator(gpu).manual_seed(k))))
              for k in range(5)]
        torch.autograd.backward(outs, gs)
        res.append([o.float() for o in outs] + [xt.grad.float()] + [m.weight.grad.clone() for m in c3 + c1])
    for a, b in zip(res[0], res[1]):
        assert _rel(b, a) < 5e-3, _rel(b, a)


def test_conv_group_inputs(gpu):
    """UNet concat: conv over two input tensors without materialising torch.cat."""
    torch.manual_seed(2)
    n, h, w, ci, co = 2, 12, 12, 32, 32
    m = nn.Conv2d(2 * ci, co, 3, 1, 1, bias=False).to(gpu)
    plan = ConvPlan(3, 3, ci, co, [Branch(m.weight)], padding=(1, 1), Gi=2)
    a = _bf(torch.randn(n, ci, h, w, device=gpu))
    b = _bf(torch.randn(n, ci, h, w, device=gpu))
    af, bf_ = to_fm_reference(a).requires_grad_(True), to_fm_reference(b).requires_grad_(True)
    (y,), _ = conv(plan, [af, bf_])
    xr = torch.cat([a, b], 1).requires_grad_(True)
    wr = _bf(m.weight.detach()).requires_grad_(True)
    yr = F.conv2d(xr, wr, None, 1, 1)
    assert _rel(from_fm_reference(y, co), yr) < 1e-2
    g = _bf(torch.randn_like(yr))
    yr.backward(g)
    y.backward(to_fm_reference(g))
    assert _rel(from_fm_reference(af.grad, ci), xr.grad[:, :ci]) < 2e-2
    assert _rel(from_fm_reference(bf_.grad, ci), xr.grad[:, ci:]) < 2e-2
    assert _rel(m.weight.grad, wr.grad) < 2e-2


def test_conv_transpose(gpu):
    torch.manual_seed(3)
    n, h, w, ci, co = 2, 8, 8, 64, 32
    m = nn.ConvTranspose2d(ci, co, 3, 2, 1, output_padding=1).to(gpu)
    plan = ConvPlan(3, 3, ci, co, [Branch(m.weight)], stride=2, padding=(1, 1), transposed=True, output_padding=1,
                    bias=m.bias)
    x = _bf(torch.randn(n, ci, h, w, device=gpu))
    xf = to_fm_reference(x).requires_grad_(True)
    (y,), _ = conv(plan, [xf])
    xr = x.clone().requires_grad_(True)
    wr = _bf(m.weight.detach()).requires_grad_(True)
    br = m.bias.detach().clone().requires_grad_(True)
    yr = F.conv_transpose2d(xr, wr, br, 2, 1, 1)
    assert y.shape[1:3] == yr.shape[2:]
    assert _rel(from_fm_reference(y, co), yr) < 1e-2
    g = _bf(torch.randn_like(yr))
    yr.backward(g)
    y.backward(to_fm_reference(g))
    assert _rel(from_fm_reference(xf.grad, ci), xr.grad) < 2e-2
    assert _rel(m.weight.grad, wr.grad) < 2e-2
    assert _rel(m.bias.grad, br.grad) < 2e-2


def test_conv_phase_matches_gather(gpu):
    """The phase-decomposed strided data-gradient equals the full-tap TRANS gather up to fp32
    summation order (same products; the compacted K chunks group them differently)."""
    from medical_segmentation_pytorch_amd.ops import _ext
    C = _ext.require()
    torch.manual_seed(5)
    m = nn.Conv2d(34, 68, 3, 2, 1, bias=False).to(gpu)
    plan = ConvPlan(3, 3, 34, 68, [Branch(m.weight)], stride=2, padding=(1, 1))
    outs = []
    for on in (True, False):
        C.conv_set_phase(on)
        xf = to_fm_reference(_bf(torch.randn(3, 34, 21, 19, device=gpu, generator=torch.Generator(gpu).manual_seed(0))))
        xf.requires_grad_(True)
        (y,), _ = conv(plan, [xf])
        y.backward(torch.ones_like(y))
        outs.append(xf.grad.clone())
    C.conv_set_phase(True)
    assert _rel(outs[0], outs[1]) < 2e-3


@pytest.mark.parametrize('C,k', [(17, 1), (34, 2), (136, 6), (3, 1)])
def test_bn_act(gpu, C, k):
    torch.manual_seed(4)
    n, h, w = 4, 16, 16
    bn = nn.BatchNorm2d(C).to(gpu)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn_ref = nn.BatchNorm2d(C).to(gpu)
    bn_ref.load_state_dict(bn.state_dict())
    xs = [_bf(torch.randn(n, C, h, w, device=gpu) * 2 + 0.3) for _ in range(k)]
    xfs = [to_fm_reference(x).requires_grad_(True) for x in xs]
    st = BNState.from_module(bn)
    z = bn_act(xfs, st, relu=True, training=True)
    xrs = [x.clone().requires_grad_(True) for x in xs]
    s = xrs[0]
    for x in xrs[1:]:
        s = s + x
    if k > 1:
        s = s + (_bf(s.detach()) - s.detach())  # the fused sum is stored in bf16
    zr = F.relu(bn_ref(s))
    assert _rel(from_fm_reference(z, C), zr) < 1e-2
    assert torch.allclose(bn.running_mean, bn_ref.running_mean, atol=1e-4, rtol=1e-3)
    assert torch.allclose(bn.running_var, bn_ref.running_var, atol=1e-4, rtol=1e-3)
    assert int(bn.num_batches_tracked) == 1
    g = _bf(torch.randn_like(zr))
    zr.backward(g)
    z.backward(to_fm_reference(g))
    for xf, xr in zip(xfs, xrs):
        assert _rel(from_fm_reference(xf.grad, C), xr.grad) < 2e-2
    assert _rel(bn.weight.grad, bn_ref.weight.grad) < 1e-2
    assert _rel(bn.bias.grad, bn_ref.bias.grad) < 1e-2
    # eval mode uses running stats
    bn.eval(); bn_ref.eval()
    ze = bn_act([xfs[0].detach()], BNState.from_module(bn), relu=True, training=False)
    assert _rel(from_fm_reference(ze, C), F.relu(bn_ref(xs[0]))) < 1e-2


def test_elementwise(gpu):
    from medical_segmentation_pytorch_amd.ops.elementwise import add_n, from_fm, to_fm, up2_add
    torch.manual_seed(5)
    x = torch.randn(2, 3, 16, 16, device=gpu)
    fm = to_fm(x)
    assert torch.equal(fm, to_fm_reference(x))
    back = from_fm(fm, 3)
    assert torch.equal(back, from_fm_reference(fm, 3))
    low = to_fm_reference(torch.randn(2, 34, 8, 8, device=gpu)).requires_grad_(True)
    skip = to_fm_reference(torch.randn(2, 34, 16, 16, device=gpu)).requires_grad_(True)
    out = up2_add(low, skip)
    ref = F.interpolate(from_fm_reference(low, 34), size=(16, 16), mode='nearest') + from_fm_reference(skip, 34)
    assert _rel(from_fm_reference(out, 34), ref) < 1e-2
    g = to_fm_reference(torch.randn(2, 34, 16, 16, device=gpu))
    out.backward(g)
    gl = F.avg_pool2d(from_fm_reference(g, 34), 2) * 4
    assert _rel(from_fm_reference(low.grad, 34), gl) < 1e-2
    a, b, c = [to_fm_reference(torch.randn(2, 5, 4, 4, device=gpu)) for _ in range(3)]
    s = add_n(a, b, c)
    assert _rel(s.float(), a.float() + b.float() + c.float()) < 1e-2


@pytest.mark.parametrize('k,s,p,hw', [(3, 2, 1, (16, 16)), (3, 2, 1, (17, 11)), (2, 2, 0, (8, 8))])
def test_maxpool(gpu, k, s, p, hw):
    from medical_segmentation_pytorch_amd.ops.pool import maxpool, maxpool_reference
    torch.manual_seed(7)
    x = to_fm_reference(torch.randn(2, 20, *hw, device=gpu)).requires_grad_(True)
    y = maxpool(x, k, s, p)
    assert torch.equal(y, maxpool_reference(x.detach(), k, s, p))    # max is exact in bf16
    g = to_fm_reference(torch.randn(2, 20, y.shape[1], y.shape[2], device=gpu))
    y.backward(g)
    xr = x.detach().permute(0, 3, 1, 2).float().requires_grad_(True)
    F.max_pool2d(xr, k, s, p).backward(g.permute(0, 3, 1, 2).float())
    ref = xr.grad.permute(0, 2, 3, 1)
    assert _rel(x.grad.float(), ref) < 1e-2
    assert x.grad[..., 20:].abs().sum() == 0


@pytest.mark.parametrize('cl,cs', [(64, 32), (20, 12), (16, 0)])
def test_up2_cat_and_add_act(gpu, cl, cs):
    from medical_segmentation_pytorch_amd.ops.pool import add_act, up2_cat, up2_cat_reference
    torch.manual_seed(8)
    low = to_fm_reference(torch.randn(2, cl, 5, 6, device=gpu)).requires_grad_(True)
    skip = to_fm_reference(torch.randn(2, cs, 10, 12, device=gpu)).requires_grad_(True) if cs else None
    out = up2_cat(low, skip, cl, cs)
    assert torch.equal(out, up2_cat_reference(low.detach(), skip.detach() if cs else None, cl, cs))
    g = to_fm_reference(torch.randn(2, cl + cs, 10, 12, device=gpu))
    out.backward(g)
    gl = F.avg_pool2d(from_fm_reference(g, cl + cs)[:, :cl], 2) * 4
    assert _rel(from_fm_reference(low.grad, cl), gl) < 1e-2
    if cs:
        assert torch.equal(from_fm_reference(skip.grad, cs), from_fm_reference(g, cl + cs)[:, cl:])
    a = to_fm_reference(torch.randn(2, 12, 4, 4, device=gpu)).requires_grad_(True)
    b = to_fm_reference(torch.randn(2, 12, 4, 4, device=gpu)).requires_grad_(True)
    z = add_act(a, b, relu=True)
    zr = torch.relu(a.detach().float() + b.detach().float())
    assert _rel(z.float(), zr) < 1e-2
    dz = torch.randn_like(z)
    z.backward(dz)
    ref = dz.float() * (z.float() > 0)
    assert _rel(a.grad.float(), ref) < 1e-2 and torch.equal(a.grad, b.grad)


@pytest.mark.parametrize('weighted', [False, True])
def test_cross_entropy(gpu, weighted):
    from medical_segmentation_pytorch_amd.ops.losses import cross_entropy
    torch.manual_seed(6)
    logits = torch.randn(3, 4, 10, 12, device=gpu, requires_grad=True)
    tgt = torch.randint(0, 4, (3, 10, 12), device=gpu)
    tgt[0, :2] = 255
    w = torch.tensor([1.0, 2.0, 0.5, 1.5], device=gpu) if weighted else None
    loss = cross_entropy(logits, tgt, w, 255)
    lr = logits.detach().clone().requires_grad_(True)
    ref = F.cross_entropy(lr, tgt, weight=w, ignore_index=255)
    assert abs(loss.item() - ref.item()) < 1e-4
    loss.backward(); ref.backward()
    assert _rel(logits.grad, lr.grad) < 1e-4


def test_ohem_and_kd(gpu):
    from medical_segmentation_pytorch_amd.ops.losses import kd_kl_div, ohem_cross_entropy
    torch.manual_seed(7)
    logits = torch.randn(2, 2, 16, 16, device=gpu, requires_grad=True)
    tgt = torch.randint(0, 2, (2, 16, 16), device=gpu)
    loss = ohem_cross_entropy(logits, tgt, 0.7, 255)
    lr = logits.detach().clone().requires_grad_(True)
    px = F.cross_entropy(lr, tgt, ignore_index=255, reduction='none').view(-1)
    hard = px[px > -math.log(0.7)]
    n_min = tgt.numel() // 16
    if hard.numel() < n_min:
        hard, _ = px.topk(n_min)
    ref = hard.mean()
    assert abs(loss.item() - ref.item()) < 1e-4
    loss.backward(); ref.backward()
    assert _rel(logits.grad, lr.grad) < 1e-4
    s = torch.randn(2, 3, 8, 8, device=gpu, requires_grad=True)
    t = torch.randn(2, 3, 8, 8, device=gpu)
    kd = kd_kl_div(s, t, 4.0)
    sr = s.detach().clone().requires_grad_(True)
    kr = F.kl_div(F.log_softmax(sr / 4, 1), F.softmax(t / 4, 1), reduction='mean') * 16
    assert abs(kd.item() - kr.item()) < 1e-5
    kd.backward(); kr.backward()
    assert _rel(s.grad, sr.grad) < 1e-4


def test_kd_mse_and_bce_dice(gpu):
    from medical_segmentation_pytorch_amd.ops.losses import bce_dice, kd_mse
    torch.manual_seed(9)
    s = torch.randn(2, 3, 8, 8, device=gpu, requires_grad=True)
    t = torch.randn(2, 3, 8, 8, device=gpu)
    sr = s.detach().clone().requires_grad_(True)
    a, b = kd_mse(s, t), F.mse_loss(sr, t)
    assert abs(a.item() - b.item()) < 1e-5
    (3 * a).backward(); (3 * b).backward()
    assert _rel(s.grad, sr.grad) < 1e-5
    # binary head: fused kernels vs the plain-torch BceDiceLoss formula (upstream grad != 1)
    x = torch.randn(3, 1, 20, 24, device=gpu, requires_grad=True)
    y = (torch.rand(3, 20, 24, device=gpu) > 0.6).float()
    xr = x.detach().clone().requires_grad_(True)
    got = bce_dice(x, y.unsqueeze(1), 1.0, 1.0, 1.0)
    p = torch.sigmoid(xr)
    inter = (p * y.unsqueeze(1)).flatten(1).sum(1)
    den = p.flatten(1).sum(1) + y.flatten(1).sum(1)
    ref = F.binary_cross_entropy_with_logits(xr, y.unsqueeze(1)) + 1 - ((2 * inter + 1) / (den + 1)).mean()
    assert abs(got.item() - ref.item()) < 1e-5
    (0.5 * got).backward(); (0.5 * ref).backward()
    assert _rel(x.grad, xr.grad) < 1e-4


def test_optim_and_ema(gpu):
    from medical_segmentation_pytorch_amd import _C
    torch.manual_seed(8)
    n = 1000
    for adamw in (False, True):
        p = torch.randn(n, device=gpu)
        pr = p.clone().requires_grad_(True)
        opt = (torch.optim.AdamW if adamw else torch.optim.Adam)([pr], lr=1e-2, weight_decay=0.1)
        m = torch.zeros(n, device=gpu); v = torch.zeros(n, device=gpu)
        for step in range(1, 4):
            g = torch.randn(n, device=gpu)
            pr.grad = g.clone()
            opt.step()
            hyper = torch.tensor([1e-2, 0.9, 0.999, 1e-8, 0.1, 1 - 0.9 ** step, 1 - 0.999 ** step, 1.0], device=gpu)
            _C.adam_step(p, g, m, v, hyper, adamw)
        assert _rel(p, pr.detach()) < 1e-5
    p = torch.randn(n, device=gpu)
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.SGD([pr], lr=1e-2, momentum=0.9, weight_decay=1e-4)
    buf = torch.zeros(n, device=gpu)
    for _ in range(3):
        g = torch.randn(n, device=gpu)
        pr.grad = g.clone()
        opt.step()
        _C.sgd_step(p, g, buf, torch.tensor([1e-2, 0.9, 1e-4, 1.0], device=gpu))
    assert _rel(p, pr.detach()) < 1e-5
    e = torch.randn(n, device=gpu); mm = torch.randn(n, device=gpu)
    ref = 0.3 * e + 0.7 * mm
    _C.ema_update(e, mm, torch.tensor([0.3], device=gpu))
    assert _rel(e, ref) < 1e-6


def test_confmat(gpu):
    from medical_segmentation_pytorch_amd import _C
    torch.manual_seed(9)
    logits = torch.randn(2, 3, 9, 9, device=gpu)
    tgt = torch.randint(0, 3, (2, 9, 9), device=gpu)
    tgt[0, 0] = 255
    cm = torch.zeros(3, 3, dtype=torch.long, device=gpu)
    _C.confmat_update(logits, tgt, cm, 255)
    pred = logits.argmax(1)
    valid = tgt != 255
    ref = torch.bincount(tgt[valid] * 3 + pred[valid], minlength=9).view(3, 3)
    assert torch.equal(cm, ref)


HALO_CASES = [
    # N, H, W, Cin, Cout, (kh, kw), pad, dil, Go   (stride 1; partial tiles in both dims)
    (2, 70, 90, 17, 17, (3, 3), (1, 1), (1, 1), 1),
    (1, 45, 37, 34, 34, (3, 3), (3, 3), (3, 3), 1),
    (2, 33, 50, 17, 17, (1, 7), (0, 3), (1, 1), 1),
    (1, 40, 29, 68, 68, (7, 1), (3, 0), (1, 1), 1),
    (2, 44, 44, 17, 17, (3, 3), (1, 1), (1, 1), 8),
    (1, 22, 22, 34, 34, (3, 3), (1, 1), (1, 1), 3),
    (2, 19, 23, 8, 40, (3, 3), (1, 1), (1, 1), 1),
]


@pytest.mark.parametrize('case', HALO_CASES)
def test_conv_halo_matches_gather(gpu, case):
    """The halo-tiled stride-1 kernel vs the gather igemm kernel (same packed operands) and vs fp32.
    (The LDS-tiled GEMM kernel, which takes >= 64-channel inputs by default, is off here.)"""
    from medical_segmentation_pytorch_amd.ops import _ext
    C = _ext.require()
    C.conv_set_gemm(False)
    C.conv_set_fwd_fused(False)   # (the fused forward has its own oracle: test_gpu_fused_bwd_oracle.py)
    try:
        _halo_vs_gather(gpu, case, C)
    finally:
        C.conv_set_gemm(True)
        C.conv_set_fwd_fused(True)


@pytest.mark.parametrize('case', HALO_CASES)
def test_conv_halo_split_bank_image_is_bitwise(gpu, case):
    """The split-bank tile image (two copies, one per k-group parity: csrc/conv.hip halo_phys) changes only
    LDS addresses: forward, BN partials and data-gradient are bitwise those of the single image."""
    from medical_segmentation_pytorch_amd.ops import _ext
    C = _ext.require()
    n, h, w, ci, co, (kh, kw), pad, dil, go = case
    torch.manual_seed(4)
    convs = [nn.Conv2d(ci, co, (kh, kw), 1, pad, dil, bias=False).to(gpu) for _ in range(go)]
    plan = ConvPlan(kh, kw, ci, co, [Branch(c.weight, g, 0, kh * kw) for g, c in enumerate(convs)], padding=pad,
                    dilation=dil, Go=go)
    x = _bf(torch.randn(n, ci, h, w, device=gpu))
    gs = [to_fm_reference(_bf(torch.randn(n, co, h, w, device=gpu, generator=torch.Generator(gpu).manual_seed(9 + i))))
          for i in range(go)]
    outs = []
    C.conv_set_gemm(False)
    C.conv_set_fwd_fused(False)
    try:
        for mode in (0, 2):
            C.conv_set_halo_split(mode)
            xf = to_fm_reference(x).requires_grad_(True)
            ys, part = conv(plan, [xf], want_stats=True)
            torch.autograd.backward(ys, gs)
            torch.cuda.synchronize()
            outs.append(([y.clone() for y in ys], part.clone(), xf.grad.clone()))
    finally:
        C.conv_set_halo_split(1)
        C.conv_set_gemm(True)
        C.conv_set_fwd_fused(True)
    (y0, p0, d0), (y2, p2, d2) = outs
    assert all(torch.equal(a, b) for a, b in zip(y0, y2))
    assert torch.equal(p0, p2)
    assert torch.equal(d0, d2)


def _halo_vs_gather(gpu, case, C):
    n, h, w, ci, co, (kh, kw), pad, dil, go = case
    torch.manual_seed(4)
    convs = [nn.Conv2d(ci, co, (kh, kw), 1, pad, dil, bias=False).to(gpu) for _ in range(go)]
    plan = ConvPlan(kh, kw, ci, co, [Branch(c.weight, g, 0, kh * kw) for g, c in enumerate(convs)], padding=pad,
                    dilation=dil, Go=go)
    x = _bf(torch.randn(n, ci, h, w, device=gpu))
    dims = plan.fwd_dims(n, h, w, h, w)
    dy, dx = [t[0] for t in plan.taps_fwd], [t[1] for t in plan.taps_fwd]
    assert C.conv_uses_halo(dims, dy, dx, False), 'case must exercise the halo kernel'
    if go > 1:   # data-gradient reads go dY groups: the channel-chunked halo path
        _, kp_d = plan.pack_dgrad(gpu)
        dims_d = [n, h, w, plan.Go, plan.Cgo, h, w, 1, plan.Cgi, ci, plan.T, kp_d, 1]
        bdy, bdx = [t[0] for t in plan.taps_bwd], [t[1] for t in plan.taps_bwd]
        assert C.conv_uses_halo(dims_d, bdy, bdx, False), 'dgrad must exercise the chunked halo kernel'
    outs = {}
    for mode in (True, False):
        C.conv_set_halo(mode)
        try:
            xf = to_fm_reference(x).requires_grad_(True)
            ys, part = conv(plan, [xf], want_stats=True)
            gs = [to_fm_reference(_bf(torch.randn(n, co, h, w, device=gpu, generator=torch.Generator(gpu).manual_seed(9 + i))))
                  for i in range(go)]
            torch.autograd.backward(ys, gs)
            outs[mode] = ([y.float() for y in ys], part.sum(0), xf.grad.float(), [c.weight.grad.clone() for c in convs])
            for c in convs:
                c.weight.grad = None
        finally:
            C.conv_set_halo(True)
    (yh, ph, dxh, wh), (yg, pg, dxg, wg) = outs[True], outs[False]
    for a, b, cv in zip(yh, yg, convs):
        assert _rel(a, b) < 5e-3
        ref = F.conv2d(x, _bf(cv.weight.detach()), None, 1, pad, dil)
        assert _rel(from_fm_reference(a.to(torch.bfloat16), co), ref) < 1e-2
    assert (ph - pg).abs().max() / pg.abs().max() < 2e-3
    assert _rel(dxh, dxg) < 5e-3
    for a, b in zip(wh, wg):
        assert _rel(a, b) < 5e-3


@pytest.mark.parametrize('ac', [False, True])
def test_bilinear_and_colorize(gpu, ac):
    from medical_segmentation_pytorch_amd.ops.resample import colorize, resize_bilinear
    torch.manual_seed(11)
    x = torch.randn(2, 3, 37, 50, device=gpu)
    for size in [(32, 64), (74, 100), (37, 50)]:
        y = resize_bilinear(x, size, align_corners=ac)
        ref = F.interpolate(x, size, mode='bilinear', align_corners=ac)
        assert (y - ref).abs().max().item() < 1e-5
    lut = torch.randint(0, 256, (4, 3), device=gpu, dtype=torch.uint8)
    logits = torch.randn(2, 4, 9, 7, device=gpu)
    assert torch.equal(colorize(logits, lut), lut[logits.argmax(1)])
    b = torch.randn(2, 1, 9, 7, device=gpu)
    assert torch.equal(colorize(b, lut), lut[(b[:, 0] > 0).long()])


@pytest.mark.parametrize('relu,halo', [(True, True), (False, True), (True, False)])
def test_bn_partials_from_dgrad_epilogue(gpu, relu, halo):
    """BN output feeding one stride-1 conv: the conv's data-gradient epilogue emits the BN backward
    partials (conv_fwd_bn) -- gradients must match the separate partial-sum pass."""
    from medical_segmentation_pytorch_amd.ops import _ext
    from medical_segmentation_pytorch_amd.ops.bn import BwdStatsHandle
    C = _ext.require()
    torch.manual_seed(12)
    n, h, w, c = 2, 20, 24, 17
    bnm = nn.BatchNorm2d(c).to(gpu)
    conv_m = nn.Conv2d(c, 34, 3, 1, 1, bias=False).to(gpu)
    res = []
    C.conv_set_halo(halo)
    try:
        for use in (False, True):
            bnm.weight.grad = bnm.bias.grad = conv_m.weight.grad = None
            st = BNState.from_module(bnm)
            plan = ConvPlan(3, 3, c, 34, [Branch(conv_m.weight, 0, 0, 9)], padding=(1, 1))
            y = to_fm_reference(_bf(torch.randn(n, c, h, w, device=gpu, generator=torch.Generator(gpu).manual_seed(3))))
            y.requires_grad_(True)
            hdl = BwdStatsHandle() if use else None
            z = bn_act([y], st, relu, True, None, handle=hdl)
            (o,), _ = conv(plan, [z], want_stats=False, bn_handle=hdl)
            g = to_fm_reference(_bf(torch.randn(n, 34, h, w, device=gpu, generator=torch.Generator(gpu).manual_seed(4))))
            o.backward(g)
            if use:
                assert hdl.part is None, 'BN backward must have consumed the epilogue partials'
            res.append((y.grad.float().clone(), bnm.weight.grad.clone(), bnm.bias.grad.clone(), conv_m.weight.grad.clone()))
    finally:
        C.conv_set_halo(True)
    for a, b in zip(res[0], res[1]):
        assert _rel(b, a) < 1e-3, _rel(b, a)


BNE_CASES = [
    # c, co, (kh, kw), dilation, n_3x3 groups, n_1x1 groups, (n, h, w), halo
    (64, 64, (3, 3), 1, 1, 0, (2, 20, 24), True),       # multi-row-group halo (MI >= 2 row tiles)
    (160, 96, (3, 3), 1, 1, 0, (2, 12, 16), True),      # wide input, several row groups
    (17, 17, (3, 3), 2, 1, 0, (2, 20, 24), True),       # dilated DUCK branches
    (17, 17, (3, 3), 3, 1, 0, (2, 20, 24), True),
    (17, 17, (1, 7), 1, 1, 0, (2, 20, 24), True),       # separated 1x7 / 7x1
    (17, 17, (7, 1), 1, 1, 0, (2, 20, 24), True),
    (17, 17, (3, 3), 1, 1, 1, (2, 20, 24), True),       # residual chain: fused 3x3 + 1x1 (Go = 2)
    (64, 64, (3, 3), 1, 5, 3, (2, 24, 32), True),       # DUCK-style Go = 8: chunked halo data-gradient
    (64, 64, (3, 3), 1, 1, 1, (2, 20, 24), False),      # implicit-GEMM data-gradient, Go = 2
]


@pytest.mark.parametrize('case', BNE_CASES)
def test_bn_partials_from_dgrad_epilogue_geometries(gpu, case):
    """The BN-epilogue data-gradient (conv_fwd_bn) over the geometries the executor marks single-consumer:
    several row groups, dilation 2/3, 1x7/7x1, Go = 2 residual-chain and Go = 8 (chunked halo) fused
    plans, and the implicit-GEMM path -- dx, dgamma, dbeta and dW must equal the separate-pass ones."""
    from medical_segmentation_pytorch_amd.ops import _ext
    from medical_segmentation_pytorch_amd.ops.bn import BwdStatsHandle
    C = _ext.require()
    c, co, (kh, kw), dil, n3, n1, (n, h, w), halo = case
    torch.manual_seed(21)
    bnm = nn.BatchNorm2d(c).to(gpu)
    with torch.no_grad():
        bnm.weight.uniform_(0.5, 1.5)
        bnm.bias.uniform_(-0.5, 0.5)
    convs = [nn.Conv2d(c, co, (kh, kw), 1, (dil * (kh // 2), dil * (kw // 2)), (dil, dil), bias=False).to(gpu)
             for _ in range(n3)]
    convs += [nn.Conv2d(c, co, 1, bias=False).to(gpu) for _ in range(n1)]
    T = kh * kw
    branches = [Branch(m.weight, g, 0, T) for g, m in enumerate(convs[:n3])]
    branches += [Branch(m.weight, n3 + g, T // 2, 1) for g, m in enumerate(convs[n3:])]
    y0 = to_fm_reference(_bf(torch.randn(n, c, h, w, device=gpu, generator=torch.Generator(gpu).manual_seed(3))))
    gs = [to_fm_reference(_bf(torch.randn(n, co, h, w, device=gpu, generator=torch.Generator(gpu).manual_seed(4 + g))))
          for g in range(n3 + n1)]
    res = []
    C.conv_set_halo(halo)
    try:
        for use in (False, True):
            for m in [bnm] + convs:
                for p in m.parameters():
                    p.grad = None
            st = BNState.from_module(bnm)
            plan = ConvPlan(kh, kw, c, co, branches, padding=(dil * (kh // 2), dil * (kw // 2)), dilation=(dil, dil),
                            Go=n3 + n1)
            y = y0.clone().requires_grad_(True)
            hdl = BwdStatsHandle() if use else None
            z = bn_act([y], st, True, True, None, handle=hdl)
            outs, _ = conv(plan, [z], want_stats=False, bn_handle=hdl)
            torch.autograd.backward(outs, gs)
            if use:
                assert hdl.part is None, 'BN backward must have consumed the epilogue partials'
            res.append([y.grad.float().clone(), bnm.weight.grad.clone(), bnm.bias.grad.clone()] +
                       [m.weight.grad.clone() for m in convs])
    finally:
        C.conv_set_halo(True)
    for a, b in zip(res[0], res[1]):
        assert _rel(b, a) < 1e-3, _rel(b, a)


def _ohem_ref(logits, tgt, thresh, ignore=255):
    px = F.cross_entropy(logits, tgt, ignore_index=ignore, reduction='none').view(-1)
    hard = px[px > -math.log(thresh)]
    n_min = int((tgt != ignore).sum()) // 16
    if hard.numel() < n_min:
        hard, _ = px.topk(n_min)
    return hard.mean()


@pytest.mark.parametrize('case', ['threshold', 'topk', 'ignore', 'ties'])
def test_ohem_device_selection(gpu, case):
    """Device-side OHEM (threshold count + exact radix top-k, no host sync) vs the reference formula
    (core/loss.py:13-20) in both branches, with ignored pixels and with ties at the k-th loss."""
    from medical_segmentation_pytorch_amd.ops.losses import ohem_cross_entropy
    torch.manual_seed(17)
    n, h, w = 3, 40, 48
    tgt = torch.randint(0, 2, (n, h, w), device=gpu)
    if case == 'threshold':
        logits = torch.randn(n, 2, h, w, device=gpu)                  # many hard pixels
    elif case == 'topk':
        logits = (tgt * 2 - 1).float()[:, None] * torch.tensor([-2.5, 2.5], device=gpu)[None, :, None, None]
        logits = logits + 0.5 * torch.randn_like(logits)             # confident: few above thr
    elif case == 'ignore':
        logits = torch.randn(n, 2, h, w, device=gpu) * 3
        tgt[:, :10] = 255
    else:                                                            # every loss identical: all tied
        tgt = torch.zeros_like(tgt)
        logits = torch.tensor([5.0, -5.0], device=gpu)[None, :, None, None].expand(n, 2, h, w).contiguous()
    lf = logits.clone().requires_grad_(True)
    lr = logits.clone().requires_grad_(True)
    loss = ohem_cross_entropy(lf, tgt, 0.7, 255)
    ref = _ohem_ref(lr, tgt, 0.7)
    assert abs(loss.item() - ref.item()) <= 1e-5 * max(1.0, abs(ref.item())), (loss.item(), ref.item())
    (2.0 * loss).backward()
    (2.0 * ref).backward()
    if case == 'ties':   # torch picks an arbitrary subset of the ties; the gradient's total agrees
        assert _rel(lf.grad.sum((0, 2, 3)), lr.grad.sum((0, 2, 3))) < 1e-4
    else:
        assert _rel(lf.grad, lr.grad) < 1e-4


def test_ohem_in_captured_graph(gpu):
    """OHEM inside a hipGraph: replays with new data match the reference every time."""
    from medical_segmentation_pytorch_amd.ops.losses import ohem_cross_entropy
    torch.manual_seed(3)
    x = torch.randn(2, 2, 32, 32, device=gpu, requires_grad=True)
    tgt = torch.randint(0, 2, (2, 32, 32), device=gpu)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm-up outside the capture
        ohem_cross_entropy(x, tgt).backward()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    x.grad = None
    with torch.cuda.graph(g):
        out = ohem_cross_entropy(x, tgt)
        out.backward()
    for scale in (1.0, 0.05, 4.0):   # 0.05: confident logits -> the top-k branch
        with torch.no_grad():
            x.copy_(torch.randn_like(x) * scale)
            tgt.copy_(torch.randint(0, 2, tgt.shape, device=gpu))
            x.grad.zero_()
        g.replay()
        torch.cuda.synchronize()
        xr = x.detach().clone().requires_grad_(True)
        ref = _ohem_ref(xr, tgt, 0.7)
        ref.backward()
        assert abs(out.item() - ref.item()) < 1e-5, (scale, out.item(), ref.item())
        assert _rel(x.grad, xr.grad) < 1e-4


@pytest.mark.parametrize('deferred_identity', [False, True])
def test_res_tail_bitwise_and_parked_identity_gradient(gpu, deferred_identity):
    """ResNet block tail in one pass (``bn_add_act``) is bitwise the materialise + add_act chain; its
    backward parks the identity gradient for conv1, whose data-gradient epilogue adds it: dL/dx equals the
    autograd sum of the two contributions (to one bf16 rounding)."""
    from medical_segmentation_pytorch_amd.ops import pool
    from medical_segmentation_pytorch_amd.ops import conv as convmod
    from medical_segmentation_pytorch_amd.ops.bn import Deferred, materialize
    torch.manual_seed(3)
    n, h, w, c = 2, 12, 20, 64
    yd = torch.randn(n, h, w, c, device=gpu).to(torch.bfloat16)
    x0 = torch.randn(n, h, w, c, device=gpu).to(torch.bfloat16)

    def stats():
        st = torch.zeros(4, c, device=gpu)
        st[0].uniform_(0.5, 1.5)
        st[1].uniform_(-0.5, 0.5)
        return st
    sa, sb = stats(), stats()
    m = nn.Conv2d(c, c, 1, bias=False).to(gpu)
    plan = ConvPlan(1, 1, c, c, [Branch(m.weight, 0, 0, 1)], padding=(0, 0))
    dz = torch.randn(n, h, w, c, device=gpu).to(torch.bfloat16)
    res = []
    for fused in (False, True):
        m.weight.grad = None
        x = x0.clone().requires_grad_(True)
        (c1,), _ = conv(plan, [x])   # conv1 of the block reads the block input; the tail consumes its chain
        t = c1 * 1.0   # (in a block, conv1's output gradient comes from bn1: never the tail's tensor)
        o = Deferred(t, sa, False)
        idt = Deferred(yd.clone().requires_grad_(True), sb, False) if deferred_identity else x
        if fused:
            z = pool.res_tail(o, idt, park_identity=not deferred_identity)
        else:
            z = pool.add_act(materialize(o), materialize(idt), relu=True)
        t.retain_grad()
        z.backward(dz)
        torch.cuda.synchronize()
        convmod.check_parked_grads()
        res.append((z.detach().clone(), t.grad.clone(), x.grad.clone(), m.weight.grad.clone()))
    (z0, t0, x0g, w0), (z1, t1, x1g, w1) = res
    assert torch.equal(z0, z1)
    assert torch.equal(t0, t1)
    # the epilogue adds the parked gradient to the fp32 accumulator and rounds once (autograd rounds the
    # dgrad to bf16, then adds): within a bf16 rounding, not bitwise
    assert _rel(x1g, x0g) < 4e-3
    assert torch.equal(w0, w1)


def test_parked_gradient_aliasing_its_own_dy_is_not_overwritten(gpu):
    """A parked identity gradient that is also the conv's own dY (conv output read by the tail directly)
    must not be accumulated into in place: the weight gradient reads dY after the data-gradient."""
    from medical_segmentation_pytorch_amd.ops import pool
    from medical_segmentation_pytorch_amd.ops.bn import Deferred, materialize
    torch.manual_seed(5)
    n, h, w, c = 2, 8, 12, 64
    x0 = torch.randn(n, h, w, c, device=gpu).to(torch.bfloat16)
    st = torch.zeros(4, c, device=gpu)
    st[0] = 1.0
    m = nn.Conv2d(c, c, 1, bias=False).to(gpu)
    plan = ConvPlan(1, 1, c, c, [Branch(m.weight, 0, 0, 1)], padding=(0, 0))
    dz = torch.randn(n, h, w, c, device=gpu).to(torch.bfloat16)
    res = []
    for fused in (False, True):
        m.weight.grad = None
        x = x0.clone().requires_grad_(True)
        (c1,), _ = conv(plan, [x])
        o = Deferred(c1, st, False)
        z = pool.res_tail(o, x, park_identity=True) if fused else pool.add_act(materialize(o), x, relu=True)
        z.backward(dz)
        torch.cuda.synchronize()
        res.append((x.grad.clone(), m.weight.grad.clone()))
    assert _rel(res[1][0], res[0][0]) < 4e-3
    assert torch.equal(res[1][1], res[0][1])



@pytest.mark.parametrize('c,groups,stride', [(128, 32, 1), (64, 32, 2), (256, 32, 1), (512, 32, 2), (1024, 32, 1),
                                             (64, 8, 1), (48, 48, 1), (192, 192, 2), (96, 96, 2), (96, 96, 1),
                                             (256, 4, 1), (128, 2, 2), (96, 6, 1), (96, 6, 2)])
def test_grouped_conv_matches_fp32(gpu, c, groups, stride):
    """HIP grouped 3x3 (csrc/gconv.hip; ResNeXt conv2, CG = 4..32 channels per group, stride 1 / 2) vs the
    fp32 PyTorch conv on the same bf16 inputs: output, input gradient and weight gradient."""
    from medical_segmentation_pytorch_amd.ops.gconv import gconv
    torch.manual_seed(8)
    n, h, w = 2, 14, 18
    m = nn.Conv2d(c, c, 3, stride, 1, groups=groups, bias=False).to(gpu)
    x = torch.randn(n, h, w, c, device=gpu).to(torch.bfloat16)
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    wr = m.weight.detach().float().clone().requires_grad_(True)
    ref = F.conv2d(xr, wr, None, stride, 1, 1, groups)
    g = torch.randn_like(ref).to(torch.bfloat16)
    ref.backward(g.float())
    xf = x.clone().requires_grad_(True)
    y = gconv(xf, m)
    y.backward(g.permute(0, 2, 3, 1).contiguous())
    assert y.shape == (n, ref.shape[2], ref.shape[3], c)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 1e-2
    assert _rel(xf.grad.permute(0, 3, 1, 2), xr.grad) < 1e-2
    assert _rel(m.weight.grad, wr.grad) < 1e-3


@pytest.mark.parametrize('c,groups,stride', [(128, 32, 1), (256, 32, 2), (1024, 32, 2), (256, 4, 1)])
def test_grouped_conv_mfma_matches_valu(gpu, c, groups, stride, monkeypatch):
    """The MFMA grouped 3x3 (gconv_mfma: block-diagonal weights over a max(16, CG) window) against the VALU
    kernels on the same bf16 inputs: both accumulate in fp32, so outputs and input gradients agree to bf16
    rounding, weight gradients to fp32 summation order; the MFMA path is the one the ResNeXt shapes take."""
    from medical_segmentation_pytorch_amd.ops import gconv as G
    torch.manual_seed(9)
    m = nn.Conv2d(c, c, 3, stride, 1, groups=groups, bias=False).to(gpu)
    x = torch.randn(3, 13, 21, c, device=gpu).to(torch.bfloat16)
    assert G._mfma_ok(c, c // groups, 9)
    out = []
    for mfma in (True, False):
        monkeypatch.setattr(G, '_MFMA', mfma)
        xf = x.clone().requires_grad_(True)
        y = G.gconv(xf, m)
        g = torch.randn_like(y, dtype=torch.float32).mul(0.5).to(torch.bfloat16) if not out else out[0][2]
        m.weight.grad = None
        y.backward(g)
        out.append((y.detach().float(), xf.grad.float(), g, m.weight.grad.clone()))
    assert _rel(out[0][0], out[1][0]) < 5e-3
    assert _rel(out[0][1], out[1][1]) < 5e-3
    assert _rel(out[0][3], out[1][3]) < 1e-4   # both fp32 accumulations of the same bf16 products


def test_relu6_forward_backward(gpu):
    """ReLU6 on the HIP elementwise kernels (MobileNetV2) vs torch's hardtanh: bitwise on bf16."""
    from medical_segmentation_pytorch_amd.ops.elementwise import relu6
    torch.manual_seed(2)
    x = (torch.randn(2, 8, 9, 16, device=gpu) * 5).to(torch.bfloat16)
    g = torch.randn_like(x)
    xr = x.clone().requires_grad_(True)
    ref = F.relu6(xr)
    ref.backward(g)
    xf = x.clone().requires_grad_(True)
    y = relu6(xf)
    y.backward(g)
    assert torch.equal(y, ref)
    assert torch.equal(xf.grad, xr.grad)


def test_bn_relu6_one_pass_matches_two_pass(gpu, monkeypatch):
    """MobileNetV2's BN -> ReLU6 as ONE apply pass (ops.elementwise._BNReLU6, bn_act_apply_relu6) is bitwise
    the materialised BN output followed by the ReLU6 pass, forward and backward."""
    from medical_segmentation_pytorch_amd.ops import elementwise as E
    from medical_segmentation_pytorch_amd.ops.bn import Deferred
    torch.manual_seed(6)
    P, Cp, C = 3 * 29 * 31, 24, 20
    t0 = (torch.randn(P, Cp, device=gpu) * 3).to(torch.bfloat16)
    t0[:, C:] = 0
    stats = torch.zeros(4, Cp, device=gpu)
    stats[0, :C] = torch.rand(C, device=gpu) * 2 + 0.5
    stats[1, :C] = torch.randn(C, device=gpu) * 2
    g = torch.randn(P, Cp, device=gpu).to(torch.bfloat16)
    out = []
    for fused in (True, False):
        monkeypatch.setattr(E, '_BN_RELU6', fused)
        t = t0.clone().requires_grad_(True)
        y = E.relu6(Deferred(t, stats, False))
        y.backward(g)
        out.append((y.detach(), t.grad))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])
    assert out[0][0].max().item() == 6.0 and out[0][0].min().item() == 0.0
