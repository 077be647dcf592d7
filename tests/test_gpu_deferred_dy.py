"""Deferred BatchNorm data-gradient (``ops.bn.DeferredGrad``): a training BN whose input is a conv output
read by that BN only never writes dL/dy; the producing conv rebuilds it while staging its data-gradient
and weight-gradient loads (the halo kernels' BN-backward prologue, ``csrc/conv.hip`` BWD), or resolves it
(one ``bn_act_bwd_apply`` pass) when a launch cannot.  Every gradient must match the materialised path;
where the two paths plan identical launches the results are bitwise equal."""
import pytest
import torch
import torch.nn as nn

from medical_segmentation_pytorch_amd.ops import bn as bnmod
from medical_segmentation_pytorch_amd.ops.bn import BNState, BwdStatsHandle, bn_act, materialize
from medical_segmentation_pytorch_amd.ops.conv import Branch, ConvPlan, conv
from medical_segmentation_pytorch_amd.ops.fm import to_fm_reference

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-20)).item()


def _bf(t):
    return t.to(torch.bfloat16).float()


CASES = [
    # cin, co, (kh, kw), dilation, n 3x3 groups, n 1x1 groups, (n, h, w), chain (BN1 -> conv: BNE epilogue too)
    (17, 17, (3, 3), 1, 1, 0, (2, 24, 32), False),
    (17, 17, (3, 3), 1, 1, 0, (2, 24, 32), True),
    (17, 17, (3, 3), 2, 1, 0, (2, 24, 32), True),
    (17, 17, (3, 3), 3, 1, 0, (2, 24, 32), False),
    (17, 17, (1, 7), 1, 1, 0, (2, 24, 32), True),
    (17, 17, (7, 1), 1, 1, 0, (2, 24, 32), False),
    (34, 34, (3, 3), 1, 1, 0, (2, 24, 32), True),      # 40 padded channels (L2 width)
    (17, 17, (3, 3), 1, 1, 1, (2, 24, 32), False),     # Go = 2: 3x3 + 1x1 at the centre tap, both deferred
    (17, 17, (3, 3), 1, 5, 3, (2, 24, 32), False),     # DUCK fused-8: chunked data-gradient -> resolved
    (64, 64, (3, 3), 1, 1, 0, (2, 16, 16), False),     # >= 64 channels: GEMM kernels -> resolved
    (17, 17, (3, 3), 1, 1, 0, (12, 128, 128), True),   # 384 tiles > the 256-block persistent grid: blocks
                                                       # loop over tiles (the double-buffered staging)
    (17, 17, (3, 3), 1, 1, 1, (12, 128, 128), True),   # the Go = 2 fused backward (3x3 + centre 1x1), multi-tile
    (16, 16, (3, 3), 1, 1, 0, (4, 64, 96), True),      # 16 channels: 2 slots of a 3-slot pixel pitch (the third
                                                       # never staged: no K unit may read it)
    (17, 17, (3, 3), 2, 1, 1, (2, 40, 56), True),      # Go = 2, dilation 2
]


MODES = [  # (deferred BN data-gradient, fused data+weight-gradient kernel, deferred dY in the separate kernels)
    (True, False, True),     # the separate halo kernels' BN-backward prologue
    (True, True, False),     # the fused backward consuming the deferred gradient (the default)
    (False, True, False),    # the fused backward on a materialised dY
]


@pytest.mark.parametrize('mode', MODES)
@pytest.mark.parametrize('case', CASES)
def test_deferred_bn_data_gradient(gpu, case, mode, monkeypatch):
    from medical_segmentation_pytorch_amd.ops import conv as convmod
    cin, co, (kh, kw), dil, n3, n1, (n, h, w), chain = case
    torch.manual_seed(5)
    convs = [nn.Conv2d(cin, co, (kh, kw), 1, (dil * (kh // 2), dil * (kw // 2)), (dil, dil), bias=False).to(gpu)
             for _ in range(n3)]
    convs += [nn.Conv2d(cin, co, 1, bias=False).to(gpu) for _ in range(n1)]
    bns = [nn.BatchNorm2d(co).to(gpu) for _ in range(n3 + n1)]
    bn1 = nn.BatchNorm2d(cin).to(gpu)
    with torch.no_grad():
        for b in bns + [bn1]:
            b.weight.uniform_(0.5, 1.5)
            b.bias.uniform_(-0.5, 0.5)
    T = kh * kw
    branches = [Branch(m.weight, g, 0, T) for g, m in enumerate(convs[:n3])]
    branches += [Branch(m.weight, n3 + g, T // 2, 1) for g, m in enumerate(convs[n3:])]
    x0 = to_fm_reference(_bf(torch.randn(n, cin, h, w, device=gpu, generator=torch.Generator(gpu).manual_seed(3))))
    gs = [to_fm_reference(_bf(torch.randn(n, co, h, w, device=gpu, generator=torch.Generator(gpu).manual_seed(9 + g))))
          for g in range(n3 + n1)]
    res, resolved = [], []
    for defer, fused, separate in ((False, False, False), mode):
        monkeypatch.setattr(bnmod, 'DEFER_DY', defer)
        monkeypatch.setattr(convmod, 'FUSED_BWD', fused)
        monkeypatch.setattr(convmod, 'DEFER_SEPARATE', separate)
        for m in convs + bns + [bn1]:
            for p in m.parameters():
                p.grad = None
        # the running statistics must not drift between the two passes
        state = [{k: v.clone() for k, v in b.state_dict().items()} for b in bns + [bn1]]
        plan = ConvPlan(kh, kw, cin, co, branches, padding=(dil * (kh // 2), dil * (kw // 2)), dilation=(dil, dil),
                        Go=n3 + n1)
        x = x0.clone().requires_grad_(True)
        hdl = None
        if chain:   # BN1 -> this conv only: its data-gradient also emits BN1's backward partials (BNE)
            hdl = BwdStatsHandle()
            xin = bn_act([x], BNState.from_module(bn1), True, True, None, handle=hdl, deferred=True, defer_bwd=True)
        else:
            xin = x
        ys, _ = conv(plan, [xin], want_stats=False, bn_handle=hdl)
        zs = [materialize(bn_act([y], BNState.from_module(b), True, True, None, deferred=True, defer_bwd=True))
              for y, b in zip(ys, bns)]
        n_before = len(bnmod._DEFERRED)
        torch.autograd.backward(zs, gs)
        torch.cuda.synchronize()
        resolved.append(len(bnmod._DEFERRED))
        res.append([x.grad.float().clone()] + [m.weight.grad.clone() for m in convs] +
                   [t.grad.clone() for b in bns for t in (b.weight, b.bias)])
        for b, sd in zip(bns + [bn1], state):
            b.load_state_dict(sd)
        assert n_before == 0
        bnmod.clear_deferred()
    for i, (a, b) in enumerate(zip(res[1], res[0])):
        assert _rel(a, b) < 1e-3, (i, _rel(a, b))
    # every token was claimed by its producer or resolved: nothing is left behind after the backward
    assert resolved == [0, 0], resolved


def test_deferred_tokens_reach_the_halo_prologue(gpu, monkeypatch):
    """The narrow single-group case really consumes the token in the kernels (no resolve pass): with
    the apply launch disabled, the deferred path still produces the materialised path's gradients."""
    C = bnmod.require()
    calls = []
    orig = bnmod.resolve

    from medical_segmentation_pytorch_amd.ops import conv as convmod
    monkeypatch.setattr(bnmod, 'DEFER_DY', True)
    monkeypatch.setattr(convmod, 'FUSED_BWD', False)
    monkeypatch.setattr(convmod, 'DEFER_SEPARATE', True)

    def spy(g):
        calls.append(bnmod.peek_deferred(g) is not None)
        return orig(g)
    monkeypatch.setattr(bnmod, 'resolve', spy)
    import medical_segmentation_pytorch_amd.ops.bn as b2
    assert b2.resolve is spy
    torch.manual_seed(1)
    m = nn.Conv2d(17, 17, 3, 1, 1, bias=False).to(gpu)
    bnm = nn.BatchNorm2d(17).to(gpu)
    plan = ConvPlan(3, 3, 17, 17, [Branch(m.weight, 0, 0, 9)], padding=(1, 1))
    x = to_fm_reference(_bf(torch.randn(2, 17, 24, 32, device=gpu))).requires_grad_(True)
    dims = plan.fwd_dims(2, 24, 32, 24, 32)
    assert C.conv_wgrad_uses_halo(dims, [t[0] for t in plan.taps_fwd], [t[1] for t in plan.taps_fwd], False)
    (y,), _ = conv(plan, [x])
    z = materialize(bn_act([y], BNState.from_module(bnm), True, True, None, deferred=True, defer_bwd=True))
    z.backward(torch.randn_like(z))
    assert not any(calls), 'the single 17-channel 3x3 conv must consume the deferred gradient in its kernels'
    assert x.grad is not None and torch.isfinite(x.grad.float()).all()


def test_fused_backward_runs_for_the_residual_pair(gpu, monkeypatch):
    """The ResidualBlock's 3x3 + 1x1 pair (Go = 2, the 1x1 at the centre tap) takes the fused backward and
    consumes both deferred BN gradients."""
    from medical_segmentation_pytorch_amd.ops import conv as convmod
    monkeypatch.setattr(bnmod, 'DEFER_DY', True)
    monkeypatch.setattr(convmod, 'FUSED_BWD', True)
    calls = []
    orig = convmod._fused_bwd

    def spy(*a, **k):
        r = orig(*a, **k)
        calls.append(r is not None)
        return r
    monkeypatch.setattr(convmod, '_fused_bwd', spy)
    torch.manual_seed(3)
    m3 = nn.Conv2d(17, 17, 3, 1, 1, bias=False).to(gpu)
    m1 = nn.Conv2d(17, 17, 1, bias=False).to(gpu)
    bns = [nn.BatchNorm2d(17).to(gpu) for _ in range(2)]
    plan = ConvPlan(3, 3, 17, 17, [Branch(m3.weight, 0, 0, 9), Branch(m1.weight, 1, 4, 1)], padding=(1, 1), Go=2)
    x = to_fm_reference(_bf(torch.randn(2, 17, 40, 48, device=gpu))).requires_grad_(True)
    ys, _ = conv(plan, [x])
    zs = [materialize(bn_act([y], BNState.from_module(b), True, True, None, deferred=True, defer_bwd=True))
          for y, b in zip(ys, bns)]
    torch.autograd.backward(zs, [torch.randn_like(z) for z in zs])
    torch.cuda.synchronize()
    assert calls == [True], calls
    assert not bnmod._DEFERRED


def test_fused_backward_runs_for_narrow_convs(gpu, monkeypatch):
    """The 17-channel 3x3 chain conv takes the fused data+weight-gradient kernel (one launch, no separate
    halo data-/weight-gradient launch) and consumes the deferred BN gradient without a resolve pass."""
    from medical_segmentation_pytorch_amd.ops import conv as convmod
    monkeypatch.setattr(bnmod, 'DEFER_DY', True)
    monkeypatch.setattr(convmod, 'FUSED_BWD', True)
    calls = []
    orig = convmod._fused_bwd

    def spy(*a, **k):
        r = orig(*a, **k)
        calls.append(r is not None)
        return r
    monkeypatch.setattr(convmod, '_fused_bwd', spy)
    torch.manual_seed(2)
    m = nn.Conv2d(17, 17, 3, 1, 2, 2, bias=False).to(gpu)
    bnm = nn.BatchNorm2d(17).to(gpu)
    plan = ConvPlan(3, 3, 17, 17, [Branch(m.weight, 0, 0, 9)], padding=(2, 2), dilation=(2, 2))
    x = to_fm_reference(_bf(torch.randn(2, 17, 40, 48, device=gpu))).requires_grad_(True)
    (y,), _ = conv(plan, [x])
    z = materialize(bn_act([y], BNState.from_module(bnm), True, True, None, deferred=True, defer_bwd=True))
    z.backward(torch.randn_like(z))
    torch.cuda.synchronize()
    assert calls == [True], calls
    assert not bnmod._DEFERRED


@pytest.mark.parametrize('go', [1, 8])
def test_deferred_dy_without_data_gradient(gpu, go, monkeypatch):
    """The first conv (input = the image, no data-gradient): the deferred BN gradients go straight into
    the halo weight-gradient's staging (no apply pass) and the weight gradients match the materialised path."""
    from medical_segmentation_pytorch_amd.ops import conv as convmod
    calls = []
    orig = bnmod.resolve

    def spy(g):
        calls.append(bnmod.peek_deferred(g) is not None)
        return orig(g)
    torch.manual_seed(4)
    convs = [nn.Conv2d(3, 17, 3, 1, 1, bias=False).to(gpu) for _ in range(go)]
    bns = [nn.BatchNorm2d(17).to(gpu) for _ in range(go)]
    plan = ConvPlan(3, 3, 3, 17, [Branch(m.weight, g, 0, 9) for g, m in enumerate(convs)], padding=(1, 1), Go=go)
    x = to_fm_reference(_bf(torch.randn(2, 3, 40, 56, device=gpu)))
    gs = [to_fm_reference(_bf(torch.randn(2, 17, 40, 56, device=gpu, generator=torch.Generator(gpu).manual_seed(9 + g))))
          for g in range(go)]
    res = []
    for defer in (False, True):
        monkeypatch.setattr(bnmod, 'DEFER_DY', defer)
        monkeypatch.setattr(bnmod, 'resolve', spy if defer else orig)
        for m in convs:
            m.weight.grad = None
        state = [{k: v.clone() for k, v in b.state_dict().items()} for b in bns]
        ys, _ = conv(plan, [x])
        zs = [materialize(bn_act([y], BNState.from_module(b), True, True, None, deferred=True, defer_bwd=True))
              for y, b in zip(ys, bns)]
        torch.autograd.backward(zs, gs)
        torch.cuda.synchronize()
        res.append([m.weight.grad.clone() for m in convs])
        for b, sd in zip(bns, state):
            b.load_state_dict(sd)
        bnmod.clear_deferred()
    for a, b in zip(res[1], res[0]):
        assert _rel(a, b) < 1e-3
    assert not any(calls), 'no apply pass: the weight-gradient staging rebuilds dY'
    assert convmod is not None
