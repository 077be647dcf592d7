"""Direct fp32 oracle of the fused narrow-conv backward (csrc/conv_bwd.hip ``conv_bwd_fused``): the kernel's
data-gradient, weight-gradient split-K slabs and upstream-BN backward partials against ``F.conv2d``'s
input / weight gradients in fp32 on the same bf16 operands -- not against the materialised HIP path.

Chain case of the DUCKNet L1 level (reference models/ducknet.py:95-96,144-179): BN1 -> conv -> BN2, with
  * x  = relu(BN1(y1)) rebuilt from y1 by the staging prologue (xc), y1 also the BN epilogue's input (the
    kernel rebuilds y1 from the staged x tile),
  * dY = bwd(dz2, y2) rebuilt from the deferred BN2 backward (bwd1 in csrc/common.h),
for Go = 1 (3x3 at dilation 1 / 2 / 3, 1x7, 7x1) and Go = 2 (the ResidualBlock's 3x3 + 1x1 pair), padded
widths 8 / 16 / 24 (17 real) / 32 channels and the 34-channel level's 40 / 48 (three 16-channel blocks), on grids
of several tiles and blocks (MI355X only).

The same kernel's FORWARD mode (``conv_fwd_fused``: the 17-channel level's forward convs) is scored the same way:
y = conv(relu(BN(x))) (+ bias) against ``F.conv2d`` in fp32 and its BN-statistics partials against the sums of
the stored output, for symmetric and one-sided tap sets, and against the halo kernel it replaces."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CASES = [
    # n, h, w, ci, co, (kh, kw), dil, go
    (3, 40, 56, 17, 17, (3, 3), 1, 1),
    (2, 33, 70, 17, 17, (3, 3), 2, 1),
    (2, 45, 38, 16, 16, (3, 3), 3, 1),
    (2, 30, 66, 17, 17, (1, 7), 1, 1),
    (2, 66, 30, 17, 17, (7, 1), 1, 1),
    (2, 36, 52, 8, 8, (3, 3), 1, 1),
    (2, 28, 44, 32, 32, (3, 3), 1, 1),
    (3, 40, 56, 17, 17, (3, 3), 1, 2),
    (2, 31, 47, 16, 16, (3, 3), 1, 2),
    # 34-channel level (40 padded: three 16-channel blocks, 256-pixel tiles; the dilated halos in 128-pixel ones)
    (2, 36, 52, 34, 34, (3, 3), 1, 1),
    (2, 30, 44, 34, 34, (3, 3), 2, 1),
    (1, 45, 38, 34, 34, (3, 3), 3, 1),
    (2, 44, 30, 34, 34, (7, 1), 1, 1),
    (2, 28, 66, 34, 34, (1, 7), 1, 1),
    (1, 30, 40, 40, 24, (3, 3), 1, 1),
    # the 8-channel image input (the first DUCK's convs) into 17 channels: single and pair
    (2, 36, 44, 8, 17, (3, 3), 1, 1),
    (2, 33, 41, 8, 17, (3, 3), 1, 2),
    # the 34-channel level's 3x3 + 1x1 pair: two stacked 40-channel dY groups, 128-pixel tiles
    (2, 36, 52, 34, 34, (3, 3), 1, 2),
    (1, 29, 43, 40, 40, (3, 3), 1, 2),
]


@pytest.mark.parametrize('acc', [False, True])
@pytest.mark.parametrize('case', CASES)
def test_fused_bwd_vs_fp32_conv_grads(gpu, case, acc):
    """``acc``: the accumulate epilogue (dx += this launch's data-gradient, the DUCK first convs' sibling launches)
    on a pre-filled dx, without the BN epilogue (the kernel takes one or the other)."""
    from medical_segmentation_pytorch_amd.ops._ext import require
    from medical_segmentation_pytorch_amd.ops.conv import Branch, ConvPlan, _taps
    from medical_segmentation_pytorch_amd.ops.fm import cpad
    C = require()
    n, h, w, ci, co, (kh, kw), dil, go = case
    g = torch.Generator(device=gpu).manual_seed(11)
    T = kh * kw
    pad = (dil * (kh // 2), dil * (kw // 2))
    W0 = torch.randn(co, ci, kh, kw, device=gpu, generator=g) * 0.2
    branches = [Branch(W0, 0, 0, T)]
    ws = [W0]
    if go == 2:   # the 1x1 shortcut at the centre tap (runtime.fused_model.plan_fused3x3)
        W1 = torch.randn(co, ci, 1, 1, device=gpu, generator=g) * 0.2
        branches.append(Branch(W1, 1, T // 2, 1))
        ws.append(W1)
    plan = ConvPlan(kh, kw, ci, co, branches, padding=pad, dilation=(dil, dil), Go=go)
    cp, cq = cpad(ci), cpad(co)
    dims = plan.fwd_dims(n, h, w, h, w)
    tdy, tdx = _taps(plan.taps_fwd)
    nblk = C.conv_bwd_fused_blocks(dims, tdy, tdx)
    assert nblk > 1, 'the case must span several blocks'

    def fm(t, c):   # NCHW fp32 -> NHWC bf16 padded to c channels
        o = torch.zeros(t.shape[0], t.shape[2], t.shape[3], c, device=gpu, dtype=torch.bfloat16)
        o[..., :t.shape[1]] = t.permute(0, 2, 3, 1).to(torch.bfloat16)
        return o

    def nchw(t, c):
        return t[..., :c].permute(0, 3, 1, 2).float()

    # BN1 (the conv's input BN): y1 -> x = relu(sc1 * y1 + sh1), its backward coefficients' mean row
    y1 = fm(torch.randn(n, ci, h, w, device=gpu, generator=g), cp)
    st1 = torch.zeros(4, cp, device=gpu)
    st1[0, :ci] = torch.rand(ci, device=gpu, generator=g) + 0.5
    st1[1, :ci] = torch.randn(ci, device=gpu, generator=g) * 0.3
    st1[2, :ci] = torch.randn(ci, device=gpu, generator=g) * 0.2   # mean (BN epilogue centring)
    x = _bf(torch.relu(nchw(y1, ci) * st1[0, :ci].view(1, -1, 1, 1) + st1[1, :ci].view(1, -1, 1, 1)))
    # BN2 of each output group: dY = k1 * [sc2 * y2 + sh2 > 0] * dz2 + k2 * y2 + k3
    dzs, y2s, st2s, k2s, dYs = [], [], [], [], []
    for _ in range(go):
        dz = fm(torch.randn(n, co, h, w, device=gpu, generator=g), cq)
        y2 = fm(torch.randn(n, co, h, w, device=gpu, generator=g), cq)
        st2 = torch.zeros(4, cq, device=gpu)
        st2[0, :co] = torch.rand(co, device=gpu, generator=g) + 0.5
        st2[1, :co] = torch.randn(co, device=gpu, generator=g) * 0.3
        k = torch.zeros(3, cq, device=gpu)
        k[0, :co] = torch.rand(co, device=gpu, generator=g) + 0.5
        k[1, :co] = torch.randn(co, device=gpu, generator=g) * 0.1
        k[2, :co] = torch.randn(co, device=gpu, generator=g) * 0.1
        y2f, dzf = nchw(y2, co), nchw(dz, co)
        v = lambda r: r[:co].view(1, -1, 1, 1)  # noqa: E731
        mask = (y2f * v(st2[0]) + v(st2[1])) > 0
        dYs.append(_bf(v(k[0]) * torch.where(mask, dzf, torch.zeros_like(dzf)) + v(k[1]) * y2f + v(k[2])))
        dzs.append(dz); y2s.append(y2); st2s.append(st2); k2s.append(k)
    # fp32 oracle: conv input / weight gradients on the bf16 operands
    wb = [_bf(t) for t in ws]
    dx_ref = F.grad.conv2d_input(x.shape, wb[0], dYs[0], padding=pad, dilation=dil)
    dw_ref = [F.grad.conv2d_weight(x, wb[0].shape, dYs[0], padding=pad, dilation=dil)]
    if go == 2:
        dx_ref = dx_ref + F.grad.conv2d_input(x.shape, wb[1], dYs[1])
        dw_ref.append(F.grad.conv2d_weight(x, wb[1].shape, dYs[1]))
    # the kernel
    wd, kp = plan.pack_dgrad(gpu)
    dxt = torch.empty(n, h, w, cp, dtype=torch.bfloat16, device=gpu)
    if acc:
        dxt.zero_()
        dxt[..., :ci] = torch.randn(n, h, w, ci, device=gpu, generator=g).to(torch.bfloat16)
        dx_ref = dx_ref + nchw(dxt, ci)
    part = torch.empty(nblk, 2, cp, device=gpu)
    dwp = torch.empty(nblk * plan.rows * plan.T * plan.Cip, device=gpu)
    kw2 = {}
    if go == 2:
        kw2 = dict(dz2=dzs[1], gy2=y2s[1], gs2=st2s[1], gk2=k2s[1], grelu2=True, t1=T // 2)
    C.conv_bwd_fused(dzs[0], y2s[0], st2s[0], k2s[0], True, y1, st1, True, wd, kp, dxt, None if acc else y1,
                     None if acc else st1[:3].contiguous(), True, None if acc else part, dwp, dims, tdy, tdx,
                     accumulate=acc, **kw2)
    torch.cuda.synchronize()
    dx = nchw(dxt, ci)
    assert torch.isfinite(dx).all()
    assert _rel(dx, dx_ref) < 1e-2, _rel(dx, dx_ref)
    if cp > ci:
        assert dxt[..., ci:].float().abs().max().item() == 0.0   # padding channels stay zero
    slab = dwp.view(nblk, plan.rows, plan.T, plan.Cip).sum(0)   # fixed-order split-K sum (as unpack_wgrad)
    for gi, ref in enumerate(dw_ref):
        got = slab[gi * cq:gi * cq + co, :, :ci]                   # [co][t][ci]
        if gi == 0:
            got = got.permute(0, 2, 1).reshape(co, ci, kh, kw)
        else:
            got = got[:, T // 2, :].reshape(co, ci, 1, 1)
        assert _rel(got, ref) < 1e-2, (gi, _rel(got, ref))
    if acc:
        return
    # BN1 backward partials of the kernel's own (bf16) data-gradient: sum g, sum g * (y1 - mean)
    y1f = nchw(y1, ci)
    m1 = (y1f * st1[0, :ci].view(1, -1, 1, 1) + st1[1, :ci].view(1, -1, 1, 1)) > 0
    gm = torch.where(m1, dx, torch.zeros_like(dx))
    s_ref = gm.sum((0, 2, 3))
    q_ref = (gm * (y1f - st1[2, :ci].view(1, -1, 1, 1))).sum((0, 2, 3))
    p = part.sum(0)
    assert _rel(p[0, :ci], s_ref) < 2e-3, _rel(p[0, :ci], s_ref)
    assert _rel(p[1, :ci], q_ref) < 2e-2, _rel(p[1, :ci], q_ref)


FWD_CASES = [
    # n, h, w, ci, co, (kh, kw), pad, dil, prologue, bias
    (3, 40, 56, 17, 17, (3, 3), (1, 1), 1, True, False),
    (2, 33, 70, 17, 17, (3, 3), (2, 2), 2, True, False),
    (2, 45, 38, 16, 16, (3, 3), (3, 3), 3, False, False),
    (2, 30, 66, 17, 17, (1, 7), (0, 3), 1, True, False),
    (2, 66, 30, 17, 17, (7, 1), (3, 0), 1, True, True),
    (2, 36, 52, 8, 24, (3, 3), (1, 1), 1, False, True),
    (2, 28, 44, 32, 17, (3, 3), (1, 1), 1, True, False),
    (1, 37, 41, 24, 32, (3, 3), (0, 0), 1, False, False),   # one-sided taps (valid-padding geometry, same size)
    (2, 36, 52, 34, 34, (3, 3), (1, 1), 1, True, False),    # 34-channel level: three 16-channel blocks
    (2, 30, 66, 34, 40, (1, 7), (0, 3), 1, True, True),
]


@pytest.mark.parametrize('case', FWD_CASES)
def test_fused_forward_vs_fp32_conv(gpu, case):
    from medical_segmentation_pytorch_amd.ops._ext import require
    from medical_segmentation_pytorch_amd.ops.conv import Branch, ConvPlan, _taps
    from medical_segmentation_pytorch_amd.ops.fm import cpad
    C = require()
    n, h, w, ci, co, (kh, kw), pad, dil, pro, with_bias = case
    g = torch.Generator(device=gpu).manual_seed(21)
    W = torch.randn(co, ci, kh, kw, device=gpu, generator=g) * 0.2
    b = torch.randn(co, device=gpu, generator=g) if with_bias else None
    plan = ConvPlan(kh, kw, ci, co, [Branch(W, 0, 0, kh * kw)], padding=pad, dilation=(dil, dil), bias=b)
    cp, cq = cpad(ci), cpad(co)
    dims = plan.fwd_dims(n, h, w, h, w)
    dy, dx = _taps(plan.taps_fwd)
    assert C.conv_fwd_fused_ok(dims, dy, dx), 'the case must take the fused forward'
    x = torch.zeros(n, h, w, cp, device=gpu, dtype=torch.bfloat16)
    x[..., :ci] = torch.randn(n, h, w, ci, device=gpu, generator=g).to(torch.bfloat16)
    coefs, rmask = [None], 0
    xin = x[..., :ci].permute(0, 3, 1, 2).float()
    if pro:
        st = torch.zeros(4, cp, device=gpu)
        st[0, :ci] = torch.rand(ci, device=gpu, generator=g) + 0.5
        st[1, :ci] = torch.randn(ci, device=gpu, generator=g) * 0.3
        coefs, rmask = [st], 1
        xin = _bf(torch.relu(xin * st[0, :ci].view(1, -1, 1, 1) + st[1, :ci].view(1, -1, 1, 1)))
    wb = _bf(W)
    if pad == (0, 0):
        ref = F.conv2d(F.pad(xin, (0, 2 * dil, 0, 2 * dil)), wb, None, 1, 0, dil)
    else:
        ref = F.conv2d(xin, wb, None, 1, pad, dil)
    if b is not None:
        ref = ref + b.view(1, -1, 1, 1)
    nblk = C.conv_stat_blocks(dims, dy, dx)
    outs = {}
    for fused in (True, False):
        C.conv_set_fwd_fused(fused)
        try:
            y = torch.empty(n, h, w, cq, device=gpu, dtype=torch.bfloat16)
            part = torch.empty(C.conv_stat_blocks(dims, dy, dx), 2, plan.rows, device=gpu)
            bias = b.float().contiguous() if b is not None else None
            C.conv_fwd([x], plan.pack_fwd(gpu), [y], bias, part, dims, dy, dx, False, coefs, rmask)
            torch.cuda.synchronize()
            outs[fused] = (y, part)
        finally:
            C.conv_set_fwd_fused(True)
    y, part = outs[True]
    assert part.shape[0] == nblk
    got = y[..., :co].permute(0, 3, 1, 2).float()
    assert torch.isfinite(got).all()
    assert _rel(got, ref) < 1e-2, _rel(got, ref)
    if cq > co:
        assert y[..., co:].float().abs().max().item() == 0.0   # padding channels stay zero
    yh, ph = outs[False]
    assert _rel(got, yh[..., :co].permute(0, 3, 1, 2).float()) < 5e-3
    # BN statistics partials: of the stored bf16 output
    s_ref = got.sum((0, 2, 3))
    q_ref = (got * got).sum((0, 2, 3))
    p = part.sum(0)
    assert _rel(p[0, :co], s_ref) < 1e-3, _rel(p[0, :co], s_ref)
    assert _rel(p[1, :co], q_ref) < 1e-3, _rel(p[1, :co], q_ref)


PAIR_FWD_CASES = [
    # n, h, w, ci, co, prologue  (ResidualBlock 3x3 + 1x1 pair: co <= 24 -> 48 stacked rows, three 16-row blocks)
    (3, 40, 56, 17, 17, True),
    (2, 37, 45, 24, 24, False),
    (2, 33, 70, 8, 17, True),
    # the 34-channel level's pair: 2 x 40 = 80 stacked rows, five 16-row blocks
    (2, 36, 52, 34, 34, True),
    (2, 29, 43, 40, 40, False),
]


@pytest.mark.parametrize('case', PAIR_FWD_CASES)
def test_fused_pair_forward_vs_fp32_conv(gpu, case):
    """The ResidualBlock's 3x3 + 1x1 pair (one Go = 2 plan, the 1x1 at the centre tap) on the fused kernel's
    forward mode (48 or 80 stacked output rows): both output tensors and the stacked BN-statistics rows against fp32 convs, and the halo kernel."""
    from medical_segmentation_pytorch_amd.ops._ext import require
    from medical_segmentation_pytorch_amd.ops.conv import Branch, ConvPlan, _taps
    from medical_segmentation_pytorch_amd.ops.fm import cpad
    C = require()
    n, h, w, ci, co, pro = case
    g = torch.Generator(device=gpu).manual_seed(33)
    W3 = torch.randn(co, ci, 3, 3, device=gpu, generator=g) * 0.2
    W1 = torch.randn(co, ci, 1, 1, device=gpu, generator=g) * 0.3
    plan = ConvPlan(3, 3, ci, co, [Branch(W3, 0, 0, 9), Branch(W1, 1, 4, 1)], padding=(1, 1), Go=2)
    cp, cq = cpad(ci), cpad(co)
    dims = plan.fwd_dims(n, h, w, h, w)
    dy, dx = _taps(plan.taps_fwd)
    assert C.conv_fwd_fused_ok(dims, dy, dx), 'the pair must take the fused forward'
    x = torch.zeros(n, h, w, cp, device=gpu, dtype=torch.bfloat16)
    x[..., :ci] = torch.randn(n, h, w, ci, device=gpu, generator=g).to(torch.bfloat16)
    coefs, rmask = [None], 0
    xin = x[..., :ci].permute(0, 3, 1, 2).float()
    if pro:
        st = torch.zeros(4, cp, device=gpu)
        st[0, :ci] = torch.rand(ci, device=gpu, generator=g) + 0.5
        st[1, :ci] = torch.randn(ci, device=gpu, generator=g) * 0.3
        coefs, rmask = [st], 1
        xin = _bf(torch.relu(xin * st[0, :ci].view(1, -1, 1, 1) + st[1, :ci].view(1, -1, 1, 1)))
    refs = [F.conv2d(xin, _bf(W3), None, 1, 1), F.conv2d(xin, _bf(W1), None, 1, 0)]
    outs = {}
    for fused in (True, False):
        C.conv_set_fwd_fused(fused)
        try:
            ys = [torch.full((n, h, w, cq), float('nan'), device=gpu, dtype=torch.bfloat16) for _ in range(2)]
            part = torch.empty(C.conv_stat_blocks(dims, dy, dx), 2, plan.rows, device=gpu)
            C.conv_fwd([x], plan.pack_fwd(gpu), ys, None, part, dims, dy, dx, False, coefs, rmask)
            torch.cuda.synchronize()
            outs[fused] = (ys, part)
        finally:
            C.conv_set_fwd_fused(True)
    ys, part = outs[True]
    p = part.sum(0)
    for gi, (y, ref) in enumerate(zip(ys, refs)):
        got = y[..., :co].permute(0, 3, 1, 2).float()
        assert torch.isfinite(got).all()
        assert _rel(got, ref) < 1e-2, (gi, _rel(got, ref))
        if cq > co:
            assert y[..., co:].float().abs().max().item() == 0.0
        yh = outs[False][0][gi]
        assert _rel(got, yh[..., :co].permute(0, 3, 1, 2).float()) < 5e-3
        s_ref, q_ref = got.sum((0, 2, 3)), (got * got).sum((0, 2, 3))
        o = gi * cq
        assert _rel(p[0, o:o + co], s_ref) < 1e-3, (gi, _rel(p[0, o:o + co], s_ref))
        assert _rel(p[1, o:o + co], q_ref) < 1e-3, (gi, _rel(p[1, o:o + co], q_ref))
