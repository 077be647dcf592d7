"""MAnet position-attention products on ``csrc/attention.hip`` (``ops.attention.pab_attention``) against the
fp32 PyTorch reference of the same op -- ``softmax((center @ top^T).view(b, -1)).view(b, hw, hw) @ bottom``
(the smp MAnet PAB of the reference hub, models/__init__.py:8-10) -- forward and all three input gradients,
for the 352-input stride-32 map (hw = 121) and a ragged small one."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize('b,hw,p,c', [(2, 121, 64, 256), (3, 37, 16, 40), (1, 200, 64, 2048)])
def test_pab_attention_vs_fp32(gpu, b, hw, p, c):
    from medical_segmentation_pytorch_amd.ops.attention import pab_attention
    g = torch.Generator(device=gpu).manual_seed(5)
    center = (torch.randn(b, hw, p, device=gpu, generator=g) * 0.3).to(torch.bfloat16)
    top = (torch.randn(b, hw, p, device=gpu, generator=g) * 0.3).to(torch.bfloat16)
    bottom = torch.randn(b, hw, c, device=gpu, generator=g).to(torch.bfloat16)
    dout = torch.randn(b, hw, c, device=gpu, generator=g).to(torch.bfloat16)
    xs = [t.clone().requires_grad_(True) for t in (center, top, bottom)]
    out = pab_attention(*xs)
    out.backward(dout)
    rs = [t.float().clone().requires_grad_(True) for t in (center, top, bottom)]
    s = rs[0] @ rs[1].transpose(1, 2)
    prob = torch.softmax(s.reshape(b, -1), dim=1).reshape(b, hw, hw)
    ref = prob @ rs[2]
    ref.backward(dout.float())
    assert out.dtype == torch.bfloat16 and out.shape == (b, hw, c)
    assert _rel(out, ref) < 2e-2, _rel(out, ref)
    for got, want, name in zip(xs, rs, ('center', 'top', 'bottom')):
        assert torch.isfinite(got.grad.float()).all(), name
        assert _rel(got.grad, want.grad) < 5e-2, (name, _rel(got.grad, want.grad))
