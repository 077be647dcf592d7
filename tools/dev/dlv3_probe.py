"""Dev: per-stage encoder feature parity of the fused executor vs eager fp32 on DeepLabV3(resnet18)
(dilated, output stride 8), with the GEMM conv path on and off."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from medical_segmentation_pytorch_amd.models import smp  # noqa: E402
from medical_segmentation_pytorch_amd.ops import _ext  # noqa: E402
from medical_segmentation_pytorch_amd.ops.bn import materialize  # noqa: E402
from medical_segmentation_pytorch_amd.ops.fm import from_fm  # noqa: E402
from medical_segmentation_pytorch_amd.runtime.fused_model import FusedExecutor  # noqa: E402


def cos(a, b):
    return F.cosine_similarity(a.flatten().float(), b.flatten().float(), dim=0).item()


C = _ext.require()
gpu = torch.device('cuda', 0)
torch.manual_seed(0)
model = smp.DeepLabV3(encoder_name='resnet18', encoder_weights=None, in_channels=3, classes=2).to(gpu).eval()
x = torch.randn(4, 3, 128, 128, device=gpu)
with torch.no_grad(), torch.backends.cudnn.flags(enabled=False):
    ref = model.encoder(x)
for gemm in (True, False):
    C.conv_set_gemm(gemm)
    ex = FusedExecutor(model)
    with torch.no_grad():
        feats = ex.resnet_encoder(model.encoder, x, False)
    chans = list(model.encoder.out_channels[1:])
    print('gemm', gemm, [round(cos(from_fm(materialize(f), c), r), 4) for f, c, r in zip(feats, chans, ref[1:])],
          flush=True)
    for name, m in model.encoder.named_modules():
        if isinstance(m, torch.nn.Conv2d) and gemm:
            print('  ', name, m.in_channels, m.out_channels, m.kernel_size, m.stride, m.padding, m.dilation)
