"""Host-side conv launch planning (the extension's planners run on the CPU): the stat-partial rows a
forward allocates must equal the pixel-tile grid of the kernel that launch takes.  Regression: a strided
transposed conv (UNet / Linknet upsampling) from 64 input channels up was sized by the GEMM kernel's
grid while it runs on the gather kernel -> out-of-bounds stat writes."""
import pytest
import torch

from medical_segmentation_pytorch_amd.ops import _ext
from medical_segmentation_pytorch_amd.ops.conv import Branch, ConvPlan

pytestmark = pytest.mark.skipif(not _ext.available(), reason='HIP extension not built')


@pytest.mark.parametrize('cin,cout,k,op,n,h', [(512, 256, 3, 1, 2, 4), (256, 128, 3, 1, 2, 8), (128, 128, 4, 0, 2, 16),
                                              (64, 64, 4, 0, 4, 32), (32, 32, 3, 1, 2, 32)])
def test_transposed_stat_rows_match_gather_grid(cin, cout, k, op, n, h):
    C = _ext.require()
    w = torch.zeros(cin, cout, k, k)
    p = ConvPlan(k, k, cin, cout, [Branch(w, 0, 0, k * k)], stride=2, padding=(1, 1), transposed=True,
                 output_padding=op)
    oh, ow = p.out_hw(h, h)
    dims = p.fwd_dims(n, h, h, oh, ow)
    dy, dx = [t[0] for t in p.taps_bwd], [t[1] for t in p.taps_bwd]
    try:
        C.conv_set_gemm(False)
        C.conv_set_halo(False)
        gather = C.conv_stat_blocks(dims, dy, dx, False)   # the gather kernel's pixel-tile grid
    finally:
        C.conv_set_gemm(True)
        C.conv_set_halo(True)
    assert p.stat_blocks(n, h, h) == C.conv_stat_blocks(dims, dy, dx, True) == gather
