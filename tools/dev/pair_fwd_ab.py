"""Dev: run one pytest selection with the Go = 2 pair forward on the fused kernel (mode 1) or back on the halo
kernel (mode 2), in-process (conv_set_fwd_fused is module state).   usage: pair_fwd_ab.py <mode> <pytest args...>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pytest  # noqa: E402

from medical_segmentation_pytorch_amd.ops._ext import require  # noqa: E402

require().conv_set_fwd_fused(int(sys.argv[1]))
sys.exit(pytest.main(sys.argv[2:]))
