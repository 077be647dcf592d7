"""Import-path parity with the reference's ``models/modules.py``: user code doing
``from models.modules import ConvBNAct`` keeps working.  The implementations live in :mod:`.layers`."""
from .layers import (Activation, ConvBNAct, DeConvBNAct, DSConvBNAct, DWConvBNAct, PWConvBNAct,  # noqa: F401
                     PyramidPoolingModule, SegHead, channel_shuffle, conv1x1, conv3x3)
