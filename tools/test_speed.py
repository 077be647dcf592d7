#!/usr/bin/env python3
"""Inference FPS benchmark -- reference ``tools/test_speed.py:9-67`` protocol: batch 1, 3 x (1024*r)
x (2048*r) input (r = 0.5 by default), 10 warm-ups, iteration count auto-calibrated to ~6 s,
synchronize + wall clock.  Runs the fused MI355X executor for DUCKNet/UNet (``--engine fused``,
default when available), otherwise eager PyTorch (optionally bf16 autocast with ``--amp``).
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from medical_segmentation_pytorch_amd.configs import MyConfig, load_parser  # noqa: E402
from medical_segmentation_pytorch_amd.models import get_model  # noqa: E402


def test_model_speed(config, ratio=0.5, imgw=2048, imgh=1024, iterations=None, seconds=6.0):
    if ratio != 1.0:
        assert ratio > 0, 'Ratio should be larger than 0.\n'
        imgw, imgh = int(imgw * ratio), int(imgh * ratio)
    device = torch.device('cuda')
    model = get_model(config).eval().to(device)
    fwd = model
    from medical_segmentation_pytorch_amd.utils.parallel import FusedModel, use_fused
    fused = use_fused(config, model, device)
    if fused:
        fwd = FusedModel(model).eval()
    print('\n=========Speed Testing=========')
    print(f'Model: {config.model}\nEncoder: {config.encoder}\nDecoder: {config.decoder}')
    print(f'Engine: {"fused MI355X" if fused else "eager"}\nSize (W, H): {imgw}, {imgh}')
    x = torch.randn(1, 3, imgh, imgw, device=device)
    amp = bool(getattr(config, 'amp_training', False)) and not fused
    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp):
        for _ in range(10):
            fwd(x)
        if iterations is None:
            elapsed, iterations = 0.0, 100
            while elapsed < 1:
                torch.cuda.synchronize()
                t0 = time.time()
                for _ in range(iterations):
                    fwd(x)
                torch.cuda.synchronize()
                elapsed = time.time() - t0
                iterations *= 2
            iterations = int(iterations / elapsed * seconds / 2)
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(iterations):
            fwd(x)
        torch.cuda.synchronize()
        latency = (time.time() - t0) / iterations * 1000
    torch.cuda.empty_cache()
    fps = 1000 / latency
    print(f'FPS: {fps}\n')
    return fps


if __name__ == '__main__':
    config = MyConfig()
    config.init_dependent_config()
    config = load_parser(config)
    test_model_speed(config)
