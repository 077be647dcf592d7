#!/usr/bin/env python3
"""Dev probe: do independent L1/L2 convs (the DUCK block's parallel branches) gain from running on
concurrent HIP streams?  Times K independent convs issued on one stream vs spread over K streams.
    python tools/dev/stream_probe.py [batch] [K]"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from medical_segmentation_pytorch_amd.ops.conv import Branch, ConvPlan, conv  # noqa: E402


def run(label, fns, streams, iters=10):
    main = torch.cuda.current_stream()
    for _ in range(2):
        for f in fns:
            f()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(iters):
        if streams is None:
            for f in fns:
                f()
        else:
            for s, f in zip(streams, fns):
                s.wait_stream(main)
                with torch.cuda.stream(s):
                    f()
            for s in streams:
                main.wait_stream(s)
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / iters
    print(f'{label:40s} {ms:8.3f} ms per round of {len(fns)} convs', flush=True)
    return ms


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    for c, hw in ((17, 352), (34, 176)):
        plans, xs = [], []
        for k in range(K):
            m = nn.Conv2d(c, c, 3, padding=1 + (k % 3), dilation=1 + (k % 3), bias=False).to(dev)
            plans.append(ConvPlan(3, 3, c, c, [Branch(m.weight, 0, 0, 9)], padding=m.padding, dilation=m.dilation))
            xs.append(torch.randn(batch, hw, hw, (c + 7) // 8 * 8, device=dev).to(torch.bfloat16))
        fns = [lambda p=p, x=x: conv(p, [x], want_stats=True) for p, x in zip(plans, xs)]
        streams = [torch.cuda.Stream() for _ in range(K)]
        a = run(f'L{1 if c == 17 else 2} {K}x 3x3 {c}ch bs{batch}: one stream', fns, None)
        b = run(f'L{1 if c == 17 else 2} {K}x 3x3 {c}ch bs{batch}: {K} streams', fns, streams)
        print(f'  concurrency gain {a / b:.2f}x', flush=True)


if __name__ == '__main__':
    main()
