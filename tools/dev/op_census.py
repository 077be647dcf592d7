"""Dev: census of ATen copy/fill ops issued by one fused training step (eager, no graph), by call site."""
import collections
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, '.')
from medical_segmentation_pytorch_amd.runtime.bench_step import build_bench_step  # noqa: E402

WATCH = ('copy_', 'fill_', 'zero_', 'zeros', 'zeros_like', 'clone', 'new_zeros', 'cat', '_to_copy')


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__
        if any(name.startswith(w) for w in WATCH):
            st = [f for f in traceback.extract_stack() if 'medical_segmentation' in f.filename or 'bench' in f.filename]
            site = f'{st[-1].filename.split("/")[-1]}:{st[-1].lineno} {st[-1].line}' if st else '?'
            self.c[(name, site)] += 1
        return func(*args, **(kwargs or {}))


dev = torch.device('cuda', 0)
step = build_bench_step(impl='fused', batch=8, size=128, base_channel=17, device=dev, use_graph=False)
for _ in range(2):
    step()
torch.cuda.synchronize()
m = Census()
with m:
    step()
torch.cuda.synchronize()
for (name, site), n in m.c.most_common(40):
    print(f'{n:6d}  {name:20s} {site}')
