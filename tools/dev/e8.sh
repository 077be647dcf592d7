#!/bin/bash
# Dev: wgrad NB=1 unroll A/B (L1/L2 conv bench), default bench, then the eager config baselines
set -e
out=gpurun_out/e8
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 200 python -u tools/conv_bench.py --batch 128 --iters 10 --levels 1,2 2>/dev/null > $out/cb.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err
bash tools/dev/eager_configs.sh
