#!/bin/bash
# Dev: kernel-change A/B -- conv numerics tests, L1/L2 conv bench, default bench -> gpurun_out/<tag>/
set -e
tag=${1:-ab}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prologue.py tests/test_gpu_conv_gemm.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 200 python -u tools/conv_bench.py --batch 128 --iters 10 --levels ${LEVELS:-1,2} 2>/dev/null > $out/cb.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > $out/models.log 2>&1
