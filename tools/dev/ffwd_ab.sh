#!/bin/bash
# Dev (round 5): fused forward (conv_fwd_fused) -- numerics tests, conv_bench levels 1-2 with the fused forward
# on / off (MSP_CONV_FWD_FUSED), then the bench -> gpurun_out/<tag>/
set -e -o pipefail
tag=${1:-ffwd}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_bwd_oracle.py tests/test_gpu_kernels.py tests/test_gpu_deferred_dy.py \
  tests/test_gpu_conv_gemm.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
for m in 0 1; do
  MSP_CONV_FWD_FUSED=$m timeout -k 10 300 python -u tools/conv_bench.py --batch 320 --iters 5 --levels ${LEVELS:-1,2} 2>/dev/null > $out/ffwd$m.log
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err
