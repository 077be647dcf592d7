#!/bin/bash
# Dev (round 5): fused narrow-conv kernels extended to the 34-channel level -- numerics tests, conv_bench level 2
# forward with the fused forward on / off, then the bench with the new eligibility -> gpurun_out/<tag>/
set -e -o pipefail
tag=${1:-l2ab}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_bwd_oracle.py tests/test_gpu_deferred_dy.py tests/test_gpu_kernels.py \
  tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
for m in 0 1; do
  MSP_CONV_FWD_FUSED=$m timeout -k 10 300 python -u tools/conv_bench.py --batch 320 --iters 5 --levels 2 2>/dev/null > $out/cb_ffwd$m.log
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err
