#!/bin/bash
# Dev (round 5): fused backward compute-wave layout A/B (conv_bwd_fused_plan's CW rule vs forced 4 / 8):
# numerics tests under the default rule and forced CW = 8, the micro-bench at d = 1 / 2 / 3 and Go = 2 per
# setting, then the default bench -> gpurun_out/<tag>/
set -e -o pipefail
tag=${1:-fbcw}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_bwd_oracle.py tests/test_gpu_deferred_dy.py -x -q \
  --timeout 200 --timeout-method thread > $out/tests.log 2>&1
MSP_FB_CW=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_bwd_oracle.py -x -q \
  --timeout 200 --timeout-method thread > $out/tests_cw8.log 2>&1
for cw in 0 4 8; do
  for dg in "1 1" "2 1" "3 1" "1 2"; do
    MSP_FB_CW=$cw timeout -k 10 120 python -u tools/dev/fused_bwd_bench.py 320 352 $dg 2>&1 | { grep -v amdgpu.ids || true; } | sed "s/^/cw=$cw /" >> $out/bench.log
  done
done
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err
fi
