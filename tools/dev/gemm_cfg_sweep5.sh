#!/bin/bash
# Dev (round 5): GEMM tile-configuration sweep at the bench batch -> gpurun_out/<tag>/cfg_<fwd>_<wg>.log
set -e
tag=${1:-cfg5}
B=${BATCH:-320}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_gemm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/tests.log 2>&1
for pair in ${PAIRS:--1:-1 5:6 6:7 7:8 8:-1}; do
  f=${pair%%:*}; w=${pair##*:}
  MSP_CONV_GEMM_CFG=$f MSP_WGRAD_GEMM_CFG=$w timeout -k 10 300 python -u tools/conv_bench.py --batch $B --iters 5 --levels ${LEVELS:-3,4,5,6} 2>/dev/null > gpurun_out/$tag/cfg_${f}_${w}.log
done
