#!/bin/bash
# Dev (round 5): GEMM-kernel change A/B -- GEMM numerics tests, the >= 64-channel levels of conv_bench at the
# bench batch under the given fwd:wgrad config pairs, then the default bench -> gpurun_out/<tag>/
set -e
tag=${1:-abg}
B=${BATCH:-320}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_gemm.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
for pair in ${PAIRS:--1:-1}; do
  f=${pair%%:*}; w=${pair##*:}
  MSP_CONV_GEMM_CFG=$f MSP_WGRAD_GEMM_CFG=$w timeout -k 10 300 python -u tools/conv_bench.py --batch $B --iters 5 --levels ${LEVELS:-3,4,5,6} 2>/dev/null > $out/cfg_${f}_${w}.log
done
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err
fi
