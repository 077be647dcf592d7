#!/bin/bash
# Dev (round 5): GEMM block-order sweep (MSP_GEMM_PXG pixel tiles per co-tile group) -> gpurun_out/<tag>/pxg_<p>.log
set -e
tag=${1:-pxg}
mkdir -p gpurun_out/$tag
for p in ${PXGS:-1 4 8 16 32 64}; do
  MSP_GEMM_PXG=$p timeout -k 10 300 python -u tools/conv_bench.py --batch ${BATCH:-320} --iters 5 --levels ${LEVELS:-3,4,5,6} 2>/dev/null > gpurun_out/$tag/pxg_$p.log
done
