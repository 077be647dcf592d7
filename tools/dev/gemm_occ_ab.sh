#!/bin/bash
# Dev (round 6): LDS-DMA GEMM tile configurations incl. the 3-4 blocks/CU BK-32 tiles, forced for every GEMM
# launch (fwd + dgrad), DUCKNet levels 3-6 at bs320 -> gpurun_out/gemm_occ/cfg_<c>.log
set -e
mkdir -p gpurun_out/gemm_occ
for c in ${CFGS:--1 9 10 11 12 13}; do
  timeout -k 10 200 python -u tools/conv_bench.py --batch ${BATCH:-320} --iters 5 --levels ${LEVELS:-3,4,5,6} \
    --gemm-cfg $c 2>/dev/null > gpurun_out/gemm_occ/cfg_$c.log
done
