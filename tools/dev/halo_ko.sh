#!/bin/bash
# Dev: phase knock-outs of the halo conv kernel (profiling build, csrc/build.py MSP_BUILD_VARIANT=ko) over
# tools/conv_bench.py layers -> gpurun_out/halo_ko_<tag>.log.  MSP_HALO_DBG bits: 1 no y stores, 2 no
# staging loads, 4 no MFMAs, 8 no staging, 16 no epilogue, 32 no weight loads.  Timings only: knocked-out outputs are wrong.
set -e
tag=${1:-cur}
only=${2:-L1 fused8}
out=gpurun_out/halo_ko_$tag.log
: > $out
for dbg in ${DBGS:-0 8 16 24 1 4 28}; do
  echo "dbg=$dbg" >> $out
  MSP_C_SO=build/ko/_C.so MSP_HALO_DBG=$dbg timeout -k 10 120 python -u tools/conv_bench.py --batch 128 --iters 10 \
    --only "$only" 2>/dev/null | grep -v '^{' >> $out
done
