#!/bin/bash
# Dev: kernel knock-outs -- side builds of the extension with profiling -D flags (csrc/build.py
# MSP_BUILD_VARIANT=<v> MSP_BUILD_DEFINES=...: GK_KO_{MFMA,DMA,LDS} for the GEMM convs, DW_KO_{LOAD,MFMA} for
# the halo weight-gradient) timed by tools/conv_bench.py -> gpurun_out/<tag>/ko_<variant>.log
#   VARIANTS="default ko_mfma ko_dma ko_lds" LEVELS=3,4,5,6 BATCH=320 EXTRA="--prologue" bash gemm_knockouts.sh <tag>
set -e
tag=${1:-gemm_ko}
B=${BATCH:-320}
mkdir -p gpurun_out/$tag
for v in ${VARIANTS:-default ko_mfma ko_dma ko_lds}; do
  so=""
  [ "$v" != default ] && so="build/$v/_C.so"
  MSP_C_SO=$so timeout -k 10 240 python -u tools/conv_bench.py --batch $B --iters 5 --levels ${LEVELS:-3,4,5,6} \
    ${EXTRA:-} 2>/dev/null > gpurun_out/$tag/ko_$v.log
done
