#!/bin/bash
# Dev: GEMM-kernel knock-outs (csrc/conv_gemm.hip, conv_wgrad_gemm.hip built with -DGK_KO_{MFMA,DMA,LDS} as
# side variants under build/ko_*) timed on the >= 64-channel DUCKNet levels -> gpurun_out/<tag>/ko_<variant>.log
set -e
tag=${1:-gemm_ko}
B=${BATCH:-320}
mkdir -p gpurun_out/$tag
for v in default ko_mfma ko_dma ko_lds; do
  so=""
  [ "$v" != default ] && so="build/$v/_C.so"
  MSP_C_SO=$so timeout -k 10 240 python -u tools/conv_bench.py --batch $B --iters 5 --levels ${LEVELS:-3,4,5,6} 2>/dev/null > gpurun_out/$tag/ko_$v.log
done
