#!/bin/bash
# Dev (round 5): fused forward knock-outs (tools/dev/fused_bwd_bench.py ... fwd) for the default build and the
# variants in $VARIANTS -> gpurun_out/<tag>/bench.log
set -e -o pipefail
tag=${1:-ffko}
out=gpurun_out/$tag
mkdir -p $out
for v in default ${VARIANTS}; do
  so=""
  [ "$v" != default ] && so=build/$v/_C.so
  for d in 1 3; do
    MSP_C_SO=$so timeout -k 10 120 python -u tools/dev/fused_bwd_bench.py 320 352 $d 1 fwd 2>&1 | { grep -v amdgpu.ids || true; } >> $out/bench.log
  done
done
