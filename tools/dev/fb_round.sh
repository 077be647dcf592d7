#!/bin/bash
# Dev (round 5): fused narrow-conv kernels + attention after a change -- numerics tests, the micro-benches for
# the default build and the knock-out variants in $VARIANTS, then the bench -> gpurun_out/<tag>/
set -e -o pipefail
tag=${1:-fbr}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_bwd_oracle.py tests/test_gpu_deferred_dy.py tests/test_gpu_attention.py \
  -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
for v in default ${VARIANTS}; do
  so=""
  [ "$v" != default ] && so=build/$v/_C.so
  for args in "1 1" "3 1" "1 2" "1 1 fwd"; do
    MSP_C_SO=$so timeout -k 10 120 python -u tools/dev/fused_bwd_bench.py 320 352 $args 2>&1 | { grep -v amdgpu.ids || true; } >> $out/bench.log
  done
done
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err
fi
