#!/bin/bash
# Dev (round 5): fused narrow-conv backward staging A/B -- the kernel's numerics tests, then
# tools/dev/fused_bwd_bench.py at the bench shape (dilation 1 / 3, Go = 1) for the default build and each
# variant in $VARIANTS (build/<name>/_C.so, csrc/build.py MSP_BUILD_VARIANT) -> gpurun_out/<tag>/
set -e -o pipefail
tag=${1:-fbab}
out=gpurun_out/$tag
mkdir -p $out
[ "${TESTS:-1}" = 1 ] && timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_bwd_oracle.py tests/test_gpu_deferred_dy.py -x -q \
  --timeout 200 --timeout-method thread > $out/tests.log 2>&1
for v in default ${VARIANTS}; do
  so=""
  [ "$v" != default ] && so=build/$v/_C.so
  for dg in "1 1" "3 1" "1 2"; do
    MSP_C_SO=$so timeout -k 10 120 python -u tools/dev/fused_bwd_bench.py 320 352 $dg 2>&1 | { grep -v amdgpu.ids || true; } >> $out/bench.log
  done
done
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err
fi
