#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/t16_kernels.log 2>&1; rc=$?
tail -2 gpurun_out/t16_kernels.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_bench.py --halo 1 > gpurun_out/cb16.log 2>&1 || exit $?
grep -v "^{" gpurun_out/cb16.log | cut -c1-120
for b in 16 32 64 128; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/b16_bs$b.json 2>gpurun_out/b16_bs$b.err || exit $?
  cat gpurun_out/b16_bs$b.json
done
