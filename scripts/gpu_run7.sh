#!/bin/bash
# halo conv kernel: numerics, distributed test, per-layer A/B bench, then model bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/t7_kernels.log 2>&1; rc=$?; echo "kernel tests exit $rc" >> gpurun_out/status7.txt
tail -4 gpurun_out/t7_kernels.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m pytest tests/test_gpu_distributed.py -x -q -s > gpurun_out/t7_dist.log 2>&1; echo "dist exit $?" >> gpurun_out/status7.txt
grep -E "rel diff|passed|failed" gpurun_out/t7_dist.log
timeout -k 10 300 python tools/conv_bench.py --halo 1 > gpurun_out/cb7_halo.log 2>&1 || exit $?
timeout -k 10 300 python tools/conv_bench.py --halo 0 > gpurun_out/cb7_gather.log 2>&1 || exit $?
grep -v "^{" gpurun_out/cb7_halo.log | cut -c1-80
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t7_gpu.log 2>&1; echo "all gpu tests exit $?" >> gpurun_out/status7.txt
tail -3 gpurun_out/t7_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b7_bs16.json 2>gpurun_out/b7_bs16.err || exit $?
cat gpurun_out/b7_bs16.json
MSP_CONV_HALO=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b7_bs16_gather.json 2>gpurun_out/b7_bs16_gather.err || exit $?
cat gpurun_out/b7_bs16_gather.json
