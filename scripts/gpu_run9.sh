#!/bin/bash
# chunked halo conv + fewer wgrad splits: numerics + per-layer bench + model bench + dist test
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/t9_kernels.log 2>&1; rc=$?; echo "kernel tests exit $rc" >> gpurun_out/status9.txt
tail -2 gpurun_out/t9_kernels.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_bench.py --halo 1 > gpurun_out/cb9_halo.log 2>&1 || exit $?
grep -v "^{" gpurun_out/cb9_halo.log | cut -c1-120
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b9_bs16.json 2>gpurun_out/b9_bs16.err || exit $?
cat gpurun_out/b9_bs16.json
timeout -k 10 300 python -m pytest tests/test_gpu_distributed.py -x -q -s > gpurun_out/t9_dist.log 2>&1; echo "dist exit $?" >> gpurun_out/status9.txt
grep -E "rel diff|passed|failed" gpurun_out/t9_dist.log | cut -c1-400
