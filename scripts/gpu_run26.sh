#!/bin/bash
# NCB wgrad: numerics (halo/conv/model tests), per-layer wgrad NCB=1 vs default, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_distributed.py -x -v --timeout 150 --timeout-method thread > gpurun_out/t26_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t26_gpu.log
[ $rc -eq 0 ] || exit $rc
MSP_DW_NCB=1 timeout -k 10 200 python tools/conv_bench.py --batch 64 --iters 10 > gpurun_out/cb26_ncb1.log 2>&1 || exit $?
timeout -k 10 200 python tools/conv_bench.py --batch 64 --iters 10 > gpurun_out/cb26_ncb3.log 2>&1 || exit $?
grep -E "^L" gpurun_out/cb26_ncb1.log | awk '{print $1, $2, $3, "wgrad", $(NF-1), $NF}'
echo ---
grep -E "^L" gpurun_out/cb26_ncb3.log | awk '{print $1, $2, $3, "wgrad", $(NF-1), $NF}'
timeout -k 10 300 python bench.py > gpurun_out/b26_default.json 2>gpurun_out/b26_default.err || exit $?
cat gpurun_out/b26_default.json
timeout -k 10 300 python bench.py --batch 16 > gpurun_out/b26_bs16.json 2>gpurun_out/b26_bs16.err || exit $?
cat gpurun_out/b26_bs16.json
