#!/bin/bash
# kernel numerics + bench bs128 + kernel-trace profile (bs64) + per-layer conv bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t19_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t19_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 128 > gpurun_out/b19_bs128.json 2>gpurun_out/b19_bs128.err || exit $?
cat gpurun_out/b19_bs128.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof19 -o prof -- python3 bench.py --steps 5 --warmup 2 --batch 64 > gpurun_out/prof19.log 2>&1 || exit $?
timeout -k 10 300 python tools/conv_bench.py --batch 64 > gpurun_out/cb19.log 2>&1 || exit $?
tail -30 gpurun_out/cb19.log | cut -c1-140
