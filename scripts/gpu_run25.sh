#!/bin/bash
# full GPU tier + default bench (bs128) + bs16 + kernel profile (bs128) + eager reference at bs128
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 150 --timeout-method thread > gpurun_out/t25_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t25_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/b25_default.json 2>gpurun_out/b25_default.err || exit $?
cat gpurun_out/b25_default.json
timeout -k 10 300 python bench.py --batch 16 > gpurun_out/b25_bs16.json 2>gpurun_out/b25_bs16.err || exit $?
cat gpurun_out/b25_bs16.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof25 -o prof -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof25.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --impl eager --channels-last --steps 5 --warmup 2 > gpurun_out/b25_eager_bs128.json 2>gpurun_out/b25_eager_bs128.err || exit $?
cat gpurun_out/b25_eager_bs128.json
