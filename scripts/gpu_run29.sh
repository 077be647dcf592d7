#!/bin/bash
# BN-partials-in-dgrad-epilogue: full GPU tier, then bench (bs128, bs16)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 150 --timeout-method thread > gpurun_out/t29_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t29_gpu.log
[ $rc -eq 0 ] || exit $rc
grep -E "grad cos|logits cos" gpurun_out/t29_gpu.log | head -12
timeout -k 10 300 python bench.py > gpurun_out/b29_default.json 2>gpurun_out/b29_default.err || exit $?
cat gpurun_out/b29_default.json
timeout -k 10 300 python bench.py --batch 16 > gpurun_out/b29_bs16.json 2>gpurun_out/b29_bs16.err || exit $?
cat gpurun_out/b29_bs16.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof29 -o prof -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof29.log 2>&1 || exit $?
