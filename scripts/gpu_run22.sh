#!/bin/bash
# re-entry validation: full GPU test tier + default bench + bs128 bench + kernel-trace stats (bs16)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t22_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t22_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/b22_default.json 2>gpurun_out/b22_default.err || exit $?
cat gpurun_out/b22_default.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 128 > gpurun_out/b22_bs128.json 2>gpurun_out/b22_bs128.err || exit $?
cat gpurun_out/b22_bs128.json
timeout -k 10 300 python bench.py --impl eager --channels-last --steps 10 --warmup 3 > gpurun_out/b22_eager.json 2>gpurun_out/b22_eager.err || exit $?
cat gpurun_out/b22_eager.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof22 -o prof -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof22.log 2>&1 || exit $?
find gpurun_out/prof22 -name "*stats*"
