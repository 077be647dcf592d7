#!/bin/bash
# GPU tests + bench sweep + kernel-trace profile of the fused step (bs 64).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t18_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t18_gpu.log
[ $rc -eq 0 ] || exit $rc
for b in 16 64 128 256; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/b18_bs$b.json 2>gpurun_out/b18_bs$b.err || exit $?
  cat gpurun_out/b18_bs$b.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof18 -o prof -- python3 bench.py --steps 5 --warmup 2 --batch 64 > gpurun_out/prof18.log 2>&1 || exit $?
ls -R gpurun_out/prof18 | head -20
