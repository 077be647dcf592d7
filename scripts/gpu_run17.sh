#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t17_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t17_gpu.log
[ $rc -eq 0 ] || exit $rc
for b in 16 128; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/b17_bs$b.json 2>gpurun_out/b17_bs$b.err || exit $?
  cat gpurun_out/b17_bs$b.json
done
