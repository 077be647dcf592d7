#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 16 32 64 128; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/b15_bs$b.json 2>gpurun_out/b15_bs$b.err || exit $?
  cat gpurun_out/b15_bs$b.json
done
