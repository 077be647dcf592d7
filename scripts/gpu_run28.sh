#!/bin/bash
# per-GPU batch sweep beyond 128 (HBM sizing)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 192 256; do
  timeout -k 10 300 python bench.py --batch $b --steps 10 --warmup 3 > gpurun_out/b28_bs$b.json 2>gpurun_out/b28_bs$b.err || exit $?
  cat gpurun_out/b28_bs$b.json
done
