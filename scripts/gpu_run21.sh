#!/bin/bash
# wgrad grid-size sweep (blocks per CU) on the per-layer conv bench, bs64
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for sp in 256 512 768 1024; do
  MSP_DW_SPLIT=$sp timeout -k 10 200 python tools/conv_bench.py --batch 64 --iters 10 > gpurun_out/cb21_sp$sp.log 2>&1 || exit $?
  echo "split $sp"; grep -E "^L" gpurun_out/cb21_sp$sp.log | awk '{print $1, $2, $3, "wgrad", $(NF-1), $NF}'
done
