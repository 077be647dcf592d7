#!/bin/bash
# Dev: chunked halo dgrad knock-outs (weight loads / staging / MFMAs) + halo wgrad grid-size A/B
set -e
out=gpurun_out/e5
mkdir -p $out
DBGS="0 32 8 4 40" bash tools/dev/halo_ko.sh chunk_l1 "L1 fused8"
DBGS="0 32 8 4 40" bash tools/dev/halo_ko.sh chunk_l1in "L1in fused8"
for sp in 256 512 1024; do
  echo "MSP_DW_SPLIT=$sp" >> $out/dw_split.log
  MSP_DW_SPLIT=$sp timeout -k 10 150 python -u tools/conv_bench.py --batch 128 --iters 10 --levels 1,2 2>/dev/null | grep -v '^{' >> $out/dw_split.log
done
