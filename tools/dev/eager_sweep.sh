#!/bin/bash
# Dev: eager (stock PyTorch-ROCm) reference-speed sweep -> gpurun_out/eager/*.json
#   DUCKNet-17 channels-last at bs 32/64/128/256 (the denominator of bench.py's vs_baseline), then the
#   eager baselines of BASELINE configs #3 (smp-Unet R101) and #4 (DUCKNet-34 + R101 KD).
# Each run has its own time limit; the script stops at the first failure (no GPU step after a fault).
set -e
out=gpurun_out/eager
mkdir -p $out
for b in 32 64 128 256; do
  timeout -k 10 420 python -u bench.py --impl eager --channels-last --batch $b --steps 10 --warmup 3 --val-images 0 \
    > $out/ducknet17_cl_bs$b.json 2> $out/ducknet17_cl_bs$b.err
done
timeout -k 10 420 python -u bench.py --impl eager --channels-last --model smp-resnet101 --batch 64 --steps 10 --warmup 3 \
  --val-images 0 > $out/r101_cl_bs64.json 2> $out/r101_cl_bs64.err
timeout -k 10 420 python -u bench.py --impl eager --channels-last --base-channel 34 --teacher smp-resnet101 --batch 32 \
  --steps 10 --warmup 3 --val-images 0 > $out/kd_cl_bs32.json 2> $out/kd_cl_bs32.err
