#!/bin/bash
# Dev: eager (stock PyTorch-ROCm, channels-last, MIOpen) speeds of BASELINE configs #3 and #4 -> the
# vs_baseline denominators of those configs.  Each run has its own limit; stops at the first failure.
set -e
out=gpurun_out/eager
mkdir -p $out
timeout -k 10 540 python -u bench.py --impl eager --channels-last --model smp-resnet101 --batch 64 --steps 10 --warmup 3 \
  --val-images 0 > $out/r101_cl_bs64.json 2> $out/r101_cl_bs64.err
timeout -k 10 540 python -u bench.py --impl eager --channels-last --base-channel 34 --teacher smp-resnet101 --batch 32 \
  --steps 10 --warmup 3 --val-images 0 > $out/kd_cl_bs32.json 2> $out/kd_cl_bs32.err
