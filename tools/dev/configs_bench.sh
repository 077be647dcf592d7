#!/bin/bash
# Dev: fused-engine benches of the other BASELINE configs (#3 smp-Unet R101, #4 DUCKNet-34 + R101 KD
# teacher, the student alone for the teacher's share) and a fully fused non-Unet decoder (FPN R101)
# -> gpurun_out/cfg_<tag>/
set -e
out=gpurun_out/cfg_${1:-cur}
mkdir -p $out
timeout -k 10 300 python -u bench.py --model smp-resnet101 --batch 64 --steps 10 --warmup 3 > $out/r101_b64.json 2> $out/r101_b64.err
timeout -k 10 300 python -u bench.py --base-channel 34 --teacher smp-resnet101 --batch 32 --steps 10 --warmup 3 > $out/kd_b32.json 2> $out/kd_b32.err
timeout -k 10 300 python -u bench.py --base-channel 34 --batch 32 --steps 10 --warmup 3 --val-images 0 > $out/ducknet34_b32.json 2> $out/ducknet34_b32.err
timeout -k 10 300 python -u bench.py --model smp-fpn-resnet101 --batch 64 --steps 10 --warmup 3 > $out/fpn_r101_b64.json 2> $out/fpn_r101_b64.err
