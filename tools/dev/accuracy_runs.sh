#!/bin/bash
# Dev: accuracy through python main.py (tools/accuracy_main.py) at the bench batch (320) and at the
# reference's batch (16), fp32 EMA validation as the reference -> gpurun_out/acc/*.json
set -e
out=gpurun_out/acc
mkdir -p $out
timeout -k 10 780 python -u tools/accuracy_main.py --batch 320 --epochs 300 --val-every 10 --val-fp32 \
  --out $out/accuracy_main_ducknet17_bs320.json > $out/bs320.log 2>&1
timeout -k 10 400 python -u tools/accuracy_main.py --batch 16 --epochs 55 --val-every 5 --val-fp32 \
  --out $out/accuracy_main_ducknet17_bs16.json > $out/bs16.log 2>&1
