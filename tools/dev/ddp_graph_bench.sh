#!/bin/bash
# Dev (round 6): the multi-rank step on ONE GPU through the world-1 RCCL path (--ddp: process group, gradient
# bucketer, rebuilt buckets), hipGraph-captured vs not, at the reference's per-GPU batch 16 and at 64
# -> gpurun_out/ddp_graph/b<batch>_<on|off>.json (+ the single-process graph step for reference)
set -e
out=gpurun_out/ddp_graph
mkdir -p $out
port=29611
for b in ${BATCHES:-16 64}; do
  for g in on off; do
    port=$((port + 1))
    timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 1 --ddp --batch $b --graph-ddp $g --steps ${STEPS:-30} --warmup 5 \
      --comm-steps 0 > $out/b${b}_$g.json 2> $out/b${b}_$g.err
  done
  timeout -k 10 300 python -u bench.py --batch $b --steps ${STEPS:-30} --warmup 5 > $out/b${b}_single.json 2> $out/b${b}_single.err
done
