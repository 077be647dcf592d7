#!/bin/bash
# Dev (round 6): the bench's 25-step val Dice across trainer seeds on ONE tree (bs320, 20+5 steps, the same
# protocol as BENCH_r0N.json) -> gpurun_out/dice_spread/seed_<s>.json: how far summation-order-free
# run-to-run differences (a different init / data order) move that number.
set -e
mkdir -p gpurun_out/dice_spread
for sd in ${SEEDS:-1 2 3 4}; do
  timeout -k 10 400 python -u bench.py --seed $sd > gpurun_out/dice_spread/seed_$sd.json 2> gpurun_out/dice_spread/seed_$sd.err
done
