#!/bin/bash
# Dev (round 5): halo PIPE A/B (MSP_HALO_PIPE 1 = MI 3 thin-halo only, 2 = every MI <= 3 tap set) on
# tools/conv_bench.py levels 1-2 and the bench -> gpurun_out/<tag>/
set -e -o pipefail
tag=${1:-pipeab}
out=gpurun_out/$tag
mkdir -p $out
for m in 1 2; do
  MSP_HALO_PIPE=$m timeout -k 10 300 python -u tools/conv_bench.py --batch 320 --iters 5 --levels ${LEVELS:-1,2} 2>/dev/null > $out/pipe$m.log
done
for m in 1 2; do
  MSP_HALO_PIPE=$m timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench_pipe$m.json 2> $out/bench_pipe$m.err
done
