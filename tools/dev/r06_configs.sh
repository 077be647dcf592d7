#!/bin/bash
# Dev (round 6): end-of-round evidence on one box -- smoke(), the default bench, its kernel profile and every
# non-headline BASELINE config -> gpurun_out/r06final/
set -e
out=gpurun_out/r06final
mkdir -p $out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err
bash tools/dev/prof_bench.sh r06final
bash tools/dev/configs_bench.sh r06final
for m in smp-resnext50_32x4d smp-mobilenet_v2 smp-deeplabv3plus-resnet101; do
  timeout -k 10 300 python -u bench.py --model $m --batch 64 --steps 10 --warmup 3 > gpurun_out/cfg_r06final/$m.json 2> gpurun_out/cfg_r06final/$m.err
done
