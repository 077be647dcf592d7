set -e
out=gpurun_out/cfg
mkdir -p $out
timeout -k 10 300 python -u bench.py --base-channel 34 --teacher smp-resnet101 --batch 32 --steps 10 --warmup 3 > $out/kd_b32.json 2> $out/kd_b32.err
timeout -k 10 300 python -u bench.py --base-channel 34 --batch 32 --steps 10 --warmup 3 --val-images 0 > $out/ducknet34_b32.json 2> $out/ducknet34_b32.err
timeout -k 10 300 python -u bench.py --model smp-fpn-resnet101 --batch 64 --steps 10 --warmup 3 > $out/fpn_r101_b64.json 2> $out/fpn_r101_b64.err
timeout -k 10 300 python -u bench.py --model smp-resnet101 --batch 256 --steps 10 --warmup 3 > $out/r101_b256.json 2> $out/r101_b256.err
bash tools/dev/prof_bench.sh v8
