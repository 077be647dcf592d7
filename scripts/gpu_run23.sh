#!/bin/bash
# new pool/up2cat/add_act kernels, 7x7 stem conv, smp ResNet-UNet fused executor; smp + KD benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -v --timeout 120 --timeout-method thread -k "maxpool or up2_cat or conv_fwd_bwd or matches_eager" > gpurun_out/t23_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/t23_gpu.log
[ $rc -eq 0 ] || exit $rc
grep -E "cos" gpurun_out/t23_gpu.log | head -20
timeout -k 10 300 python bench.py --model smp-resnet101 --batch 64 --steps 10 --warmup 3 > gpurun_out/b23_r101.json 2>gpurun_out/b23_r101.err || exit $?
cat gpurun_out/b23_r101.json
timeout -k 10 300 python bench.py --model smp-resnet101 --batch 64 --steps 10 --warmup 3 --impl eager --channels-last > gpurun_out/b23_r101_eager.json 2>gpurun_out/b23_r101_eager.err || exit $?
cat gpurun_out/b23_r101_eager.json
timeout -k 10 300 python bench.py --base-channel 34 --teacher smp-resnet101 --batch 32 --steps 10 --warmup 3 > gpurun_out/b23_kd.json 2>gpurun_out/b23_kd.err || exit $?
cat gpurun_out/b23_kd.json
timeout -k 10 300 python bench.py --base-channel 34 --teacher smp-resnet101 --batch 32 --steps 10 --warmup 3 --impl eager --channels-last > gpurun_out/b23_kd_eager.json 2>gpurun_out/b23_kd_eager.err || exit $?
cat gpurun_out/b23_kd_eager.json
