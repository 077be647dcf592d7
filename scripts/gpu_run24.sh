#!/bin/bash
# GPU augmentation numerics, trainer (now on the device loader), KD + smp eager reference benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_augment.py tests/test_gpu_trainer.py -x -v -s --timeout 150 --timeout-method thread > gpurun_out/t24_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/t24_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --base-channel 34 --teacher smp-resnet101 --batch 32 --steps 10 --warmup 3 > gpurun_out/b24_kd.json 2>gpurun_out/b24_kd.err || exit $?
cat gpurun_out/b24_kd.json
timeout -k 10 400 python bench.py --model smp-resnet101 --batch 64 --steps 10 --warmup 3 --impl eager --channels-last > gpurun_out/b24_r101_eager.json 2>gpurun_out/b24_r101_eager.err || exit $?
cat gpurun_out/b24_r101_eager.json
timeout -k 10 400 python bench.py --base-channel 34 --teacher smp-resnet101 --batch 32 --steps 10 --warmup 3 --impl eager --channels-last > gpurun_out/b24_kd_eager.json 2>gpurun_out/b24_kd_eager.err || exit $?
cat gpurun_out/b24_kd_eager.json
