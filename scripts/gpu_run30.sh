#!/bin/bash
# NaN hunt: trainer test with and without the BN dgrad epilogue; model-level grads; A/B bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MSP_BN_EPILOGUE=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -v -s --timeout 150 --timeout-method thread -k "fused-False" > gpurun_out/t30_off.log 2>&1; echo "off rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -v -s --timeout 150 --timeout-method thread -k "fused-False" > gpurun_out/t30_on.log 2>&1; echo "on rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -s --timeout 150 --timeout-method thread -k "epilogue" > gpurun_out/t30_ep.log 2>&1; echo "ep rc=$?"
tail -2 gpurun_out/t30_off.log gpurun_out/t30_on.log gpurun_out/t30_ep.log
MSP_BN_EPILOGUE=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b30_off.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b30_on.json 2>/dev/null || exit $?
cut -c1-150 gpurun_out/b30_off.json gpurun_out/b30_on.json
