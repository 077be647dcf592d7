#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q > gpurun_out/t_kernels.log 2>&1; echo "kernels exit $?" >> gpurun_out/status.txt
tail -3 gpurun_out/t_kernels.log
timeout -k 10 400 python -m pytest tests/test_gpu_models.py -q > gpurun_out/t_models.log 2>&1; echo "models exit $?" >> gpurun_out/status.txt
tail -8 gpurun_out/t_models.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fused -o fused -- python $GRAFT_REPO_ROOT/bench.py --no-graph --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_fused.log 2>&1; echo "prof exit $?" >> $GRAFT_REPO_ROOT/gpurun_out/status.txt
cd $GRAFT_REPO_ROOT
cat gpurun_out/status.txt
