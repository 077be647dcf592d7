#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -q -s > gpurun_out/t_gpu.log 2>&1; echo "tests exit $?" >> gpurun_out/status.txt
tail -12 gpurun_out/t_gpu.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b_fused_graph.json 2> gpurun_out/b_fused_graph.err; echo "bench graph exit $?" >> gpurun_out/status.txt
cat gpurun_out/b_fused_graph.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fused -o fused -- python $GRAFT_REPO_ROOT/bench.py --no-graph --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_fused.log 2>&1; echo "prof exit $?" >> $GRAFT_REPO_ROOT/gpurun_out/status.txt
cd $GRAFT_REPO_ROOT
cat gpurun_out/status.txt
