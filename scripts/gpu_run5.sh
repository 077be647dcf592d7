#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_distributed.py -x -q > gpurun_out/t_dist.log 2>&1; echo "dist test exit $?" >> gpurun_out/status.txt
tail -15 gpurun_out/t_dist.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_v3 -o fused -- python $GRAFT_REPO_ROOT/bench.py --no-graph --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_v3.log 2>&1; echo "prof exit $?" >> $GRAFT_REPO_ROOT/gpurun_out/status.txt
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 32 > gpurun_out/b_bs32.json 2>gpurun_out/b_bs32.err; echo "bench32 exit $?" >> gpurun_out/status.txt
cat gpurun_out/b_bs32.json
cat gpurun_out/status.txt
