#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/t_gpu_all.log 2>&1; echo "gpu tests exit $?" >> gpurun_out/status.txt
tail -5 gpurun_out/t_gpu_all.log
timeout -k 10 600 python tools/conv_bench.py --miopen --iters 10 > gpurun_out/conv_bench.log 2>&1; echo "conv_bench exit $?" >> gpurun_out/status.txt
head -30 gpurun_out/conv_bench.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b_fused_graph.json 2> gpurun_out/b_fused_graph.err; echo "bench exit $?" >> gpurun_out/status.txt
cat gpurun_out/b_fused_graph.json
cat gpurun_out/status.txt
