#!/bin/bash
# GPU round-1 check: kernel numerics, fused-vs-eager model parity, fused bench (no graph / graph), profile.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/t_kernels.log 2>&1; echo "kernels exit $?" >> gpurun_out/status.txt
tail -5 gpurun_out/t_kernels.log
timeout -k 10 400 python -m pytest tests/test_gpu_models.py -x -q > gpurun_out/t_models.log 2>&1; echo "models exit $?" >> gpurun_out/status.txt
tail -5 gpurun_out/t_models.log
timeout -k 10 300 python bench.py --no-graph --steps 10 --warmup 3 > gpurun_out/b_fused_nograph.json 2> gpurun_out/b_fused_nograph.err; echo "bench nograph exit $?" >> gpurun_out/status.txt
cat gpurun_out/b_fused_nograph.json; tail -3 gpurun_out/b_fused_nograph.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b_fused_graph.json 2> gpurun_out/b_fused_graph.err; echo "bench graph exit $?" >> gpurun_out/status.txt
cat gpurun_out/b_fused_graph.json; tail -3 gpurun_out/b_fused_graph.err
cat gpurun_out/status.txt
