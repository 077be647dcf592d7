#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_distributed.py -q -s > gpurun_out/t12_dist.log 2>&1; echo "dist exit $?" >> gpurun_out/status12.txt
grep -E "replicated|worst|update rel|passed|failed" gpurun_out/t12_dist.log | cut -c1-1500
