#!/bin/bash
# First GPU probe: eager reference-speed baseline + rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python bench.py --impl eager --steps 10 --warmup 3 --batch 16 > gpurun_out/eager_nchw_b16.json 2> gpurun_out/eager_nchw_b16.err && \
timeout -k 10 300 python bench.py --impl eager --channels-last --steps 10 --warmup 3 --batch 16 > gpurun_out/eager_cl_b16.json 2> gpurun_out/eager_cl_b16.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_eager -o eager -- python bench.py --impl eager --steps 3 --warmup 2 --batch 16 > gpurun_out/prof_eager.log 2>&1
echo "exit $?"
cat gpurun_out/*.json
