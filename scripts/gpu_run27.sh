#!/bin/bash
# PMC passes on the fused8 convs (MFMA busy, LDS conflicts, HBM bytes), no-graph bench (host overhead of
# the DDP path), kernel-trace profile of the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in "L1 fused8" "L3 fused8"; do
  tag=$(echo $L | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/pmc27_$tag -o pmc -- python3 tools/conv_bench.py --batch 64 --iters 3 --only "$L" > gpurun_out/pmc27_$tag.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc27b_$tag -o pmc -- python3 tools/conv_bench.py --batch 64 --iters 3 --only "$L" > gpurun_out/pmc27b_$tag.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc27c_$tag -o pmc -- python3 tools/conv_bench.py --batch 64 --iters 3 --only "$L" > gpurun_out/pmc27c_$tag.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --no-graph > gpurun_out/b27_nograph.json 2>gpurun_out/b27_nograph.err || exit $?
cat gpurun_out/b27_nograph.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof27 -o prof -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof27.log 2>&1 || exit $?
ls gpurun_out/prof27
