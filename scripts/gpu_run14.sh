#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof14 $R/gpurun_out/pmc14
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof14 -o fused -- python3 $R/bench.py --no-graph --steps 4 --warmup 2 > $R/gpurun_out/prof14/log.txt 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc14 -o sq -- python3 $R/tools/conv_bench.py --only "L1 3x3 17" --iters 3 > $R/gpurun_out/pmc14/sq.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc14 -o lds -- python3 $R/tools/conv_bench.py --only "L1 3x3 17" --iters 3 > $R/gpurun_out/pmc14/lds.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $R/gpurun_out/pmc14 -o fetch -- python3 $R/tools/conv_bench.py --only "L1 3x3 17" --iters 3 > $R/gpurun_out/pmc14/fetch.log 2>&1 || exit $?
echo done
