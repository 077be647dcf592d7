#!/bin/bash
# SyncBN param-grad fix (dist test) + PMC counters of the L1 3x3 conv kernels (fwd/dgrad/wgrad)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc10
timeout -k 10 300 python -m pytest tests/test_gpu_distributed.py -x -q -s > gpurun_out/t10_dist.log 2>&1; echo "dist exit $?" >> gpurun_out/status10.txt
grep -E "rel diff|passed|failed" gpurun_out/t10_dist.log | cut -c1-300
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc10 -o sq -- python3 $R/tools/conv_bench.py --only "L1 3x3 17" --iters 3 > $R/gpurun_out/pmc10/sq.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $R/gpurun_out/pmc10 -o fetch -- python3 $R/tools/conv_bench.py --only "L1 3x3 17" --iters 3 > $R/gpurun_out/pmc10/fetch.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_EA0_ATOMIC_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmc10 -o write -- python3 $R/tools/conv_bench.py --only "L1 3x3 17" --iters 3 > $R/gpurun_out/pmc10/write.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc10 -o lds -- python3 $R/tools/conv_bench.py --only "L1 3x3 17" --iters 3 > $R/gpurun_out/pmc10/lds.log 2>&1 || exit $?
ls -R $R/gpurun_out/pmc10 | head -30
