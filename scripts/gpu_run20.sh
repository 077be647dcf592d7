#!/bin/bash
# new loss kernels' numerics + PMC counters of the L2 3x3 / L1 fused8 conv kernels (fwd, dgrad, wgrad)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "mse or ohem or cross or phase or conv_fwd" > gpurun_out/t20_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t20_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_avail.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc20a -o pmc -- python3 tools/conv_bench.py --batch 64 --iters 3 --only "L2 3x3 34" > gpurun_out/pmc20a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc20b -o pmc -- python3 tools/conv_bench.py --batch 64 --iters 3 --only "L1 fused8" > gpurun_out/pmc20b.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d gpurun_out/pmc20c -o pmc -- python3 tools/conv_bench.py --batch 64 --iters 3 --only "L2 3x3 34" > gpurun_out/pmc20c.log 2>&1 || exit $?
ls gpurun_out/pmc20a gpurun_out/pmc20b gpurun_out/pmc20c
