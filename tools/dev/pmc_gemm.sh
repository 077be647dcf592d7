#!/bin/bash
# Dev (round 5): PMC passes over one conv_bench layer (default "L4 fused8" at bs320: the fwd / dgrad GEMM and
# the wgrad GEMM kernels) -> gpurun_out/<tag>_<k>.txt.  One rocprofv3 run per pass (hardware counter limits).
set -e
tag=${1:-pmcg}
only=${2:-L4 fused8}
root="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
cd /tmp
passes=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
        "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE"
        "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
        "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE")
k=0
for p in "${passes[@]}"; do
  d="$root/gpurun_out/${tag}_$k"
  mkdir -p "$d"
  timeout -s KILL 150 rocprofv3 --pmc $p -d "$d" -o pmc -- python3 "$root/tools/conv_bench.py" --batch ${BATCH:-320} --iters 3 --only "$only" > "$d.log" 2>&1
  db=$(python3 -c "import glob,sys; f=sorted(glob.glob(sys.argv[1]+'/**/*results.db', recursive=True)); print(f[0] if f else '')" "$d")
  python3 "$root/tools/pmc_summary.py" "$db" --filter conv > "$root/gpurun_out/${tag}_$k.txt" 2>&1
  rm -rf "$d"
  k=$((k+1))
done
