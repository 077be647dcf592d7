#!/bin/bash
# Dev: PMC passes over one program, one rocprofv3 run per pass (hardware counter limits, see README
# "Profiling") -> gpurun_out/<tag>_<k>.txt via tools/pmc_summary.py.
#   usage: tools/dev/pmc.sh <tag> <kernel-name filter> <program> [args...]
#   e.g.   tools/dev/pmc.sh pmc_l4 conv python3 tools/conv_bench.py --batch 320 --iters 3 --only "L4 fused8"
# PASSES (env, optional): '|'-separated counter lists replacing the default four passes.
set -e
tag=$1; filt=$2; shift 2
root="${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
def="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE|TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE|TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
IFS='|' read -r -a passes <<< "${PASSES:-$def}"
cd /tmp
k=0
for p in "${passes[@]}"; do
  d="$root/gpurun_out/${tag}_$k"
  mkdir -p "$d"
  timeout -s KILL 150 rocprofv3 --pmc $p -d "$d" -o pmc -- "$@" > "$d.log" 2>&1
  db=$(python3 -c "import glob,sys; f=sorted(glob.glob(sys.argv[1]+'/**/*results.db', recursive=True)); print(f[0] if f else '')" "$d")
  python3 "$root/tools/pmc_summary.py" "$db" --filter "$filt" > "$root/gpurun_out/${tag}_$k.txt" 2>&1
  rm -rf "$d"
  k=$((k + 1))
done
