#!/bin/bash
# Dev (round 5): PMC passes over tools/dev/fused_bwd_bench.py (L1 fused backward at bs320; "fwd" = the
# forward mode) -> gpurun_out/<tag>/pmc_<k>.txt (tools/pmc_summary.py over each pass's rocpd DB)
set -e
tag=${1:-pmcfb}
mode=${2:-}
root="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p "$root/gpurun_out/$tag"
cd /tmp
passes=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
        "FETCH_SIZE GRBM_GUI_ACTIVE"
        "WRITE_SIZE GRBM_GUI_ACTIVE")
k=0
for p in "${passes[@]}"; do
  d="$root/gpurun_out/$tag/p$k"
  mkdir -p "$d"
  timeout -s KILL 120 rocprofv3 --pmc $p -d "$d" -o pmc -- python3 "$root/tools/dev/fused_bwd_bench.py" 320 352 1 1 $mode > "$d.log" 2>&1
  db=$(python3 -c "import glob,sys; f=sorted(glob.glob(sys.argv[1]+'/**/*results.db', recursive=True)); print(f[0] if f else '')" "$d")
  python3 "$root/tools/pmc_summary.py" "$db" --filter conv > "$root/gpurun_out/$tag/pmc_$k.txt" 2>&1
  rm -rf "$d"   # (the raw DB: gpurun copies back at most 64 MiB)
  k=$((k+1))
done
