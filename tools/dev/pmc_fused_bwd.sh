#!/bin/bash
# Dev: PMC passes over tools/dev/fused_bwd_bench.py (the L1 fused backward launch) -> gpurun_out/pmc_fb_<k>.txt
set -e
root="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
cd /tmp
passes=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE"
        "FETCH_SIZE GRBM_GUI_ACTIVE"
        "WRITE_SIZE GRBM_GUI_ACTIVE")
k=0
for p in "${passes[@]}"; do
  d="$root/gpurun_out/pmc_fb_$k"
  mkdir -p "$d"
  timeout -s KILL 120 rocprofv3 --pmc $p -d "$d" -o pmc -- python3 "$root/tools/dev/fused_bwd_bench.py" 320 352 > "$d.log" 2>&1
  db=$(python3 -c "import glob,sys; f=sorted(glob.glob(sys.argv[1]+'/**/*results.db', recursive=True)); print(f[0] if f else '')" "$d")
  python3 "$root/tools/pmc_summary.py" "$db" --filter conv > "$root/gpurun_out/pmc_fb_$k.txt" 2>&1
  k=$((k+1))
done
