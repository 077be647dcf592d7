#!/bin/bash
# Dev (round 5): L2 hit/miss + latency per GEMM kernel over a conv_bench level -> gpurun_out/<tag>_{tcc,tcp}.txt
set -e
tag=${1:-tcc}
lv=${2:-4}
root="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
cd /tmp
k=0
for p in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"; do
  d="$root/gpurun_out/${tag}_$k"
  mkdir -p "$d"
  timeout -s KILL 150 rocprofv3 --pmc $p -d "$d" -o pmc -- python3 "$root/tools/conv_bench.py" --batch ${BATCH:-320} --iters 2 --levels $lv > "$d.log" 2>&1
  db=$(python3 -c "import glob,sys; f=sorted(glob.glob(sys.argv[1]+'/**/*results.db', recursive=True)); print(f[0] if f else '')" "$d")
  python3 "$root/tools/pmc_summary.py" "$db" --filter conv --top 60 > "$root/gpurun_out/${tag}_$k.txt" 2>&1
  python3 - "$db" > "$root/gpurun_out/${tag}_${k}_dispatch.txt" 2>&1 <<'PY'
import sqlite3, sys, collections
db = sqlite3.connect(sys.argv[1])
rows = db.execute('select dispatch_id, kernel_name, counter_name, value, duration from counters_collection').fetchall()
d = collections.defaultdict(dict)
for did, kn, cn, v, du in rows:
    d[did]['k'] = kn.split('(')[0][-60:]
    d[did]['dur'] = du
    d[did][cn] = d[did].get(cn, 0) + v
for did in sorted(d):
    r = d[did]
    print(did, r['k'], round(r['dur'] / 1e3, 1), ' '.join(f'{c}={v:.3g}' for c, v in r.items() if c not in ('k', 'dur')))
PY
  rm -rf "$d"
  k=$((k+1))
done
