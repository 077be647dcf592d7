#!/bin/bash
# Dev: kernel-trace profile of a short bench run -> gpurun_out/prof_<tag>/ + prof_<tag>.txt summary
set -e
tag=${1:-cur}
shift || true
root="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p "$root/gpurun_out/prof_$tag"
cd "$root/${BENCH_DIR:-.}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/prof_$tag" -o run -- python3 bench.py --steps 5 --warmup 2 --val-images 0 "$@" > "$root/gpurun_out/prof_$tag.log" 2>&1
db=$(python3 -c "import glob,sys; f=sorted(glob.glob(sys.argv[1]+'/**/*results.db', recursive=True)); print(f[0] if f else '')" "$root/gpurun_out/prof_$tag")
cd "$root"
python3 tools/rocpd_summary.py "$db" --steps 5 --window --top 90 > "$root/gpurun_out/prof_$tag.txt" 2>&1
python3 tools/rocpd_summary.py "$db" --steps 5 --window --group >> "$root/gpurun_out/prof_$tag.txt" 2>&1
python3 tools/rocpd_timeline.py "$db" --steps 4 > "$root/gpurun_out/prof_${tag}_timeline.txt" 2>&1
python3 tools/rocpd_summary.py "$db" --sequence > "$root/gpurun_out/prof_${tag}_sequence.txt" 2>&1 || true
[ "${KEEP_DB:-0}" = 1 ] || rm -rf "$root/gpurun_out/prof_$tag"   # (raw DB: gpurun copies back at most 64 MiB)
