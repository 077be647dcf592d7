#!/bin/bash
# Dev: rocprofv3 kernel table of a conv_bench subset -> gpurun_out/cbprof_<tag>/kernels.txt (raw DB deleted)
set -e
tag=$1; shift
root="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out="$root/gpurun_out/cbprof_$tag"
mkdir -p "$out"
cd "$root"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/raw" -o run -- python3 tools/conv_bench.py "$@" > "$out/bench.log" 2>&1
db=$(python3 -c "import glob,sys; f=sorted(glob.glob(sys.argv[1]+'/**/*results.db', recursive=True)); print(f[0] if f else '')" "$out/raw")
python3 tools/rocpd_summary.py "$db" > "$out/kernels.txt" 2>&1
rm -rf "$out/raw"
