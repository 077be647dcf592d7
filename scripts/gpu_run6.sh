#!/bin/bash
# GPU tests (all) + bench bs16/bs32 + no-graph kernel profile.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu6.log 2>&1; rc=$?; echo "gpu tests exit $rc" >> gpurun_out/status6.txt
tail -5 gpurun_out/t_gpu6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b6_bs16.json 2>gpurun_out/b6_bs16.err || exit $?
cat gpurun_out/b6_bs16.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 32 > gpurun_out/b6_bs32.json 2>gpurun_out/b6_bs32.err || exit $?
cat gpurun_out/b6_bs32.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_v4 -o fused -- python $GRAFT_REPO_ROOT/bench.py --no-graph --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_v4.log 2>&1; echo "prof exit $?" >> $GRAFT_REPO_ROOT/gpurun_out/status6.txt
