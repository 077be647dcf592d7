# Dev: full GPU test tier + smoke + bench + kernel-trace profile, results under gpurun_out/<tag>/
# A test FAILURE (pytest rc 1) still lets the bench run; a time limit, abort or crash ends the script.
set -e
tag=${1:-cur}
mkdir -p gpurun_out/$tag
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$tag/gpu_tests.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping" >> gpurun_out/$tag/gpu_tests.log; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$tag/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
bash tools/dev/prof_bench.sh $tag
