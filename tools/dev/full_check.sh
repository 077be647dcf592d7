# Dev: full GPU test tier + bench + kernel-trace profile, results under gpurun_out/<tag>/
set -e
tag=${1:-cur}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$tag/gpu_tests.log 2>&1 || echo "tests failed" >> gpurun_out/$tag/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
bash tools/dev/prof_bench.sh $tag
