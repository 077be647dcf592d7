set -e
mkdir -p gpurun_out/r03_v4
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_v4/tests.log 2>&1
timeout -k 10 200 python -u tools/conv_bench.py --batch 128 --iters 10 > gpurun_out/r03_v4/bench_all.log 2>&1
timeout -k 10 200 python -u tools/conv_bench.py --batch 128 --iters 10 --prologue --levels 1,2 > gpurun_out/r03_v4/bench_pro.log 2>&1
