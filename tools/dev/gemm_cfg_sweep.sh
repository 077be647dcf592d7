set -e
mkdir -p gpurun_out/r03_v3
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_gemm.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_v3/tests.log 2>&1
for c in 0 1 2 3 4; do
  MSP_CONV_GEMM_CFG=$c timeout -k 10 120 python -u tools/conv_bench.py --batch 128 --iters 10 --levels 3,4,5,6 > gpurun_out/r03_v3/cfg$c.log 2>&1
done
timeout -k 10 120 python -u tools/conv_bench.py --batch 128 --iters 10 --levels 3,4,5,6 > gpurun_out/r03_v3/planner.log 2>&1
