#!/bin/bash
# Dev (round 6): phased strided data-gradient on the GEMM kernel -- oracle tests, the 3x3 s2 layers, the
# default bench (seed 1, twice) and the round-5 tree's bench on the same box (seed 1) -> gpurun_out/r06pc/
set -e
out=gpurun_out/r06pc
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_gemm.py > $out/tests_gemm.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py > $out/tests_kernels.log 2>&1
timeout -k 10 200 python -u tools/conv_bench.py --batch 320 --iters 5 --only 3x3s2 2>/dev/null > $out/cb_s2.log
timeout -k 10 400 python -u bench.py --seed 1 > $out/bench_seed1_a.json 2> $out/bench_seed1_a.err
timeout -k 10 400 python -u bench.py --seed 1 > $out/bench_seed1_b.json 2> $out/bench_seed1_b.err
cd _bisect/r05
timeout -k 10 400 python -u bench.py > ../../$out/bench_r05tree.json 2> ../../$out/bench_r05tree.err
