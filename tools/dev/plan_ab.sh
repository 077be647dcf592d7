#!/bin/bash
# Dev (round 5): planner A/B on tools/conv_bench.py levels 3-6 at the bench batch: forward GEMM configs
# 9 / 10 (8-wave, 3-stage) forced vs the planner, and the wgrad planner's staging cost 24 / 48 / 96
# (MSP_WGRAD_STAGE_COST) -> gpurun_out/<tag>/
set -e -o pipefail
tag=${1:-planab}
B=${BATCH:-320}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_gemm.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u tools/conv_bench.py --batch $B --iters 5 --levels ${LEVELS:-3,4,5,6} 2>/dev/null > $out/$n.log
}
run plan
run fwd9 MSP_CONV_GEMM_CFG=9
run fwd10 MSP_CONV_GEMM_CFG=10
run wg48 MSP_WGRAD_STAGE_COST=48
run wg96 MSP_WGRAD_STAGE_COST=96
