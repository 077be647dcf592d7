set -e
for v in ko_amiss ko_bmiss; do
  MSP_C_SO=$GRAFT_REPO_ROOT/build/$v/_C.so bash tools/dev/pmc_gemm.sh pmcm_$v "L4 fused8"
done
