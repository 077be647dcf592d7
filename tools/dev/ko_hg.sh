set -e
mkdir -p gpurun_out/ko
for v in default ko_dma ko_mfma; do
  so=""
  [ "$v" != default ] && so="build/$v/_C.so"
  for hg in 1 0; do
    MSP_C_SO=$so timeout -k 10 200 python -u tools/conv_bench.py --batch 320 --iters 5 --levels 3,4,5,6 --hgemm $hg 2>/dev/null > gpurun_out/ko/${v}_hg$hg.log
  done
done
