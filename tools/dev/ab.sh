#!/bin/bash
# Dev: A/B arms of one command in ONE gpurun call (interleaved rounds, one device: cdna guide §5.4 rule 24).
#   usage: tools/dev/ab.sh <tag> <rounds> '<command>' 'ARM_A_ENV' 'ARM_B_ENV' ...
#   e.g.   tools/dev/ab.sh hg 2 'python -u tools/conv_bench.py --batch 320 --levels 3,4 --hgemm $HG' 'HG=1' 'HG=0'
# Each arm runs `env <arm env> bash -c <command>` (the env is applied before anything touches the GPU) with a
# 300-s limit; output -> gpurun_out/<tag>/r<round>_a<arm>.log.  Stops at the first failing run.
set -e
tag=$1; rounds=$2; cmd=$3; shift 3
out="${GRAFT_REPO_ROOT:-.}/gpurun_out/$tag"
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  a=0
  for arm in "$@"; do
    echo "== round $r arm $a: $arm" >> "$out/index.txt"
    env $arm timeout -k 10 300 bash -c "$cmd" > "$out/r${r}_a${a}.log" 2>&1
    a=$((a + 1))
  done
done
