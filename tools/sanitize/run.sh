#!/bin/bash
# Host-side sanitizer build of the launch planners (csrc/conv.hip host code) + the self-check driver.
# GPU AddressSanitizer / xnack builds are not available on this pool, so the sanitizers instrument the
# host code only (each -fsanitize= right after -Xarch_host); the device code is compiled too (the fat
# binary must link) but nothing is launched -- the check runs on a CPU-only machine.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
root="$(cd "$here/../.." && pwd)"
out="${1:-/tmp/msp_plan_check}"
hipcc=${HIPCC:-/opt/rocm/bin/hipcc}
"$hipcc" -O1 -g -std=c++17 --offload-arch=gfx950 \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
  -fno-omit-frame-pointer -I"$root/csrc" "$root/csrc/conv.hip" "$root/csrc/conv_gemm.hip" "$root/csrc/conv_wgrad_gemm.hip" "$root/csrc/conv_bwd.hip" "$here/plan_check.cpp" -o "$out"
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$out"
