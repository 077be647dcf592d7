// Host-only driver of the conv launch-planner self-check, built with AddressSanitizer + UBSan on the
// host side (tools/sanitize/run.sh).  Runs on a CPU-only machine: nothing is launched on a GPU.
#include <cstdio>

int conv_plan_selfcheck(int verbose);

int main() {
  const int bad = conv_plan_selfcheck(1);
  std::printf("%s\n", bad == 0 ? "PLAN_CHECK_OK" : "PLAN_CHECK_FAILED");
  return bad == 0 ? 0 : 1;
}
