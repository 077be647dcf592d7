// Dev probe: which XCD (HW_REG_XCC_ID) runs each block of a plain launch -- checks the round-robin block ->
// XCD assumption behind the GEMM kernels' remap (csrc/conv_gemm.hip).  Read-only register, one store per block.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(int* out, int spin) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) out[blockIdx.x] = (int)(x & 0xf);
  // keep the block resident a little so later blocks cannot reuse its slot immediately
  long long t0 = wall_clock64();
  while (wall_clock64() - t0 < spin) {}
}

int main() {
  for (int nb : {64, 4096, 33880}) {
    int* d;
    hipMalloc(&d, nb * sizeof(int));
    hipLaunchKernelGGL(probe, dim3(nb), dim3(256), 0, 0, d, 2000);
    hipDeviceSynchronize();
    std::vector<int> h(nb);
    hipMemcpy(h.data(), d, nb * sizeof(int), hipMemcpyDeviceToHost);
    int match = 0;
    for (int b = 0; b < nb; ++b) match += h[b] == (h[b % 8]);
    printf("blocks=%d: first 24 xcc:", nb);
    for (int b = 0; b < 24 && b < nb; ++b) printf(" %d", h[b]);
    printf("  | fraction with xcc(b) == xcc(b %% 8): %.4f\n", (double)match / nb);
    hipFree(d);
  }
  return 0;
}
