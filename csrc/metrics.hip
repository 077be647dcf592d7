// Argmax -> confusion-matrix histogram (reference: torchmetrics Dice/JaccardIndex state updates,
// utils/metrics.py:4-13, core/seg_trainer.py:118-119).  One [C,C] int64 matrix feeds
// both Dice (macro) and IoU, and is the only tensor all-reduced across ranks at validation.
// confmat[target][pred]; target == ignore_index pixels are skipped.
#include "common.h"
#include "launchers.h"

namespace {
constexpr int kBlock = 256;
constexpr int kMaxBins = 1024;

__global__ __launch_bounds__(kBlock) void confmat_kernel(const float* __restrict__ logits,
                                                         const int64_t* __restrict__ target,
                                                         int64_t* __restrict__ confmat, int N, int C, long HW,
                                                         int ignore_index) {
  __shared__ unsigned int hist[kMaxBins];
  const int bins = C * C;
  for (int i = threadIdx.x; i < bins; i += kBlock) hist[i] = 0;
  __syncthreads();
  const long P = (long)N * HW;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < P; i += (long)gridDim.x * kBlock) {
    const long t = target[i];
    if (t == ignore_index || t < 0 || t >= C) continue;
    const long n = i / HW, p = i - n * HW;
    const float* x = logits + n * C * HW + p;
    int best = 0;
    float bv = x[0];
    for (int c = 1; c < C; ++c) {
      const float v = x[c * HW];
      if (v > bv) { bv = v; best = c; }
    }
    atomicAdd(&hist[t * C + best], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < bins; i += kBlock)
    if (hist[i]) atomicAdd(reinterpret_cast<unsigned long long*>(confmat + i), (unsigned long long)hist[i]);
}
}  // namespace

void confmat_update(const float* logits, const int64_t* target, int64_t* confmat, int N, int C, long HW,
                    int ignore_index, hipStream_t s) {
  long b = ((long)N * HW + kBlock * 16 - 1) / (kBlock * 16);
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(confmat_kernel, dim3(b), dim3(kBlock), 0, s, logits, target, confmat, N, C, HW, ignore_index);
}
