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

// ---- inference glue: bilinear resize and argmax -> colormap (K23) --------------------
namespace {
// F.interpolate(x, (OH, OW), mode='bilinear', align_corners=ac) on fp32 NCHW, one thread per output.
__global__ __launch_bounds__(kBlock) void bilinear_kernel(const float* __restrict__ x, float* __restrict__ y, long NC,
                                                          int IH, int IW, int OH, int OW, int ac) {
  const long total = NC * OH * OW;
  const float sh = ac ? (OH > 1 ? (float)(IH - 1) / (OH - 1) : 0.f) : (float)IH / OH;
  const float sw = ac ? (OW > 1 ? (float)(IW - 1) / (OW - 1) : 0.f) : (float)IW / OW;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int ox = (int)(i % OW);
    const long r = i / OW;
    const int oy = (int)(r % OH);
    const long nc = r / OH;
    const float fy = ac ? oy * sh : fmaxf((oy + 0.5f) * sh - 0.5f, 0.f);
    const float fx = ac ? ox * sw : fmaxf((ox + 0.5f) * sw - 0.5f, 0.f);
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < IH - 1), x1 = x0 + (x0 < IW - 1);
    const float ly = fy - y0, lx = fx - x0;
    const float* p = x + nc * IH * IW;
    y[i] = (1.f - ly) * ((1.f - lx) * p[y0 * IW + x0] + lx * p[y0 * IW + x1]) +
           ly * ((1.f - lx) * p[y1 * IW + x0] + lx * p[y1 * IW + x1]);
  }
}

// logits [N, C, HW] -> rgb [N, HW, 3] uint8 via lut [C', 3]; C == 1 -> sigmoid > 0.5 (logit > 0)
__global__ __launch_bounds__(kBlock) void colorize_kernel(const float* __restrict__ logits,
                                                          const uint8_t* __restrict__ lut, uint8_t* __restrict__ rgb,
                                                          int N, int C, long HW) {
  const long P = (long)N * HW;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < P; i += (long)gridDim.x * kBlock) {
    const long n = i / HW, p = i - n * HW;
    const float* x = logits + n * C * HW + p;
    int best = 0;
    if (C == 1) {
      best = x[0] > 0.f;
    } else {
      float bv = x[0];
      for (int c = 1; c < C; ++c) {
        const float v = x[c * HW];
        if (v > bv) { bv = v; best = c; }
      }
    }
    rgb[i * 3 + 0] = lut[best * 3 + 0];
    rgb[i * 3 + 1] = lut[best * 3 + 1];
    rgb[i * 3 + 2] = lut[best * 3 + 2];
  }
}

int grid1d(long n) {
  long b = (n + kBlock - 1) / kBlock;
  return (int)(b > 16384 ? 16384 : (b < 1 ? 1 : b));
}
}  // namespace

void bilinear_resize(const float* x, float* y, long NC, int IH, int IW, int OH, int OW, int align_corners,
                     hipStream_t s) {
  hipLaunchKernelGGL(bilinear_kernel, dim3(grid1d(NC * OH * OW)), dim3(kBlock), 0, s, x, y, NC, IH, IW, OH, OW,
                     align_corners);
}

void colorize(const float* logits, const uint8_t* lut, uint8_t* rgb, int N, int C, long HW, hipStream_t s) {
  hipLaunchKernelGGL(colorize_kernel, dim3(grid1d((long)N * HW)), dim3(kBlock), 0, s, logits, lut, rgb, N, C, HW);
}
