// Layout conversion and bandwidth-bound glue kernels for NHWC bf16 feature maps (16-B vectors).
//   nchw_to_nhwc / nhwc_to_nchw : model boundary (fp32 NCHW images / logits <-> internal NHWC bf16)
//   up2_add / pool2_sum         : DUCKNet decoder `F.interpolate(nearest, 2x) + skip`
//                                 (reference models/ducknet.py:82-84) and its backward
//   add_n                       : encoder `x_i + x` merges (ducknet.py:39-43)
#include "common.h"
#include "launchers.h"

namespace {
constexpr int kBlock = 256;

int grid_for(long n) {
  long b = (n + kBlock - 1) / kBlock;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, int N, int C, long HW,
                                    int Cp) {
  const int CG = Cp / 8;
  const long total = (long)N * HW * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int g = (int)(i % CG);
    const long pix = i / CG;
    const long n = pix / HW, p = pix - n * HW;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = 8 * g + e;
      v[e] = c < C ? x[(n * C + c) * HW + p] : 0.f;
    }
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(v);
  }
}

__global__ void nhwc_to_nchw_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, int N, int C, long HW,
                                    int Cp) {
  const long total = (long)N * C * HW;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const long p = i % HW;
    const long nc = i / HW;
    const int c = (int)(nc % C);
    const long n = nc / C;
    y[i] = bf2f(x[(n * HW + p) * Cp + c]);
  }
}

__global__ void up2_add_kernel(const uint16_t* __restrict__ low, const uint16_t* __restrict__ skip,
                               uint16_t* __restrict__ out, int N, int h, int w, int Cp, const float* __restrict__ lc,
                               int lrelu, const float* __restrict__ sc, int srelu) {
  const int CG = Cp / 8, H = 2 * h, W = 2 * w;
  const long total = (long)N * H * W * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int g = (int)(i % CG);
    long pix = i / CG;
    const int X = (int)(pix % W);
    pix /= W;
    const int Y = (int)(pix % H);
    const long n = pix / H;
    float a[8], b[8];
    uint4 va = *reinterpret_cast<const uint4*>(skip + i * 8);
    uint4 vb = *reinterpret_cast<const uint4*>(low + ((n * h + (Y >> 1)) * w + (X >> 1)) * Cp + 8 * g);
    if (sc != nullptr) va = xform8(va, sc, Cp, 8 * g, srelu != 0);   // deferred-BN prologues
    if (lc != nullptr) vb = xform8(vb, lc, Cp, 8 * g, lrelu != 0);
    unpack8(va, a);
    unpack8(vb, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] += b[e];
    *reinterpret_cast<uint4*>(out + i * 8) = pack8(a);
  }
}

__global__ void pool2_sum_kernel(const uint16_t* __restrict__ gr, uint16_t* __restrict__ out, int N, int h, int w,
                                 int Cp) {
  const int CG = Cp / 8, W = 2 * w;
  const long total = (long)N * h * w * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int g = (int)(i % CG);
    long pix = i / CG;
    const int x = (int)(pix % w);
    pix /= w;
    const int y = (int)(pix % h);
    const long n = pix / h;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(gr + ((n * 2 * h + 2 * y + dy) * W + 2 * x + dx) * Cp + 8 * g), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    *reinterpret_cast<uint4*>(out + i * 8) = pack8(acc);
  }
}

struct Ptrs { const uint16_t* p[kMaxSumInputs]; const float* c[kMaxSumInputs]; unsigned relu; };

DEVI uint4 load_vec(const Ptrs& in, int j, long i, int CG) {
  uint4 v = *reinterpret_cast<const uint4*>(in.p[j] + i * 8);
  if (in.c[j] != nullptr) v = xform8(v, in.c[j], 8 * CG, 8 * (int)(i % CG), (in.relu >> j) & 1u);
  return v;
}

// ReLU6 (MobileNetV2): y = min(max(x, 0), 6); backward dx = dy where 0 < y < 6 (hardtanh's mask, from the output)
__global__ __launch_bounds__(kBlock) void relu6_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                       long nvec) {
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < nvec; i += (long)gridDim.x * kBlock) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(x + i * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fminf(fmaxf(v[e], 0.f), 6.f);
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(v);
  }
}

// The first DUCK block's in_bn over the (8-channel padded) image, augmented for its gamma / beta gradients
// (ops.bn.aug_in_bn): out[p] = [relu(s*x + h) for c < C, (s*x + h > 0) for the next C channels, 0 ...].
// The first convs read it in place of the deferred z (their weights for channels >= C are zero), and their
// weight-gradient slabs then also hold the correlations of dY with the ReLU mask.
__global__ __launch_bounds__(kBlock) void bn_aug_mask_kernel(const uint16_t* __restrict__ x, const float* __restrict__ st,
                                                             uint16_t* __restrict__ out, long npix, int C) {
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < npix; i += (long)gridDim.x * kBlock) {
    float v[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(x + i * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < C) {
        const float a = fmaf(v[e], st[e], st[8 + e]);
        o[e] = fmaxf(a, 0.f);
        o[e + C] = a > 0.f ? 1.f : 0.f;
      }
    }
    *reinterpret_cast<uint4*>(out + i * 8) = pack8(o);
  }
}

__global__ __launch_bounds__(kBlock) void relu6_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                                                           uint16_t* __restrict__ dx, long nvec) {
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < nvec; i += (long)gridDim.x * kBlock) {
    float g[8], v[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + i * 8), g);
    unpack8(*reinterpret_cast<const uint4*>(y + i * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = (v[e] > 0.f && v[e] < 6.f) ? g[e] : 0.f;
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(g);
  }
}

__global__ void add_n_kernel(Ptrs in, int k, uint16_t* __restrict__ out, long nvec, int CG) {
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < nvec; i += (long)gridDim.x * kBlock) {
    float a[8];
    unpack8(load_vec(in, 0, i, CG), a);
    for (int j = 1; j < k; ++j) {
      float b[8];
      unpack8(load_vec(in, j, i, CG), b);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += b[e];
    }
    *reinterpret_cast<uint4*>(out + i * 8) = pack8(a);
  }
}

__global__ void scale_f32_kernel(float* __restrict__ x, const float* __restrict__ scalar, float mult, long n) {
  const float s = (scalar != nullptr ? scalar[0] : 1.f) * mult;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long)gridDim.x * kBlock) x[i] *= s;
}
}  // namespace

void nchw_to_nhwc(const float* x, uint16_t* y, int N, int C, int H, int W, int Cp, hipStream_t s) {
  const long total = (long)N * H * W * (Cp / 8);
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for(total)), dim3(kBlock), 0, s, x, y, N, C, (long)H * W, Cp);
}

void nhwc_to_nchw(const uint16_t* x, float* y, int N, int C, int H, int W, int Cp, hipStream_t s) {
  const long total = (long)N * C * H * W;
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3(grid_for(total)), dim3(kBlock), 0, s, x, y, N, C, (long)H * W, Cp);
}

void up2_add(const uint16_t* low, const uint16_t* skip, uint16_t* out, int N, int h, int w, int Cp,
             const float* lc, int lrelu, const float* sc, int srelu, hipStream_t s) {
  const long total = (long)N * 4 * h * w * (Cp / 8);
  hipLaunchKernelGGL(up2_add_kernel, dim3(grid_for(total)), dim3(kBlock), 0, s, low, skip, out, N, h, w, Cp, lc, lrelu,
                     sc, srelu);
}

void pool2_sum(const uint16_t* g, uint16_t* out, int N, int h, int w, int Cp, hipStream_t s) {
  const long total = (long)N * h * w * (Cp / 8);
  hipLaunchKernelGGL(pool2_sum_kernel, dim3(grid_for(total)), dim3(kBlock), 0, s, g, out, N, h, w, Cp);
}

void relu6(const uint16_t* x, uint16_t* y, long n_elem, hipStream_t s) {
  hipLaunchKernelGGL(relu6_kernel, dim3(grid_for(n_elem / 8)), dim3(kBlock), 0, s, x, y, n_elem / 8);
}

void bn_aug_mask(const uint16_t* x, const float* stats, uint16_t* out, long npix, int C, hipStream_t s) {
  hipLaunchKernelGGL(bn_aug_mask_kernel, dim3(grid_for(npix)), dim3(kBlock), 0, s, x, stats, out, npix, C);
}

void relu6_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n_elem, hipStream_t s) {
  hipLaunchKernelGGL(relu6_bwd_kernel, dim3(grid_for(n_elem / 8)), dim3(kBlock), 0, s, dy, y, dx, n_elem / 8);
}

void add_n(const uint16_t* const* inputs, const float* const* coefs, unsigned relu_mask, int k, uint16_t* out,
           long n_elem, int Cp, hipStream_t s) {
  Ptrs in{};
  for (int i = 0; i < k; ++i) {
    in.p[i] = inputs[i];
    in.c[i] = coefs != nullptr ? coefs[i] : nullptr;
  }
  in.relu = relu_mask;
  const long nvec = n_elem / 8;
  hipLaunchKernelGGL(add_n_kernel, dim3(grid_for(nvec)), dim3(kBlock), 0, s, in, k, out, nvec, Cp / 8);
}

void scale_f32(float* x, const float* scalar, float mult, long n, hipStream_t s) {
  hipLaunchKernelGGL(scale_f32_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, x, scalar, mult, n);
}
