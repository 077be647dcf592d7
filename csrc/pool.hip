// Pooling / resampling glue for the encoder-decoder families on NHWC bf16 feature maps (16-B vectors,
// one thread = 8 channels of one pixel).
//   maxpool_fwd / maxpool_bwd : nn.MaxPool2d(k, s, p) -- UNet encoder (reference models/unet.py:49)
//                               and the ResNet stem (smp encoder).  The forward records the winning
//                               tap per element as one byte; the backward GATHERS (each input pixel
//                               visits the <= ceil(k/s)^2 windows that contain it), so overlapping
//                               windows need no atomics and the result is deterministic.
//   up2_cat / up2_cat_bwd     : smp UnetDecoderBlock `cat([interpolate(x, 2, nearest), skip])`
//                               into one dense channel range (logical channels packed, padded once).
//   add_act / relu_bwd        : ResNet `relu(bn(conv(x)) + identity)` tail and its backward.
#include "common.h"
#include "launchers.h"

namespace {
constexpr int kBlock = 256;

int grid_for(long n) {
  long b = (n + kBlock - 1) / kBlock;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (int)b;
}

__global__ __launch_bounds__(kBlock) void maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                             uint8_t* __restrict__ idx, int N, int IH, int IW, int OH,
                                                             int OW, int Cp, int k, int s, int p) {
  const int CG = Cp / 8;
  const long total = (long)N * OH * OW * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int g = (int)(i % CG);
    long pix = i / CG;
    const int ox = (int)(pix % OW);
    pix /= OW;
    const int oy = (int)(pix % OH);
    const long n = pix / OH;
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -__builtin_inff(); arg[e] = 0; }
    const int y0 = oy * s - p, x0 = ox * s - p;
    for (int r = 0; r < k; ++r) {
      const int iy = y0 + r;
      if (iy < 0 || iy >= IH) continue;
      for (int c = 0; c < k; ++c) {
        const int ix = x0 + c;
        if (ix < 0 || ix >= IW) continue;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(x + (((n * IH + iy) * IW + ix) * Cp) + 8 * g), v);
        const uint8_t t = (uint8_t)(r * k + c);
#pragma unroll
        for (int e = 0; e < 8; ++e)      // strict '>' keeps the first maximum (torch's scan order);
          if (v[e] > best[e] || v[e] != v[e]) { best[e] = v[e]; arg[e] = t; }   // NaN propagates
      }
    }
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(best);
    uint2 a;
    a.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
    a.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
    *reinterpret_cast<uint2*>(idx + i * 8) = a;
  }
}

__global__ __launch_bounds__(kBlock) void maxpool_bwd_kernel(const uint16_t* __restrict__ dy,
                                                             const uint8_t* __restrict__ idx, uint16_t* __restrict__ dx,
                                                             int N, int IH, int IW, int OH, int OW, int Cp, int k,
                                                             int s, int p) {
  const int CG = Cp / 8;
  const long total = (long)N * IH * IW * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int g = (int)(i % CG);
    long pix = i / CG;
    const int ix = (int)(pix % IW);
    pix /= IW;
    const int iy = (int)(pix % IH);
    const long n = pix / IH;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // windows oy with oy*s - p <= iy <= oy*s - p + k - 1
    const int oy_lo = max(0, (iy + p - k + s) / s), oy_hi = min(OH - 1, (iy + p) / s);
    const int ox_lo = max(0, (ix + p - k + s) / s), ox_hi = min(OW - 1, (ix + p) / s);
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
      const int r = iy - (oy * s - p);
      if (r < 0 || r >= k) continue;
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        const int c = ix - (ox * s - p);
        if (c < 0 || c >= k) continue;
        const long o = ((n * OH + oy) * OW + ox) * Cp + 8 * g;
        const uint2 a = *reinterpret_cast<const uint2*>(idx + o);
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(dy + o), v);
        const uint32_t t = (uint32_t)(r * k + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t w = e < 4 ? a.x : a.y;
          if (((w >> (8 * (e & 3))) & 0xffu) == t) acc[e] += v[e];
        }
      }
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(acc);
  }
}

// out[n, Y, X, c] = c < Cl ? low[n, Y/2, X/2, c] : c < Cl + Cs ? skip[n, Y, X, c - Cl] : 0
__global__ __launch_bounds__(kBlock) void up2_cat_kernel(const uint16_t* __restrict__ low,
                                                         const uint16_t* __restrict__ skip, uint16_t* __restrict__ out,
                                                         int N, int h, int w, int Cl, int Cpl, int Cs, int Cps,
                                                         int Cpo) {
  const int CG = Cpo / 8, H = 2 * h, W = 2 * w;
  const long total = (long)N * H * W * CG;
  const bool aligned = (Cl % 8) == 0;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int g = (int)(i % CG);
    long pix = i / CG;
    const int X = (int)(pix % W);
    pix /= W;
    const int Y = (int)(pix % H);
    const long n = pix / H;
    const long lo = ((n * h + (Y >> 1)) * w + (X >> 1)) * Cpl;
    const long sk = ((n * H + Y) * W + X) * (long)Cps;
    const int c0 = 8 * g;
    uint4 v;
    if (aligned && c0 + 8 <= Cl) {
      v = *reinterpret_cast<const uint4*>(low + lo + c0);
    } else if (aligned && c0 >= Cl && c0 + 8 <= Cl + Cs && (Cs % 8) == 0) {
      v = *reinterpret_cast<const uint4*>(skip + sk + (c0 - Cl));
    } else {
      uint16_t e8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        e8[e] = c < Cl ? low[lo + c] : (c < Cl + Cs ? skip[sk + c - Cl] : (uint16_t)0);
      }
      v = make_uint4(e8[0] | ((uint32_t)e8[1] << 16), e8[2] | ((uint32_t)e8[3] << 16),
                     e8[4] | ((uint32_t)e8[5] << 16), e8[6] | ((uint32_t)e8[7] << 16));
    }
    *reinterpret_cast<uint4*>(out + i * 8) = v;
  }
}

// dlow[n, y, x, c] = sum_{2x2} g[n, 2y+dy, 2x+dx, c]   (c < Cl; padding channels 0)
__global__ __launch_bounds__(kBlock) void up2_cat_bwd_low_kernel(const uint16_t* __restrict__ gr,
                                                                 uint16_t* __restrict__ dlow, int N, int h, int w,
                                                                 int Cl, int Cpl, int Cpo) {
  const int CG = Cpl / 8, W = 2 * w;
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
    for (int d = 0; d < 4; ++d) {
      const long o = ((n * 2 * h + 2 * y + (d >> 1)) * W + 2 * x + (d & 1)) * (long)Cpo + 8 * g;
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(gr + o), v);   // g columns >= Cl masked below
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (8 * g + e >= Cl) acc[e] = 0.f;
    *reinterpret_cast<uint4*>(dlow + i * 8) = pack8(acc);
  }
}

// dskip[n, Y, X, c] = g[n, Y, X, Cl + c]   (c < Cs; padding channels 0)
__global__ __launch_bounds__(kBlock) void up2_cat_bwd_skip_kernel(const uint16_t* __restrict__ gr,
                                                                  uint16_t* __restrict__ dskip, long P, int Cl,
                                                                  int Cs, int Cps, int Cpo) {
  const int CG = Cps / 8;
  const long total = P * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int g = (int)(i % CG);
    const long pix = i / CG;
    const int c0 = 8 * g;
    uint4 v;
    if ((Cl % 8) == 0 && c0 + 8 <= Cs) {
      v = *reinterpret_cast<const uint4*>(gr + pix * Cpo + Cl + c0);
    } else {
      uint16_t e8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        e8[e] = c < Cs ? gr[pix * Cpo + Cl + c] : (uint16_t)0;
      }
      v = make_uint4(e8[0] | ((uint32_t)e8[1] << 16), e8[2] | ((uint32_t)e8[3] << 16),
                     e8[4] | ((uint32_t)e8[5] << 16), e8[6] | ((uint32_t)e8[7] << 16));
    }
    *reinterpret_cast<uint4*>(dskip + i * 8) = v;
  }
}

__global__ __launch_bounds__(kBlock) void add_act_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                                                         uint16_t* __restrict__ z, long nvec, int relu) {
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < nvec; i += (long)gridDim.x * kBlock) {
    float u[8], v[8];
    unpack8(*reinterpret_cast<const uint4*>(a + i * 8), u);
    unpack8(*reinterpret_cast<const uint4*>(b + i * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float t = u[e] + v[e];
      u[e] = relu ? fmaxf(t, 0.f) : t;
    }
    *reinterpret_cast<uint4*>(z + i * 8) = pack8(u);
  }
}

// g = dz * (z > 0)
__global__ __launch_bounds__(kBlock) void relu_bwd_kernel(const uint16_t* __restrict__ dz,
                                                          const uint16_t* __restrict__ z, uint16_t* __restrict__ g,
                                                          long nvec) {
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < nvec; i += (long)gridDim.x * kBlock) {
    float d[8], v[8];
    unpack8(*reinterpret_cast<const uint4*>(dz + i * 8), d);
    unpack8(*reinterpret_cast<const uint4*>(z + i * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = v[e] > 0.f ? d[e] : 0.f;
    *reinterpret_cast<uint4*>(g + i * 8) = pack8(d);
  }
}
}  // namespace

void maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int IH, int IW, int OH, int OW, int Cp, int k,
                 int s, int p, hipStream_t st) {
  const long total = (long)N * OH * OW * (Cp / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(total)), dim3(kBlock), 0, st, x, y, idx, N, IH, IW, OH, OW,
                     Cp, k, s, p);
}

void maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int IH, int IW, int OH, int OW, int Cp,
                 int k, int s, int p, hipStream_t st) {
  const long total = (long)N * IH * IW * (Cp / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total)), dim3(kBlock), 0, st, dy, idx, dx, N, IH, IW, OH, OW,
                     Cp, k, s, p);
}

void up2_cat(const uint16_t* low, const uint16_t* skip, uint16_t* out, int N, int h, int w, int Cl, int Cpl, int Cs,
             int Cps, int Cpo, hipStream_t st) {
  const long total = (long)N * 4 * h * w * (Cpo / 8);
  hipLaunchKernelGGL(up2_cat_kernel, dim3(grid_for(total)), dim3(kBlock), 0, st, low, skip, out, N, h, w, Cl, Cpl, Cs,
                     Cps, Cpo);
}

void up2_cat_bwd(const uint16_t* g, uint16_t* dlow, uint16_t* dskip, int N, int h, int w, int Cl, int Cpl, int Cs,
                 int Cps, int Cpo, hipStream_t st) {
  const long tl = (long)N * h * w * (Cpl / 8);
  hipLaunchKernelGGL(up2_cat_bwd_low_kernel, dim3(grid_for(tl)), dim3(kBlock), 0, st, g, dlow, N, h, w, Cl, Cpl, Cpo);
  if (dskip != nullptr && Cs > 0) {
    const long P = (long)N * 4 * h * w;
    hipLaunchKernelGGL(up2_cat_bwd_skip_kernel, dim3(grid_for(P * (Cps / 8))), dim3(kBlock), 0, st, g, dskip, P, Cl,
                       Cs, Cps, Cpo);
  }
}

void add_act(const uint16_t* a, const uint16_t* b, uint16_t* z, long n_elem, int relu, hipStream_t st) {
  const long nvec = n_elem / 8;
  hipLaunchKernelGGL(add_act_kernel, dim3(grid_for(nvec)), dim3(kBlock), 0, st, a, b, z, nvec, relu);
}

void relu_bwd(const uint16_t* dz, const uint16_t* z, uint16_t* g, long n_elem, hipStream_t st) {
  const long nvec = n_elem / 8;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_for(nvec)), dim3(kBlock), 0, st, dz, z, g, nvec);
}
