// Kernels of the smp decoder hub's non-conv ops, NHWC bf16 (16-B vectors of 8 channels), fp32 math,
// deterministic (no atomics: every backward is a gather, every reduction a fixed-order partial sum).
//
//   resize_bilinear_fwd/bwd : F.interpolate(mode='bilinear', align_corners=True/False) and
//                             nn.UpsamplingBilinear2d -- FPN segmentation blocks, PSP / ASPP pooling
//                             upsampling, DeepLabV3+ decoder, PAN (SURVEY §2.4 decoder_hub; reference
//                             models/__init__.py:8-10)
//   nc_sums                 : per-(image, channel) sums over the pixels (GroupNorm statistics, global /
//                             adaptive average pooling backward-free forward, GN backward sums)
//   gn_finalize / gn_bwd_finalize : nn.GroupNorm(32, C) training statistics -> per-(image, channel)
//                             affine coefficients (FPN Conv3x3GNReLU)
//   affine_nc_act / affine_nc_bwd : z = act(x*s[n,c] + h[n,c]); dx = k1*dzr + k2*x + k3 per (n, c)
//   adaptive_avgpool_fwd/bwd: nn.AdaptiveAvgPool2d (PSPNet bins 1/2/3/6, ASPP/PAN/MAnet global pooling)
//   dwconv_fwd / dwconv_wgrad : depthwise conv (DeepLabV3+ SeparableConv2d), stride 1, any taps; the
//                             data-gradient is the forward with negated tap offsets
#include <algorithm>

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

// PyTorch's bilinear source index (aten area_pixel_compute_source_index, linear mode): i0, i1, lambda
struct Lin { int i0, i1; float l; };
DEVI Lin lin_src(int o, int in, float scale, int align) {
  float src = align ? scale * (float)o : fmaxf(scale * ((float)o + 0.5f) - 0.5f, 0.f);
  int i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  Lin r;
  r.i0 = i0;
  r.i1 = i0 + (i0 < in - 1 ? 1 : 0);
  r.l = src - (float)i0;
  return r;
}

// weight of output o on input i along one dimension (both taps may land on i at the border)
DEVI float lin_w(int o, int i, int in, float scale, int align) {
  const Lin r = lin_src(o, in, scale, align);
  return (r.i0 == i ? 1.f - r.l : 0.f) + (r.i1 == i ? r.l : 0.f);
}

__global__ __launch_bounds__(kBlock) void resize_bilinear_fwd_kernel(const uint16_t* __restrict__ x,
                                                                     uint16_t* __restrict__ y, int N, int IH,
                                                                     int IW, int OH, int OW, int Cp, float sh,
                                                                     float sw, int align, int accum) {
  const int CG = Cp >> 3;
  const long total = (long)N * OH * OW * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int cg = (int)(i % CG);
    long pix = i / CG;
    const int ox = (int)(pix % OW);
    pix /= OW;
    const int oy = (int)(pix % OH);
    const long n = pix / OH;
    const Lin ry = lin_src(oy, IH, sh, align), rx = lin_src(ox, IW, sw, align);
    const uint16_t* b = x + n * IH * IW * Cp + 8 * cg;
    float f00[8], f01[8], f10[8], f11[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)ry.i0 * IW + rx.i0) * Cp), f00);
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)ry.i0 * IW + rx.i1) * Cp), f01);
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)ry.i1 * IW + rx.i0) * Cp), f10);
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)ry.i1 * IW + rx.i1) * Cp), f11);
    const float wy1 = ry.l, wy0 = 1.f - ry.l, wx1 = rx.l, wx0 = 1.f - rx.l;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = wy0 * (wx0 * f00[e] + wx1 * f01[e]) + wy1 * (wx0 * f10[e] + wx1 * f11[e]);
    uint4* yp = reinterpret_cast<uint4*>(y + i * 8);
    if (accum) {   // y += up(x): the FPN merge sum / PSP branches without a separate add pass
      float a[8];
      unpack8(*yp, a);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += a[e];
    }
    *yp = pack8(o);
  }
}

// dX[iy, ix] = sum over the outputs whose taps land on (iy, ix): a gather over a window of outputs
// (those with a source coordinate within one pixel of the input) -- no atomics, fixed order
__global__ __launch_bounds__(kBlock) void resize_bilinear_bwd_kernel(const uint16_t* __restrict__ dy,
                                                                     uint16_t* __restrict__ dx, int N, int IH,
                                                                     int IW, int OH, int OW, int Cp, float sh,
                                                                     float sw, int align) {
  const int CG = Cp >> 3;
  const long total = (long)N * IH * IW * CG;
  // output window per input index: o with |src(o) - i| < 1; src(o) ~ o*s (+ const), so o in
  // [(i - 1 - 0.5)/s - 1, (i + 1 + 0.5)/s + 1]
  const float ish = sh > 0.f ? 1.f / sh : 0.f, isw = sw > 0.f ? 1.f / sw : 0.f;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int cg = (int)(i % CG);
    long pix = i / CG;
    const int ix = (int)(pix % IW);
    pix /= IW;
    const int iy = (int)(pix % IH);
    const long n = pix / IH;
    int y0 = 0, y1 = OH - 1, x0 = 0, x1 = OW - 1;
    if (sh > 0.f) {
      y0 = max(0, (int)floorf(((float)iy - 1.5f) * ish) - 1);
      y1 = min(OH - 1, (int)ceilf(((float)iy + 1.5f) * ish) + 1);
    }
    if (sw > 0.f) {
      x0 = max(0, (int)floorf(((float)ix - 1.5f) * isw) - 1);
      x1 = min(OW - 1, (int)ceilf(((float)ix + 1.5f) * isw) + 1);
    }
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const uint16_t* b = dy + n * OH * OW * Cp + 8 * cg;
    for (int oy = y0; oy <= y1; ++oy) {
      const float wy = lin_w(oy, iy, IH, sh, align);
      if (wy == 0.f) continue;
      for (int ox = x0; ox <= x1; ++ox) {
        const float w = wy * lin_w(ox, ix, IW, sw, align);
        if (w == 0.f) continue;
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(b + ((long)oy * OW + ox) * Cp), g);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(w, g[e], acc[e]);
      }
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(acc);
  }
}

// ---- per-(image, channel) sums ----------------------------------------------------------------------
// grid (nblk, N); block: thread owns 8-channel group cg = tid % CG for rows r = tid / CG over the pixels
// of its chunk.  mode 0: (sum x, sum x^2); mode 1: GN backward (sum dzr, sum dzr * xhat) with
// dzr = dz * relu'(x*s + h), xhat = (x - mean) * rstd from the [N][4][Cp] table (s, h, mean, rstd).
// part[n][blk][2][Cp]
__global__ __launch_bounds__(kBlock) void nc_sums_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dz,
                                                         const float* __restrict__ tab, int relu, long HW, int Cp,
                                                         float* __restrict__ part) {
  __shared__ float red[2][kBlock][8];
  const int CG = Cp >> 3, R = kBlock / CG, tid = threadIdx.x, cg = tid % CG, r = tid / CG;
  const long n = blockIdx.y;
  const int nblk = gridDim.x;
  float s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; q[e] = 0.f; }
  float sc[8], sf[8], mu[8], rs[8];
  if (dz != nullptr) {
    const float* t = tab + n * 4 * Cp + 8 * cg;
    load8f(t, sc); load8f(t + Cp, sf); load8f(t + 2 * Cp, mu); load8f(t + 3 * Cp, rs);
  }
  if (r < R) {
    const long per = (HW + nblk - 1) / nblk;
    const long p0 = (long)blockIdx.x * per, p1 = min(HW, p0 + per);
    const uint16_t* xb = x + n * HW * Cp + 8 * cg;
    const uint16_t* gb = dz != nullptr ? dz + n * HW * Cp + 8 * cg : nullptr;
    for (long p = p0 + r; p < p1; p += R) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(xb + p * Cp), v);
      if (gb == nullptr) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { s[e] += v[e]; q[e] = fmaf(v[e], v[e], q[e]); }
      } else {
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(gb + p * Cp), g);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gr = (!relu || fmaf(v[e], sc[e], sf[e]) > 0.f) ? g[e] : 0.f;
          s[e] += gr;
          q[e] = fmaf(gr, (v[e] - mu[e]) * rs[e], q[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][tid][e] = s[e]; red[1][tid][e] = q[e]; }
  __syncthreads();
  for (int c = tid; c < Cp; c += kBlock) {
    const int g = c >> 3, e = c & 7;
    float ss = 0.f, qq = 0.f;
    for (int rr = 0; rr < R; ++rr) { ss += red[0][rr * CG + g][e]; qq += red[1][rr * CG + g][e]; }
    float* o = part + ((n * nblk + blockIdx.x) * 2) * Cp;
    o[c] = ss;
    o[Cp + c] = qq;
  }
}

// GroupNorm forward finalize: one thread per (n, g): fp64 sums over the blocks (fixed order) and the
// group's channels -> mean, biased var, rstd; writes tab[n][4][Cp] = (scale, shift, mean, rstd) per
// channel (padded channels: zeros)
__global__ void gn_finalize_kernel(const float* __restrict__ part, int nblk, int N, int C, int Cp, int G, float eps,
                                   const float* __restrict__ gamma, const float* __restrict__ beta, long HW,
                                   float* __restrict__ tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * G) return;
  const int n = i / G, g = i - n * G, cpg = C / G;
  double s = 0.0, q = 0.0;
  for (int b = 0; b < nblk; ++b) {
    const float* o = part + ((long)(n * nblk + b) * 2) * Cp;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) { s += o[c]; q += o[Cp + c]; }
  }
  const double M = (double)HW * cpg;
  const double m = s / M;
  double v = q / M - m * m;
  if (v < 0) v = 0;
  const float rstd = (float)(1.0 / sqrt(v + (double)eps));
  float* t = tab + (long)n * 4 * Cp;
  for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
    const float gm = gamma != nullptr ? gamma[c] : 1.f, bt = beta != nullptr ? beta[c] : 0.f;
    t[c] = gm * rstd;
    t[Cp + c] = bt - (float)m * gm * rstd;
    t[2 * Cp + c] = (float)m;
    t[3 * Cp + c] = rstd;
  }
  if (g == G - 1)
    for (int c = C; c < Cp; ++c) { t[c] = 0.f; t[Cp + c] = 0.f; t[2 * Cp + c] = 0.f; t[3 * Cp + c] = 0.f; }
}

// GroupNorm backward finalize.  A[n][c] = sum dzr, B[n][c] = sum dzr*xhat (over the blocks, fixed order).
// dgamma[c] += sum_n B, dbeta[c] += sum_n A (one thread per channel, images in order); per (n, g):
// S1 = sum_c gamma A, S2 = sum_c gamma B -> dx = k1 dzr + k2 x + k3 with k1 = rstd*gamma,
// k2 = -rstd^2 S2 / M, k3 = -rstd S1 / M - k2 * mean.  coef[n][3][Cp].
__global__ void gn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int N, int C, int Cp, int G,
                                       const float* __restrict__ gamma, const float* __restrict__ tab, long HW,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta,
                                       float* __restrict__ coef) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int cpg = C / G;
  if (i < N * G) {
    const int n = i / G, g = i - n * G;
    double s1 = 0.0, s2 = 0.0;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      double a = 0.0, b = 0.0;
      for (int k = 0; k < nblk; ++k) {
        const float* o = part + ((long)(n * nblk + k) * 2) * Cp;
        a += o[c]; b += o[Cp + c];
      }
      const double gm = gamma != nullptr ? gamma[c] : 1.0;
      s1 += gm * a; s2 += gm * b;
    }
    const float* t = tab + (long)n * 4 * Cp;
    float* k = coef + (long)n * 3 * Cp;
    const double M = (double)HW * cpg;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      const double rstd = t[3 * Cp + c], mean = t[2 * Cp + c];
      const double gm = gamma != nullptr ? gamma[c] : 1.0;
      const double k2 = -rstd * rstd * s2 / M;
      k[c] = (float)(rstd * gm);
      k[Cp + c] = (float)k2;
      k[2 * Cp + c] = (float)(-rstd * s1 / M - k2 * mean);
    }
    if (g == G - 1)
      for (int c = C; c < Cp; ++c) { k[c] = 0.f; k[Cp + c] = 0.f; k[2 * Cp + c] = 0.f; }
  }
  // parameter gradients: the first C threads (any block) own one channel each
  if (i < C && (dgamma != nullptr || dbeta != nullptr)) {
    double a = 0.0, b = 0.0;
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < nblk; ++k) {
        const float* o = part + ((long)(n * nblk + k) * 2) * Cp;
        a += o[i]; b += o[Cp + i];
      }
    if (dbeta != nullptr) dbeta[i] += (float)a;
    if (dgamma != nullptr) dgamma[i] += (float)b;
  }
}

// z = act(x * s[n,c] + h[n,c])  (tab rows 0, 1 of [N][rows][Cp])
__global__ __launch_bounds__(kBlock) void affine_nc_kernel(const uint16_t* __restrict__ x, const float* __restrict__ tab,
                                                           int rows, uint16_t* __restrict__ z, int N, long HW, int Cp,
                                                           int relu) {
  const int CG = Cp >> 3;
  const long total = (long)N * HW * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int cg = (int)(i % CG);
    const long n = i / CG / HW;
    const float* t = tab + n * rows * Cp + 8 * cg;
    float s[8], h[8];
    load8f(t, s);
    load8f(t + Cp, h);
    *reinterpret_cast<uint4*>(z + i * 8) = affine8(*reinterpret_cast<const uint4*>(x + i * 8), s, h, relu != 0);
  }
}

// dx = k1 * dzr + k2 * x + k3 per (n, c); dzr = dz * relu'(x*s + h)
__global__ __launch_bounds__(kBlock) void affine_nc_bwd_kernel(const uint16_t* __restrict__ dz,
                                                               const uint16_t* __restrict__ x,
                                                               const float* __restrict__ tab,
                                                               const float* __restrict__ coef,
                                                               uint16_t* __restrict__ dx, int N, long HW, int Cp,
                                                               int relu) {
  const int CG = Cp >> 3;
  const long total = (long)N * HW * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int cg = (int)(i % CG);
    const long n = i / CG / HW;
    const float* t = tab + n * 4 * Cp + 8 * cg;
    const float* k = coef + n * 3 * Cp + 8 * cg;
    float s[8], h[8], k1[8], k2[8], k3[8], v[8], g[8];
    load8f(t, s); load8f(t + Cp, h);
    load8f(k, k1); load8f(k + Cp, k2); load8f(k + 2 * Cp, k3);
    unpack8(*reinterpret_cast<const uint4*>(x + i * 8), v);
    unpack8(*reinterpret_cast<const uint4*>(dz + i * 8), g);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gr = (!relu || fmaf(v[e], s[e], h[e]) > 0.f) ? g[e] : 0.f;
      g[e] = k1[e] * gr + k2[e] * v[e] + k3[e];
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(g);
  }
}

// ---- adaptive average pooling (bins as nn.AdaptiveAvgPool2d: [floor(o*I/O), ceil((o+1)*I/O)) ) --------
DEVI int bin_lo(int o, int I, int O) { return (o * I) / O; }
DEVI int bin_hi(int o, int I, int O) { return ((o + 1) * I + O - 1) / O; }

// one block per output pixel (n, oy, ox): 256 threads = CG channel groups x R pixel rows, LDS reduce
__global__ __launch_bounds__(kBlock) void adaptive_avgpool_fwd_kernel(const uint16_t* __restrict__ x,
                                                                      uint16_t* __restrict__ y, int H, int W,
                                                                      int OH, int OW, int Cp) {
  __shared__ float red[kBlock][8];
  const int CG = Cp >> 3, R = kBlock / CG, tid = threadIdx.x, r = tid / CG;
  const long o = blockIdx.x;
  const int ox = (int)(o % OW), oy = (int)((o / OW) % OH);
  const long n = o / OW / OH;
  const int ys = bin_lo(oy, H, OH), ye = bin_hi(oy, H, OH), xs = bin_lo(ox, W, OW), xe = bin_hi(ox, W, OW);
  const int bw = xe - xs, cnt = (ye - ys) * bw;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const int cg = tid % CG;
  if (r < R) {
    for (int k = r; k < cnt; k += R) {
      const int py = ys + k / bw, px = xs + k % bw;
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(x + ((n * H + py) * W + px) * Cp + 8 * cg), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tid][e] = acc[e];
  __syncthreads();
  if (tid < CG) {
    float s[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = 0.f;
    for (int rr = 0; rr < R; ++rr)
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += red[rr * CG + tid][e];
    const float inv = 1.f / (float)cnt;
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] *= inv;
    *reinterpret_cast<uint4*>(y + o * Cp + 8 * tid) = pack8(s);
  }
}

__global__ __launch_bounds__(kBlock) void adaptive_avgpool_bwd_kernel(const uint16_t* __restrict__ dy,
                                                                      uint16_t* __restrict__ dx, int N, int H, int W,
                                                                      int OH, int OW, int Cp) {
  const int CG = Cp >> 3;
  const long total = (long)N * H * W * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int cg = (int)(i % CG);
    long pix = i / CG;
    const int ix = (int)(pix % W);
    pix /= W;
    const int iy = (int)(pix % H);
    const long n = pix / H;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    // bins containing iy: oy in [floor(iy*OH/H) - 1, floor(iy*OH/H) + 1] (bins overlap by < 1 bin)
    const int cy = (iy * OH) / H, cx = (ix * OW) / W;
    for (int oy = max(0, cy - 1); oy <= min(OH - 1, cy + 1); ++oy) {
      const int ys = bin_lo(oy, H, OH), ye = bin_hi(oy, H, OH);
      if (iy < ys || iy >= ye) continue;
      for (int ox = max(0, cx - 1); ox <= min(OW - 1, cx + 1); ++ox) {
        const int xs = bin_lo(ox, W, OW), xe = bin_hi(ox, W, OW);
        if (ix < xs || ix >= xe) continue;
        const float w = 1.f / (float)((ye - ys) * (xe - xs));
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(dy + ((n * OH + oy) * OW + ox) * Cp + 8 * cg), g);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(w, g[e], acc[e]);
      }
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(acc);
  }
}

// ---- depthwise conv, stride 1: y[p] = sum_t w[t] * x[p + off_t] (+ bias); w fp32 [T][Cp] ----------------
struct DwTaps { int T; int dy[kMaxTaps]; int dx[kMaxTaps]; };

__global__ __launch_bounds__(kBlock) void dwconv_fwd_kernel(const uint16_t* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, uint16_t* __restrict__ y,
                                                            int N, int H, int W, int Cp, DwTaps tp) {
  const int CG = Cp >> 3;
  const long total = (long)N * H * W * CG;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int cg = (int)(i % CG);
    long pix = i / CG;
    const int px = (int)(pix % W);
    pix /= W;
    const int py = (int)(pix % H);
    const long n = pix / H;
    float acc[8];
    if (bias != nullptr) load8f(bias + 8 * cg, acc);
    else {
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    }
    const uint16_t* b = x + n * H * W * Cp + 8 * cg;
    for (int t = 0; t < tp.T; ++t) {
      const int iy = py + tp.dy[t], ix = px + tp.dx[t];
      if ((unsigned)iy >= (unsigned)H || (unsigned)ix >= (unsigned)W) continue;
      float v[8], k[8];
      unpack8(*reinterpret_cast<const uint4*>(b + ((long)iy * W + ix) * Cp), v);
      load8f(w + (long)t * Cp + 8 * cg, k);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(v[e], k[e], acc[e]);
    }
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(acc);
  }
}

// weight (+ bias) gradient partials: part[blk][T + 1][Cp] (row T = sum dy for the bias), grid-stride
// over pixels; a thread owns one 8-channel group and keeps T*8 accumulators
template <int TM>
__global__ __launch_bounds__(kBlock) void dwconv_wgrad_kernel(const uint16_t* __restrict__ x,
                                                              const uint16_t* __restrict__ dy,
                                                              float* __restrict__ part, int N, int H, int W, int Cp,
                                                              DwTaps tp) {
  __shared__ float red[kBlock][8];
  const int CG = Cp >> 3, R = kBlock / CG, tid = threadIdx.x, cg = tid % CG, r = tid / CG;
  float acc[TM + 1][8];
#pragma unroll
  for (int t = 0; t <= TM; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[t][e] = 0.f;
  const long P = (long)N * H * W;
  if (r < R) {
    for (long p = (long)blockIdx.x * R + r; p < P; p += (long)gridDim.x * R) {
      const int px = (int)(p % W), py = (int)((p / W) % H);
      const long n = p / W / H;
      float g[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + p * Cp + 8 * cg), g);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[TM][e] += g[e];
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        if (t >= tp.T) break;
        const int iy = py + tp.dy[t], ix = px + tp.dx[t];
        if ((unsigned)iy >= (unsigned)H || (unsigned)ix >= (unsigned)W) continue;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(x + ((n * H + iy) * W + ix) * Cp + 8 * cg), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[t][e] = fmaf(v[e], g[e], acc[t][e]);
      }
    }
  }
  for (int t = 0; t <= tp.T; ++t) {
    const int ts = t == tp.T ? TM : t;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) red[tid][e] = acc[ts][e];
    __syncthreads();
    for (int c = tid; c < Cp; c += kBlock) {
      const int g = c >> 3, e = c & 7;
      float s = 0.f;
      for (int rr = 0; rr < R; ++rr) s += red[rr * CG + g][e];
      part[((long)blockIdx.x * (tp.T + 1) + t) * Cp + c] = s;
    }
  }
}

// column sums of [rows_in][ncol] fp32 partials in fixed order (fp64) -> out[ncol] (+= if accum)
__global__ void colsum_kernel(const float* __restrict__ part, int nrow, int ncol, float* __restrict__ out, int accum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncol) return;
  double s = 0.0;
  for (int r = 0; r < nrow; ++r) s += part[(long)r * ncol + c];
  out[c] = accum ? out[c] + (float)s : (float)s;
}

}  // namespace

void resize_bilinear_fwd(const uint16_t* x, uint16_t* y, int N, int IH, int IW, int OH, int OW, int Cp, float sh,
                         float sw, int align, int accum, hipStream_t s) {
  hipLaunchKernelGGL(resize_bilinear_fwd_kernel, dim3(grid_for((long)N * OH * OW * (Cp / 8))), dim3(kBlock), 0, s, x,
                     y, N, IH, IW, OH, OW, Cp, sh, sw, align, accum);
}

void resize_bilinear_bwd(const uint16_t* dy, uint16_t* dx, int N, int IH, int IW, int OH, int OW, int Cp, float sh,
                         float sw, int align, hipStream_t s) {
  hipLaunchKernelGGL(resize_bilinear_bwd_kernel, dim3(grid_for((long)N * IH * IW * (Cp / 8))), dim3(kBlock), 0, s, dy,
                     dx, N, IH, IW, OH, OW, Cp, sh, sw, align);
}

int nc_sums_blocks(long HW, int Cp) {
  const long R = kBlock / (Cp / 8);
  long b = (HW + R * 32 - 1) / (R * 32);   // >= 32 pixels per thread row
  if (b > 64) b = 64;
  if (b < 1) b = 1;
  return (int)b;
}

void nc_sums(const uint16_t* x, const uint16_t* dz, const float* tab, int relu, int N, long HW, int Cp, float* part,
             int nblk, hipStream_t s) {
  hipLaunchKernelGGL(nc_sums_kernel, dim3(nblk, N), dim3(kBlock), 0, s, x, dz, tab, relu, HW, Cp, part);
}

void gn_finalize(const float* part, int nblk, int N, int C, int Cp, int G, float eps, const float* gamma,
                 const float* beta, long HW, float* tab, hipStream_t s) {
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(cdiv((long)N * G, 64)), dim3(64), 0, s, part, nblk, N, C, Cp, G, eps,
                     gamma, beta, HW, tab);
}

void gn_bwd_finalize(const float* part, int nblk, int N, int C, int Cp, int G, const float* gamma, const float* tab,
                     long HW, float* dgamma, float* dbeta, float* coef, hipStream_t s) {
  const long n = std::max<long>((long)N * G, C);
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(cdiv(n, 64)), dim3(64), 0, s, part, nblk, N, C, Cp, G, gamma, tab, HW,
                     dgamma, dbeta, coef);
}

void affine_nc(const uint16_t* x, const float* tab, int rows, uint16_t* z, int N, long HW, int Cp, int relu,
               hipStream_t s) {
  hipLaunchKernelGGL(affine_nc_kernel, dim3(grid_for((long)N * HW * (Cp / 8))), dim3(kBlock), 0, s, x, tab, rows, z, N,
                     HW, Cp, relu);
}

void affine_nc_bwd(const uint16_t* dz, const uint16_t* x, const float* tab, const float* coef, uint16_t* dx, int N,
                   long HW, int Cp, int relu, hipStream_t s) {
  hipLaunchKernelGGL(affine_nc_bwd_kernel, dim3(grid_for((long)N * HW * (Cp / 8))), dim3(kBlock), 0, s, dz, x, tab,
                     coef, dx, N, HW, Cp, relu);
}

void adaptive_avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int H, int W, int OH, int OW, int Cp, hipStream_t s) {
  hipLaunchKernelGGL(adaptive_avgpool_fwd_kernel, dim3((unsigned)((long)N * OH * OW)), dim3(kBlock), 0, s, x, y, H, W,
                     OH, OW, Cp);
}

void adaptive_avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int H, int W, int OH, int OW, int Cp,
                          hipStream_t s) {
  hipLaunchKernelGGL(adaptive_avgpool_bwd_kernel, dim3(grid_for((long)N * H * W * (Cp / 8))), dim3(kBlock), 0, s, dy,
                     dx, N, H, W, OH, OW, Cp);
}

static DwTaps dw_taps(int T, const int* dy, const int* dx) {
  DwTaps tp{};
  tp.T = T;
  for (int t = 0; t < T; ++t) { tp.dy[t] = dy[t]; tp.dx[t] = dx[t]; }
  return tp;
}

void dwconv_fwd(const uint16_t* x, const float* w, const float* bias, uint16_t* y, int N, int H, int W, int Cp, int T,
                const int* dy, const int* dx, hipStream_t s) {
  hipLaunchKernelGGL(dwconv_fwd_kernel, dim3(grid_for((long)N * H * W * (Cp / 8))), dim3(kBlock), 0, s, x, w, bias, y,
                     N, H, W, Cp, dw_taps(T, dy, dx));
}

int dwconv_wgrad_blocks(long P, int Cp) {
  const long R = kBlock / (Cp / 8);
  long b = (P + R * 64 - 1) / (R * 64);
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (int)b;
}

int dwconv_wgrad(const uint16_t* x, const uint16_t* dyv, float* part, int nblk, int N, int H, int W, int Cp, int T,
                 const int* dy, const int* dx, hipStream_t s) {
  const DwTaps tp = dw_taps(T, dy, dx);
  if (T <= 9) {
    hipLaunchKernelGGL(dwconv_wgrad_kernel<9>, dim3(nblk), dim3(kBlock), 0, s, x, dyv, part, N, H, W, Cp, tp);
    return 0;
  }
  return 1;
}

void colsum(const float* part, int nrow, int ncol, float* out, int accum, hipStream_t s) {
  hipLaunchKernelGGL(colsum_kernel, dim3(cdiv(ncol, 256)), dim3(256), 0, s, part, nrow, ncol, out, accum);
}
