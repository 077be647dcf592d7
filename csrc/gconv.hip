// Grouped convolution (ResNeXt's grouped 3x3, torchvision ``Bottleneck.conv2`` with groups = 32) on NHWC
// bf16, fp32 accumulation -- forward, data-gradient and weight-gradient.
//
// Reference: models/__init__.py:8-10 (smp encoders incl. resnext50_32x4d; SURVEY §2 "encoders").  Until
// round 4 this was the one conv of the fused graph that ran on MIOpen's channels-last grouped kernels.
//
// A group has CG = C / groups channels in and out (ResNeXt 32x4d: 4, 8, 16, 32 on layers 1-4; depthwise 1),
// so per output channel the reduction is only CG x taps (9..288) long.  Round 5: 3x3 convs with C % 16 == 0
// run on the MFMA kernels at the end of this file (gconv_mfma / gconv_wgrad_mfma): a dense GEMM over a
// max(16, CG)-channel window with block-diagonal weights -- only CG / 16 of the MFMA work is useful at
// CG < 16, but the matrix cores have that to spare and the VALU kernels below were compute-bound (~14
// TFLOP/s): ResNeXt50 bs64 1227 -> 1749 img/s, MobileNetV2 2020 -> 2947 (profiles/r05/gconv/).
// The VALU kernels remain for the other shapes (non-3x3, C % 16 != 0, CG > 64) and as the A/B reference
// (env MSP_GCONV_MFMA=0), memory-shaped like the depthwise kernels (decoder.hip):
//   fwd / dgrad : a thread owns 8 consecutive channels of one pixel (one 16-B vector out); threads of a
//                 wave share the channel block and walk 64 consecutive pixels, so the weight reads are
//                 wave-uniform (broadcast) and the activation reads are one 16-B vector per lane per tap.
//                 CG <= 8: the 8 channels' groups are exactly the 8 input channels of the same block (one
//                 vector per tap); CG > 8: CG / 8 vectors of the group per tap.
//   wgrad       : a thread owns (tap, 8 output channels, 8 input channels of their group) = 64 fp32
//                 accumulators over a slice of the pixels; lanes are consecutive channel blocks of the
//                 same pixel (coalesced); per-slice partials [S][combos][64] are summed in slice order by
//                 colsum (bitwise deterministic).
// Weights are repacked fp32 [T][C][CG] (w[t][co][cil] = W[co][cil][kh][kw]).
#include <algorithm>

#include "common.h"
#include "launchers.h"

namespace {
constexpr int kBlock = 256;

struct GTaps { int T; int dy[kMaxTaps]; int dx[kMaxTaps]; };

int grid_for(long n) {
  long b = (n + kBlock - 1) / kBlock;
  if (b > (1L << 20)) b = 1L << 20;
  if (b < 1) b = 1;
  return (int)b;
}

// y[n, oy, ox, co] = sum_t sum_cil w[t][co][cil] * x[n, oy*s + dy_t, ox*s + dx_t, group(co)*CG + cil]
template <int CG>
__global__ __launch_bounds__(kBlock) void gconv_fwd_kernel(const uint16_t* __restrict__ x, const float* __restrict__ w,
                                                           uint16_t* __restrict__ y, int N, int IH, int IW, int OH,
                                                           int OW, int C, int stride, GTaps tp) {
  const long P = (long)N * OH * OW;
  const long total = P * (C >> 3);
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int cb = (int)(i / P);      // channel block (wave-uniform for P % 64 == 0)
    const long p = i - (long)cb * P;
    const int ox = (int)(p % OW);
    const long q = p / OW;
    const int oy = (int)(q % OH);
    const long n = q / OH;
    const int co0 = 8 * cb;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const uint16_t* xn = x + n * IH * IW * C;
    for (int t = 0; t < tp.T; ++t) {
      const int iy = oy * stride + tp.dy[t], ix = ox * stride + tp.dx[t];
      if ((unsigned)iy >= (unsigned)IH || (unsigned)ix >= (unsigned)IW) continue;
      const uint16_t* xp = xn + ((long)iy * IW + ix) * C;
      const float* wt = w + ((long)t * C + co0) * CG;
      if constexpr (CG <= 8) {
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(xp + co0), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int gb = (e / CG) * CG;
#pragma unroll
          for (int k = 0; k < CG; ++k) acc[e] = fmaf(wt[e * CG + k], v[gb + k], acc[e]);
        }
      } else {
        const int g0 = (co0 / CG) * CG;
#pragma unroll
        for (int vb = 0; vb < CG / 8; ++vb) {
          float v[8];
          unpack8(*reinterpret_cast<const uint4*>(xp + g0 + 8 * vb), v);
#pragma unroll
          for (int e = 0; e < 8; ++e)
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[e] = fmaf(wt[e * CG + 8 * vb + k], v[k], acc[e]);
        }
      }
    }
    *reinterpret_cast<uint4*>(y + p * C + co0) = pack8(acc);
  }
}

// dx[n, iy, ix, ci] = sum_t sum_{co in group(ci)} w[t][co][ci - g0] * dy[n, (iy - dy_t)/s, (ix - dx_t)/s, co]
template <int CG>
__global__ __launch_bounds__(kBlock) void gconv_dgrad_kernel(const uint16_t* __restrict__ dy, const float* __restrict__ w,
                                                             uint16_t* __restrict__ dx, int N, int IH, int IW, int OH,
                                                             int OW, int C, int stride, GTaps tp) {
  const long P = (long)N * IH * IW;
  const long total = P * (C >> 3);
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int cb = (int)(i / P);
    const long p = i - (long)cb * P;
    const int ix = (int)(p % IW);
    const long q = p / IW;
    const int iy = (int)(q % IH);
    const long n = q / IH;
    const int ci0 = 8 * cb;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const uint16_t* dn = dy + n * OH * OW * C;
    for (int t = 0; t < tp.T; ++t) {
      const int ry = iy - tp.dy[t], rx = ix - tp.dx[t];
      if (ry < 0 || rx < 0) continue;
      const int oy = ry / stride, ox = rx / stride;
      if (oy * stride != ry || ox * stride != rx || oy >= OH || ox >= OW) continue;
      const uint16_t* gp = dn + ((long)oy * OW + ox) * C;
      const float* wt = w + (long)t * C * CG;
      if constexpr (CG <= 8) {
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(gp + ci0), v);   // the same 8-channel block of outputs
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int gb = (e / CG) * CG;
#pragma unroll
          for (int k = 0; k < CG; ++k) acc[e] = fmaf(wt[(long)(ci0 + gb + k) * CG + (e - gb)], v[gb + k], acc[e]);
        }
      } else {
        const int g0 = (ci0 / CG) * CG, el = ci0 - g0;
#pragma unroll
        for (int vb = 0; vb < CG / 8; ++vb) {
          float v[8];
          unpack8(*reinterpret_cast<const uint4*>(gp + g0 + 8 * vb), v);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float* wr = wt + (long)(g0 + 8 * vb + k) * CG + el;
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = fmaf(wr[e], v[k], acc[e]);
          }
        }
      }
    }
    *reinterpret_cast<uint4*>(dx + p * C + ci0) = pack8(acc);
  }
}

// part[s][combo][64]: combo = (t, co block ob, input block ib of the group) -> acc[e][k] = sum over slice s
// of dy[p, 8*ob + e] * x[p*s + off_t, g0 + 8*ib + k] (CG < 8: k < CG, the input channels of e's group)
template <int CG>
__global__ __launch_bounds__(kBlock) void gconv_wgrad_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                             float* __restrict__ part, int N, int IH, int IW, int OH,
                                                             int OW, int C, int stride, GTaps tp, int nslice) {
  constexpr int NIB = CG >= 8 ? CG / 8 : 1;
  const int nob = C >> 3;
  const int ncombo = tp.T * nob * NIB;
  const int combo = blockIdx.x * kBlock + threadIdx.x;
  const int s = blockIdx.y;
  if (combo >= ncombo) return;
  const int t = combo / (nob * NIB);
  const int r = combo - t * nob * NIB;
  const int ib = r / nob, ob = r - ib * nob;   // lanes: consecutive output blocks (coalesced channel reads)
  const int co0 = 8 * ob;
  const int g0 = (co0 / CG) * CG;
  const int xc0 = CG >= 8 ? g0 + 8 * ib : co0;   // CG < 8: the 8-channel block holding e's groups
  float acc[8][8];
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[e][k] = 0.f;
  const long P = (long)N * OH * OW;
  const long per = (P + nslice - 1) / nslice;
  const long p0 = (long)s * per, p1 = p0 + per < P ? p0 + per : P;
  for (long p = p0; p < p1; ++p) {
    const int ox = (int)(p % OW);
    const long q = p / OW;
    const int oy = (int)(q % OH);
    const long n = q / OH;
    const int iy = oy * stride + tp.dy[t], ix = ox * stride + tp.dx[t];
    if ((unsigned)iy >= (unsigned)IH || (unsigned)ix >= (unsigned)IW) continue;
    float g[8], v[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + p * C + co0), g);
    unpack8(*reinterpret_cast<const uint4*>(x + ((n * IH + iy) * IW + ix) * C + xc0), v);
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[e][k] = fmaf(g[e], v[k], acc[e][k]);
  }
  float* o = part + ((long)s * ncombo + combo) * 64;
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int k = 0; k < 8; k += 4)
      *reinterpret_cast<float4*>(o + e * 8 + k) = make_float4(acc[e][k], acc[e][k + 1], acc[e][k + 2], acc[e][k + 3]);
}

// ---- MFMA path (round 5): forward and data-gradient on the matrix cores ----------------------------------
// The grouped conv as a dense GEMM over a KW-channel window (KW = max(16, CG): the 16-output-channel block
// of an MFMA tile reads exactly that window) with BLOCK-DIAGONAL weights -- the off-group entries are zero
// and cost MFMA cycles only, which the short per-group reduction (CG x 9 = 36..576) leaves to spare: the
// VALU kernels above were compute-bound at ~14 TFLOP/s (profiles/r04/kernels_smp_unet_resnext50_bs64.txt).
// One wave = one 16-channel output block x NCH chunks of 16 pixels; v_mfma_f32_16x16x32_bf16 with
//   A = weights [16 out][32 k] (k = tap * KW + window channel; pre-packed per lane by ops/gconv.py),
//   B = activations [32 k][16 px]: lane l loads pixel l % 16, k-slot l / 16 = 8 window channels of one tap,
//       ONE 16-B global vector (NHWC), zero outside the image / for the padding taps,
//   D = [16 out][16 px]: lane l holds 4 consecutive channels of pixel l % 16 -> one 8-B store.
// TRANS: the data-gradient (output pixels are input-space pixels; tap t reads dY at (p - d_t) / stride where
// that divides exactly).  Weights stay in VGPRs (NST x 4) across the wave's chunks.
constexpr int kGmT = 9;
constexpr int kGmNch = 4;

template <int KW, bool TRANS>
__global__ __launch_bounds__(256) void gconv_mfma_kernel(const uint16_t* __restrict__ x, const uint4* __restrict__ wpk,
                                                         uint16_t* __restrict__ y, int N, int IH, int IW, int OH,
                                                         int OW, int C, int stride, GTaps tp) {
  constexpr int NST = (kGmT * KW + 31) / 32;
  const int lane = threadIdx.x & 63, q = lane >> 4, pl = lane & 15;
  const int nob = C >> 4;
  const long gw = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int ob = (int)(gw % nob);
  const long pc = gw / nob;
  // output / source geometry: fwd reads x [N, IH, IW] for outputs [N, OH, OW]; TRANS reads dY [N, OH, OW]
  // for outputs dX [N, IH, IW]
  const int PH = TRANS ? IH : OH, PW = TRANS ? IW : OW, SH = TRANS ? OH : IH, SW = TRANS ? OW : IW;
  const long P = (long)N * PH * PW;
  if (pc * 16 * kGmNch >= P) return;
  const int co0 = 16 * ob, g0w = (co0 / KW) * KW;
  uint4 a[NST];
#pragma unroll
  for (int s = 0; s < NST; ++s) a[s] = wpk[((long)ob * NST + s) * 64 + lane];
#pragma unroll 1
  for (int ch = 0; ch < kGmNch; ++ch) {
    const long p = (pc * kGmNch + ch) * 16 + pl;
    const bool pin = p < P;
    const long pp = pin ? p : 0;
    const int ox = (int)(pp % PW);
    const long r = pp / PW;
    const int oy = (int)(r % PH);
    const long n = r / PH;
    const uint16_t* src = x + n * SH * SW * C + g0w;
    uint4 b[NST];
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      const int k0 = 32 * s + 8 * q;
      const int tap = k0 / KW, cl = k0 % KW;
      const int tA = (32 * s) / KW;
      const int tB = tA + 1 < kGmT ? tA + 1 : kGmT - 1;
      const int ddy = tap == tA ? tp.dy[tA < kGmT ? tA : kGmT - 1] : tp.dy[tB];
      const int ddx = tap == tA ? tp.dx[tA < kGmT ? tA : kGmT - 1] : tp.dx[tB];
      bool ok = pin && tap < kGmT;
      int sy, sx;
      if (!TRANS) {
        sy = oy * stride + ddy;
        sx = ox * stride + ddx;
      } else {
        const int ry = oy - ddy, rx = ox - ddx;
        sy = ry / stride;
        sx = rx / stride;
        ok = ok && ry >= 0 && rx >= 0 && sy * stride == ry && sx * stride == rx;
      }
      ok = ok && (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW;
      b[s] = ok ? *reinterpret_cast<const uint4*>(src + ((long)sy * SW + sx) * C + cl) : make_uint4(0, 0, 0, 0);
    }
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NST; ++s) acc = mfma16x16x32(a[s], b[s], acc);
    if (pin) {
      uint2 o;
      o.x = pack2(acc[0], acc[1]);
      o.y = pack2(acc[2], acc[3]);
      *reinterpret_cast<uint2*>(y + p * C + co0 + 4 * q) = o;
    }
  }
}

// Weight gradient on MFMA: dW_blk[16 co][tap][KW window ch] = sum_p dY[p][co] * X[src(p, tap)][window ch]
// (K = pixels; the block-diagonal entries are extracted on the host side, ops/gconv.py).  Block = one
// 16-co block x one pixel slice; 64-pixel stages of dY [64][16] and the 9 gathered tap rows X_t [64][KW]
// go through LDS in their NHWC row layout and feed the MFMA with ds_read_b64_tr_b16 (the transposed read:
// a lane addresses 4 channels of one pixel, the 16-lane group receives 4 pixels per channel).  The next
// stage's global loads are in flight during the current stage's MFMAs.  The 9*KW/16 output tiles are dealt
// to the 4 waves; each slice writes its partial tiles to part[slice] (summed in slice order by colsum).
typedef short s16x4_t __attribute__((ext_vector_type(4)));
DEVI uint2 gm_tr_read(const uint16_t* p) {
  s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t __attribute__((address_space(3)))*)(p));
  union { s16x4_t s; uint2 u; } c; c.s = v; return c.u;
}

constexpr int kGwPx = 64;   // pixels per stage (KW <= 32)

template <int KW>
__global__ __launch_bounds__(256) void gconv_wgrad_mfma_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                               float* __restrict__ part, int N, int IH, int IW, int OH,
                                                               int OW, int C, int stride, GTaps tp, long per) {
  constexpr int NPX = KW == 64 ? 32 : kGwPx;      // pixels per stage (KW 64: the 9 tap rows fit 40 KB)
  constexpr int NTI = kGmT * KW / 16;            // output tiles (tap, 16-ch sub-block of the window)
  constexpr int TPW = (NTI + 3) / 4;             // tiles per wave
  constexpr int PY = 16 + 4, PX = KW + 4;        // LDS row pitches (elements; 8-B aligned rows)
  constexpr int XV = KW / 8;                     // 16-B vectors per X row
  constexpr int NXS = (kGmT * NPX * XV + 255) / 256;   // X staging vectors per thread
  __shared__ __attribute__((aligned(16))) uint16_t sY[NPX * PY];
  __shared__ __attribute__((aligned(16))) uint16_t sX[kGmT * NPX * PX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4, q = lr >> 2, p4 = lr & 3;
  const int ob = blockIdx.y, co0 = 16 * ob, g0w = (co0 / KW) * KW;
  const long P = (long)N * OH * OW;
  const long p0 = (long)blockIdx.x * per, p1 = p0 + per < P ? p0 + per : P;
  const int nstage = p1 > p0 ? (int)((p1 - p0 + NPX - 1) / NPX) : 0;

  uint4 vy = make_uint4(0, 0, 0, 0);
  uint4 vx[NXS];
  auto load = [&](int st) {
    const long pb = p0 + (long)st * NPX;
    if (tid < 2 * NPX) {   // dY: NPX px x 2 vectors
      const long p = pb + (tid >> 1);
      vy = p < p1 ? *reinterpret_cast<const uint4*>(dy + p * C + co0 + 8 * (tid & 1)) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < NXS; ++u) {
      const int e = tid + 256 * u;   // (tap, px, vec)
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < kGmT * NPX * XV) {
        const int t = e / (NPX * XV), r = e - t * (NPX * XV), px = r / XV, vv = r - px * XV;
        const long p = pb + px;
        if (p < p1) {
          const int ox = (int)(p % OW);
          const long rr = p / OW;
          const int oy = (int)(rr % OH);
          const long n = rr / OH;
          const int iy = oy * stride + tp.dy[t < kGmT ? t : 0], ix = ox * stride + tp.dx[t < kGmT ? t : 0];
          if ((unsigned)iy < (unsigned)IH && (unsigned)ix < (unsigned)IW)
            v = *reinterpret_cast<const uint4*>(x + ((n * IH + iy) * IW + ix) * C + g0w + 8 * vv);
        }
      }
      vx[u] = v;
    }
  };
  auto store = [&]() {
    if (tid < 2 * NPX) {   // 8-B aligned rows: two 8-B halves
      uint2* d = reinterpret_cast<uint2*>(&sY[(tid >> 1) * PY + 8 * (tid & 1)]);
      d[0] = make_uint2(vy.x, vy.y);
      d[1] = make_uint2(vy.z, vy.w);
    }
#pragma unroll
    for (int u = 0; u < NXS; ++u) {
      const int e = tid + 256 * u;
      if (e < kGmT * NPX * XV) {
        const int t = e / (NPX * XV), r = e - t * (NPX * XV), px = r / XV, vv = r - px * XV;
        // two 8-B halves: PX rows are 8-B (not 16-B) aligned
        uint2* d = reinterpret_cast<uint2*>(&sX[(t * NPX + px) * PX + 8 * vv]);
        d[0] = make_uint2(vx[u].x, vx[u].y);
        d[1] = make_uint2(vx[u].z, vx[u].w);
      }
    }
  };

  f32x4_t acc[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // per-lane transposed-read offsets within a 32-pixel k-step: pixels 8*lg + q (lo) and + 4 (hi), channels 4*p4
  const int offYlo = (8 * lg + q) * PY + 4 * p4, offYhi = offYlo + 4 * PY;
  int offX[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int ti = wave + 4 * j < NTI ? wave + 4 * j : 0;
    const int t = ti / (KW / 16), c16 = ti % (KW / 16);
    offX[j] = (t * NPX + 8 * lg + q) * PX + 16 * c16 + 4 * p4;
  }
  if (nstage > 0) load(0);
  for (int st = 0; st < nstage; ++st) {
    __syncthreads();
    store();
    __syncthreads();
    if (st + 1 < nstage) load(st + 1);
#pragma unroll
    for (int ks = 0; ks < NPX / 32; ++ks) {
      const uint2 alo = gm_tr_read(&sY[ks * 32 * PY + offYlo]);
      const uint2 ahi = gm_tr_read(&sY[ks * 32 * PY + offYhi]);
      const uint4 a = make_uint4(alo.x, alo.y, ahi.x, ahi.y);
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const uint2 blo = gm_tr_read(&sX[ks * 32 * PX + offX[j]]);
        const uint2 bhi = gm_tr_read(&sX[ks * 32 * PX + offX[j] + 4 * PX]);
        acc[j] = mfma16x16x32(a, make_uint4(blo.x, blo.y, bhi.x, bhi.y), acc[j]);
      }
    }
  }
  // part[slice][ob][tile][16 co][16 ch]; D row (co) = 4*lg + r, column (ch) = lr
  float* o = part + ((long)blockIdx.x * gridDim.y + ob) * NTI * 256;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int ti = wave + 4 * j;
    if (ti >= NTI) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[ti * 256 + (4 * lg + r) * 16 + lr] = acc[j][r];
  }
}

GTaps make_taps(int T, const int* dyv, const int* dxv) {
  GTaps tp{};
  tp.T = T;
  for (int t = 0; t < T; ++t) { tp.dy[t] = dyv[t]; tp.dx[t] = dxv[t]; }
  return tp;
}
}  // namespace

int gconv_wgrad_slices(long P, int C, int CG, int T) {
  const int nib = CG >= 8 ? CG / 8 : 1;
  const long combos = (long)T * (C / 8) * nib;
  const long cblocks = (combos + kBlock - 1) / kBlock;
  long s = (2048 + cblocks - 1) / cblocks;            // ~2048 blocks
  s = std::min(s, std::max(1L, P / 256));             // >= 256 pixels per slice
  return (int)std::max(1L, std::min(s, 1024L));
}

#define GC_DISPATCH_(KERN, ...)                                                                            \
  switch (CG) {                                                                                           \
    case 1: hipLaunchKernelGGL(KERN<1>, __VA_ARGS__); return 0;                                           \
    case 2: hipLaunchKernelGGL(KERN<2>, __VA_ARGS__); return 0;                                           \
    case 4: hipLaunchKernelGGL(KERN<4>, __VA_ARGS__); return 0;                                           \
    case 8: hipLaunchKernelGGL(KERN<8>, __VA_ARGS__); return 0;                                           \
    case 16: hipLaunchKernelGGL(KERN<16>, __VA_ARGS__); return 0;                                         \
    case 32: hipLaunchKernelGGL(KERN<32>, __VA_ARGS__); return 0;                                         \
    case 64: hipLaunchKernelGGL(KERN<64>, __VA_ARGS__); return 0;                                         \
  }                                                                                                       \
  return 1;

int gconv_fwd(const uint16_t* x, const float* w, uint16_t* y, int N, int IH, int IW, int OH, int OW, int C, int CG,
              int stride, int T, const int* dyv, const int* dxv, hipStream_t s) {
  const GTaps tp = make_taps(T, dyv, dxv);
  const dim3 grid(grid_for((long)N * OH * OW * (C / 8)));
  GC_DISPATCH_(gconv_fwd_kernel, grid, dim3(kBlock), 0, s, x, w, y, N, IH, IW, OH, OW, C, stride, tp)
}

int gconv_dgrad(const uint16_t* dy, const float* w, uint16_t* dx, int N, int IH, int IW, int OH, int OW, int C, int CG,
                int stride, int T, const int* dyv, const int* dxv, hipStream_t s) {
  const GTaps tp = make_taps(T, dyv, dxv);
  const dim3 grid(grid_for((long)N * IH * IW * (C / 8)));
  GC_DISPATCH_(gconv_dgrad_kernel, grid, dim3(kBlock), 0, s, dy, w, dx, N, IH, IW, OH, OW, C, stride, tp)
}

int gconv_wgrad(const uint16_t* x, const uint16_t* dy, float* part, int nslice, int N, int IH, int IW, int OH, int OW,
                int C, int CG, int stride, int T, const int* dyv, const int* dxv, hipStream_t s) {
  const GTaps tp = make_taps(T, dyv, dxv);
  const int nib = CG >= 8 ? CG / 8 : 1;
  const int combos = T * (C / 8) * nib;
  const dim3 grid((unsigned)((combos + kBlock - 1) / kBlock), (unsigned)nslice);
  GC_DISPATCH_(gconv_wgrad_kernel, grid, dim3(kBlock), 0, s, x, dy, part, N, IH, IW, OH, OW, C, stride, tp, nslice)
}
#undef GC_DISPATCH_

// wpk: [C/16][NST][64 lanes] uint4 (ops/gconv.py _mfma_pack); KW = max(16, CG); TRANS: the data-gradient
// (x = dY [N, OH, OW, C], y = dX [N, IH, IW, C]).  Returns 1 when no instantiation fits (caller falls back).
int gconv_mfma(const uint16_t* x, const uint16_t* wpk, uint16_t* y, int N, int IH, int IW, int OH, int OW, int C,
               int KW, int stride, bool trans, int T, const int* dyv, const int* dxv, hipStream_t s) {
  if (T != kGmT || C % 16 != 0) return 1;
  const GTaps tp = make_taps(T, dyv, dxv);
  const long P = trans ? (long)N * IH * IW : (long)N * OH * OW;
  const long waves = (long)(C / 16) * ((P + 16 * kGmNch - 1) / (16 * kGmNch));
  const dim3 grid((unsigned)((waves + 3) / 4));
  const uint4* w = reinterpret_cast<const uint4*>(wpk);
#define GM_(KWV, TR) hipLaunchKernelGGL((gconv_mfma_kernel<KWV, TR>), grid, dim3(256), 0, s, x, w, y, N, IH, IW, OH, OW, C, stride, tp)
  switch (KW) {
    case 16: if (trans) GM_(16, true); else GM_(16, false); return 0;
    case 32: if (trans) GM_(32, true); else GM_(32, false); return 0;
    case 64: if (trans) GM_(64, true); else GM_(64, false); return 0;
  }
#undef GM_
  return 1;
}

// part [nslice][C/16][9*KW/16][16][16] fp32 (summed over slices by colsum; the block diagonal is extracted by
// ops/gconv.py).  3x3, C % 16 == 0, KW = max(16, CG) in {16, 32, 64}.
int gconv_wgrad_mfma_slices(long P, int C) {
  long s = std::max(1L, 1024L / std::max(1, C / 16));
  s = std::min(s, std::max(1L, P / 256));   // >= 4 stages per slice
  return (int)std::max(1L, std::min(s, 1024L));
}

int gconv_wgrad_mfma(const uint16_t* x, const uint16_t* dy, float* part, int nslice, int N, int IH, int IW, int OH,
                     int OW, int C, int KW, int stride, int T, const int* dyv, const int* dxv, hipStream_t s) {
  if (T != kGmT || C % 16 != 0) return 1;
  const GTaps tp = make_taps(T, dyv, dxv);
  const long P = (long)N * OH * OW;
  const long per = (P + nslice - 1) / nslice;
  const dim3 grid((unsigned)nslice, (unsigned)(C / 16));
  switch (KW) {
    case 16: hipLaunchKernelGGL((gconv_wgrad_mfma_kernel<16>), grid, dim3(256), 0, s, x, dy, part, N, IH, IW, OH, OW, C, stride, tp, per); return 0;
    case 32: hipLaunchKernelGGL((gconv_wgrad_mfma_kernel<32>), grid, dim3(256), 0, s, x, dy, part, N, IH, IW, OH, OW, C, stride, tp, per); return 0;
    case 64: hipLaunchKernelGGL((gconv_wgrad_mfma_kernel<64>), grid, dim3(256), 0, s, x, dy, part, N, IH, IW, OH, OW, C, stride, tp, per); return 0;
  }
  return 1;
}
