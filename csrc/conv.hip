// Implicit-GEMM convolution for CDNA4 (gfx950): forward, data-gradient and weight-gradient, NHWC bf16
// activations with fp32 accumulation on v_mfma_f32_16x16x32_bf16.
//
// Replaces every cuDNN/MIOpen convolution the reference dispatches:
//   3x3 d1/d2/d3 (models/ducknet.py:95-96,160-170), 1x7/7x1 (ducknet.py:177-178), 1x1
//   (ducknet.py:93, heads), 3x3 s2 and 2x2 s2 (ducknet.py:60-61), and the UNet transposed conv
//   (models/modules.py:99-102) which is exactly the data-gradient of a strided conv.
//
// GEMM view (one kernel family for all of them):
//     D[co][m] = sum_k  Wp[co][k] * Xcol[k][m]        m = output pixel (n, oh, ow), k = t*Cip + ci
// A operand = packed weights Wp[co][k] (8 consecutive k are contiguous -> one 16-B load per lane).
// B operand = the im2col column of pixel m; in NHWC the 8 consecutive k of a lane are 8 consecutive
// channels of ONE shifted input pixel -> one aligned 16-B load per lane, no transpose needed.
// Taps are an explicit (dy, dx) offset table, so dilation, asymmetric kernels (1x7), the 1x1 centre
// tap of horizontally fused convs and the flipped taps of the data-gradient are the same code.
// Output layout of the 16x16x32 tile: lane holds rows 4*(lane>>4)+r (= 4 consecutive co) of column
// lane&15 (= one pixel) -> 8-B NHWC stores.
//
// "TRANS" mode maps output pixel o to input pixel (o + d) / stride when divisible: the data-gradient
// of a stride-s conv, and the forward of ConvTranspose2d.
// Channel GROUPS (launchers.h): the logical input/output channel dims may be split over up to 8
// separate NHWC tensors; group pointers are staged in LDS and selected per lane per k-step.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "launchers.h"

namespace {

// Per-lane position in the flattened K = (tap, input group, channel) walk, advanced 32 at a time.
struct KPos { int t, gi, cl; };

DEVI KPos kpos_init(int kg, const ConvGeom& g) {
  const int Cip = g.Gi * g.Cgi;
  KPos p;
  p.t = kg / Cip;
  const int rem = kg - p.t * Cip;
  p.gi = rem / g.Cgi;
  p.cl = rem - p.gi * g.Cgi;
  return p;
}

DEVI void kpos_advance(KPos& p, int by, const ConvGeom& g) {
  p.cl += by;
  while (p.cl >= g.Cgi) {
    p.cl -= g.Cgi;
    if (++p.gi == g.Gi) { p.gi = 0; ++p.t; }
  }
}

// Maps output pixel (ph, pw) [already multiplied by stride in fwd mode] + tap offset to an input
// pixel index, or -1 when the tap falls in the zero padding / is not stride-aligned.
template <bool TRANS>
DEVI int in_pixel(int pn, int ph, int pw, int2 d, const ConvGeom& g) {
  if (!TRANS) {
    const int ih = ph + d.x, iw = pw + d.y;
    if ((unsigned)ih < (unsigned)g.IH && (unsigned)iw < (unsigned)g.IW) return pn + ih * g.IW + iw;
    return -1;
  } else {
    const int a = ph + d.x, b = pw + d.y;
    if (a < 0 || b < 0) return -1;
    const int ih = a / g.stride, iw = b / g.stride;
    if (ih * g.stride != a || iw * g.stride != b || ih >= g.IH || iw >= g.IW) return -1;
    return pn + ih * g.IW + iw;
  }
}

// Output-phase decomposition of a strided TRANS conv (data-gradient of a stride-s conv, forward of
// ConvTranspose2d): output pixels with (oh % s, ow % s) == (py, px) only see the taps t with
// (py + dy[t]) % s == 0 and (px + dx[t]) % s == 0, and for those the input pixel is
// (oh / s + qy[t], ow / s + qx[t]) with qy = (py + dy) / s exact -- a plain stride-1 gather over a
// (OH/s x OW/s) sub-grid.  The host launches one grid per phase with the reduced tap table (qy, qx)
// in g.dy/g.dx and tA[] = the taps' positions in the packed weight rows, so the K loop covers only
// the Tv valid taps (a 3x3 s2 data-gradient does 2.25 of 9 taps' work on average, not 9).
struct PhaseArgs { int s, py, px, OHp, OWp, Kloop; int tA[kMaxTaps]; };

// 16-B load through a pointer the compiler cannot prove global (read back from LDS, or a
// by-value struct member): a global_load,
// not a FLAT load (FLAT also counts in lgkmcnt, so LDS waits would drain it)
// (through an integer: an addrspacecast of the generic pointer is folded back into a FLAT load)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
DEVI uint4 ldg4(const uint16_t* p) {
  const u32x4_t v =
      *reinterpret_cast<const __attribute__((address_space(1))) u32x4_t*>(reinterpret_cast<uintptr_t>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
// 8-B global load / store through a pointer read back from LDS (the igemm epilogue's s_y table)
DEVI uint2 ldg2(const uint16_t* p) {
  const u32x2_t v =
      *reinterpret_cast<const __attribute__((address_space(1))) u32x2_t*>(reinterpret_cast<uintptr_t>(p));
  return make_uint2(v.x, v.y);
}
DEVI void stg2(uint16_t* p, uint2 v) {
  u32x2_t w;
  w.x = v.x; w.y = v.y;
  *reinterpret_cast<__attribute__((address_space(1))) u32x2_t*>(reinterpret_cast<uintptr_t>(p)) = w;
}
// load8f through a global-memory pointer read back from LDS (the s_xc table)
DEVI void load8f_g(const float* p, float* d) {
  const uint4 a = ldg4(reinterpret_cast<const uint16_t*>(p)), b = ldg4(reinterpret_cast<const uint16_t*>(p + 4));
  d[0] = __uint_as_float(a.x); d[1] = __uint_as_float(a.y); d[2] = __uint_as_float(a.z); d[3] = __uint_as_float(a.w);
  d[4] = __uint_as_float(b.x); d[5] = __uint_as_float(b.y); d[6] = __uint_as_float(b.z); d[7] = __uint_as_float(b.w);
}

template <int MI, int NJ, int WPX, bool TRANS, bool PH = false, bool BNE = false>
__global__ __launch_bounds__(64 * WPX) void conv_igemm_kernel(ConvArgs a, PhaseArgs pa) {
  const ConvGeom& g = a.g;
  __shared__ int2 s_tap[kMaxTaps];
  __shared__ int s_ta[PH ? kMaxTaps : 1];
  __shared__ const uint16_t* s_x[kMaxGroups];
  __shared__ uint16_t* s_y[kMaxGroups];
  __shared__ const float* s_xc[kMaxGroups];
  __shared__ float s_stat[WPX][2][16 * MI];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < kMaxTaps) s_tap[tid] = make_int2(g.dy[tid], g.dx[tid]);
  if (PH && tid < kMaxTaps) s_ta[tid] = pa.tA[tid];
  if (tid < kMaxGroups) { s_x[tid] = a.x[tid]; s_y[tid] = a.y[tid]; s_xc[tid] = a.xc[tid]; }
  __syncthreads();

  const long OHW = PH ? (long)pa.OHp * pa.OWp : (long)g.OH * g.OW;
  const long M = (long)g.N * OHW;
  const int Kloop = PH ? pa.Kloop : g.Kp;
  const int rows = g.Go * g.Cgo;
  // 1-D grid, XCD-aware: blocks sharing a pixel tile (all co tiles of it) get consecutive logical
  // ids placed on ONE XCD (bijective remap of the round-robin dispatch, guide T1), so the input
  // tile is fetched into that XCD's L2 once and re-read from there by the other co tiles.
  const int n_co = (rows + 16 * MI - 1) / (16 * MI);
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xq = nwg / 8, xr = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + orig / 8;
  const int co_t = wgid % n_co;
  const long px_t = wgid / n_co;
  const long m0 = (px_t * WPX + wave) * (16 * NJ);
  const int co0 = co_t * (16 * MI);
  const int lr = lane & 15, lg = lane >> 4;
  const int IHW = g.IH * g.IW;

  int pn[NJ], ph[NJ], pw[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const long m = m0 + 16 * j + lr;
    if (m < M) {
      const int n = (int)(m / OHW);
      const int r = (int)(m - (long)n * OHW);
      const int RW = PH ? pa.OWp : g.OW;   // PH: (oh, ow) index the phase sub-grid
      const int oh = r / RW, ow = r - (r / RW) * RW;
      pn[j] = n * IHW;
      ph[j] = (TRANS || PH) ? oh : oh * g.stride;
      pw[j] = (TRANS || PH) ? ow : ow * g.stride;
    } else {
      pn[j] = -1; ph[j] = 0; pw[j] = 0;
    }
  }
  const uint16_t* wrow[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) wrow[i] = a.w + (long)(co0 + 16 * i + lr) * g.Kp + (PH ? 0 : 8 * lg);

  KPos kp = kpos_init(8 * lg, g);

  // returns the NJ-bit mask of the in-image (actually loaded) pixels: the deferred-BN prologue
  // (xform_b, applied once the loads have landed) must leave the zero padding at 0
  auto load_b = [&](uint4* B, const KPos& p) -> unsigned {
    const bool kval = p.t < g.T;
    const int2 d = kval ? s_tap[p.t] : make_int2(0, 0);
    const uint16_t* xb = s_x[kval ? p.gi : 0] + p.cl;
    unsigned ok = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (pn[j] >= 0 && kval) {
        const int pix = in_pixel<TRANS>(pn[j], ph[j], pw[j], d, g);
        if (pix >= 0) { v = ldg4(xb + (long)pix * g.Cgi); ok |= 1u << j; }
      }
      B[j] = v;
    }
    return ok;
  };
  // the prologue coefficients of a k-step are fetched together with its B loads (so their latency
  // hides under the same MFMAs); returns 0 (no prologue), 1 (affine) or 3 (affine + ReLU)
  auto load_coef = [&](const KPos& p, float* sc, float* sh) -> int {
    if (PH || p.t >= g.T) return 0;
    const float* cf = s_xc[p.gi];
    if (cf == nullptr) return 0;
    load8f_g(cf + p.cl, sc);
    load8f_g(cf + g.Cgi + p.cl, sh);
    return 1 | (int)(((a.xrelu >> p.gi) & 1u) << 1);
  };
  auto xform_b = [&](uint4* B, unsigned ok, int mode, const float* sc, const float* sh) {
    if (mode == 0) return;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      if ((ok >> j) & 1u) B[j] = affine8(B[j], sc, sh, mode == 3);
  };
  auto load_a = [&](uint4* A, int k0, const KPos& p) {
    if (PH) {   // the lane's 8 k sit at tap s_ta[t] of the full packed row (zero past the valid taps)
      const int off = p.t < g.T ? s_ta[p.t] * (g.Gi * g.Cgi) + p.gi * g.Cgi + p.cl : -1;
#pragma unroll
      for (int i = 0; i < MI; ++i)
        A[i] = off >= 0 ? ldg4(wrow[i] + off) : make_uint4(0, 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < MI; ++i) A[i] = ldg4(wrow[i] + k0);
    }
  };

  f32x4_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 A[MI], B[NJ];
  float csc[8], csh[8];
  load_a(A, 0, kp);
  {
    const unsigned ok0 = load_b(B, kp);
    const int m0 = load_coef(kp, csc, csh);
    xform_b(B, ok0, m0, csc, csh);
  }
  for (int k0 = 0; k0 < Kloop; k0 += 32) {
    uint4 An[MI], Bn[NJ];
    unsigned okn = 0;
    int mode = 0;
    const bool more = k0 + 32 < Kloop;
    if (more) {
      kpos_advance(kp, 32, g);
      load_a(An, k0 + 32, kp);
      okn = load_b(Bn, kp);
      mode = load_coef(kp, csc, csh);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16x16x32(A[i], B[j], acc[i][j]);
    if (more) {
      xform_b(Bn, okn, mode, csc, csh);   // after the MFMAs: the prefetch stays in flight under them
#pragma unroll
      for (int i = 0; i < MI; ++i) A[i] = An[i];
#pragma unroll
      for (int j = 0; j < NJ; ++j) B[j] = Bn[j];
    }
  }

  // Epilogue: bias, bf16 pack, 8-B NHWC stores into the row's output group; optional per-channel
  // (sum, sum^2) partials of the stored (bf16-rounded) values for the BatchNorm that follows.
  float csum[MI][4], csq[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) { csum[i][r] = 0.f; csq[i][r] = 0.f; }
    const int cb = co0 + 16 * i + 4 * lg;
    if (cb >= rows) continue;
    const int og = cb / g.Cgo, cl = cb - (cb / g.Cgo) * g.Cgo;
    uint16_t* yb = s_y[og] + cl;
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = (a.bias != nullptr && cl + r < g.Cgo_l) ? a.bias[cl + r] : 0.f;
    uint2 ypre[BNE ? NJ : 1];
    if constexpr (BNE) {   // non-PH stride-1 data-gradient: output pixel index == m
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const long m = m0 + 16 * j + lr;
        ypre[j] = m < M ? *reinterpret_cast<const uint2*>(a.bn_y + m * g.Cgo + cb) : make_uint2(0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const long m = m0 + 16 * j + lr;
      if (m < M) {
        long mo = m;   // output pixel index
        if (PH) {
          const long n = m / OHW;
          const int r = (int)(m - n * OHW);
          const int qa = r / pa.OWp, qb = r - qa * pa.OWp;
          mo = (n * g.OH + (long)qa * pa.s + pa.py) * g.OW + (long)qb * pa.s + pa.px;
        }
        float v[4];
        float old[4] = {0.f, 0.f, 0.f, 0.f};
        if (!BNE && a.accum) {   // y += conv(x): add the stored bf16 output (sibling launches' dgrads)
          const uint2 ov = ldg2(yb + mo * g.Cgo);
          old[0] = __uint_as_float(ov.x << 16); old[1] = __uint_as_float(ov.x & 0xffff0000u);
          old[2] = __uint_as_float(ov.y << 16); old[3] = __uint_as_float(ov.y & 0xffff0000u);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float o = (cl + r < g.Cgo_l) ? acc[i][j][r] + bv[r] + old[r] : 0.f;
          v[r] = bf2f(f2bf(o));
        }
        if constexpr (BNE) {   // BN-backward partials (Go == 1: cl == cb); y prefetched per row group
          const float4 sc = *reinterpret_cast<const float4*>(a.bn_coef + cb);
          const float4 sh = *reinterpret_cast<const float4*>(a.bn_coef + g.Cgo + cb);
          const float4 mu = *reinterpret_cast<const float4*>(a.bn_coef + 2 * g.Cgo + cb);
          const uint2 yy = ypre[j];
          const float y4[4] = {__uint_as_float(yy.x << 16), __uint_as_float(yy.x & 0xffff0000u),
                               __uint_as_float(yy.y << 16), __uint_as_float(yy.y & 0xffff0000u)};
          const float s4[4] = {sc.x, sc.y, sc.z, sc.w}, h4[4] = {sh.x, sh.y, sh.z, sh.w}, m4[4] = {mu.x, mu.y, mu.z, mu.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gr = (!a.bn_relu || fmaf(y4[r], s4[r], h4[r]) > 0.f) ? v[r] : 0.f;
            csum[i][r] += gr;
            csq[i][r] += gr * (y4[r] - m4[r]);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            csum[i][r] += v[r];
            csq[i][r] += v[r] * v[r];
          }
        }
        stg2(yb + mo * g.Cgo, make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3])));
      }
    }
  }
  if (a.stat_part != nullptr) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = csum[i][r], q = csq[i][r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
        if (lr == 0) { s_stat[wave][0][16 * i + 4 * lg + r] = s; s_stat[wave][1][16 * i + 4 * lg + r] = q; }
      }
    __syncthreads();
    const long blk = px_t;
    for (int c = tid; c < 16 * MI; c += 64 * WPX) {
      const int co = co0 + c;
      if (co < rows) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int wv = 0; wv < WPX; ++wv) { s += s_stat[wv][0][c]; q += s_stat[wv][1][c]; }
        a.stat_part[(blk * 2 + 0) * rows + co] = s;
        a.stat_part[(blk * 2 + 1) * rows + co] = q;
      }
    }
  }
}

// Weight gradient: dW[co][k] = sum_m dY[m][co] * Xcol[k][m].  The reduction runs over pixels, so
// both operands need 8 consecutive PIXELS per lane: the block stages a 128-pixel chunk of dY
// ([128][CO_T]) and of the gathered im2col rows ([128][K_T]) in LDS in their natural NHWC row
// layout and feeds the MFMA with ds_read_b64_tr_b16 (hardware transpose read, CDNA4).  The next
// chunk's global loads are issued into registers before the current chunk's MFMAs (register
// double-buffering).  Each of the 4 waves reduces 32 pixels of a chunk; the waves' partial tiles are
// summed through LDS; each pixel split writes its own fp32 slab, summed in fixed order by unpack_wgrad.
constexpr int WG_M = 128;

typedef short s16x4_t __attribute__((ext_vector_type(4)));

DEVI uint2 tr_read(const uint16_t* p) {
  s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t __attribute__((address_space(3)))*)(p));
  union { s16x4_t s; uint2 u; } c; c.s = v; return c.u;
}


template <int CO_T, int K_T, bool TRANS>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradPtrs P, float* __restrict__ dw, ConvGeom g, int KT) {
  constexpr int SA_LD = CO_T + 8, SB_LD = K_T + 8;
  constexpr int A_CG = CO_T / 8, B_CG = K_T / 8;          // 16-B vectors per row
  constexpr int A_RS = 256 / A_CG, B_RS = 256 / B_CG;     // row stride between a thread's vectors
  constexpr int A_V = WG_M / A_RS, B_V = WG_M / B_RS;     // vectors per thread
  constexpr int FI = CO_T / 16, FJ = K_T / 16;
  constexpr int LDS_BYTES = WG_M * (SA_LD + SB_LD) * 2;
  static_assert(LDS_BYTES >= CO_T * K_T * 4, "reduction buffer must fit in the staging LDS");
  __shared__ __attribute__((aligned(16))) uint16_t smem[WG_M * (SA_LD + SB_LD)];
  uint16_t* sA = smem;
  uint16_t* sB = smem + WG_M * SA_LD;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k0 = blockIdx.x * K_T;
  const int co0 = blockIdx.y * CO_T;
  const int rows = g.Go * g.Cgo;
  const long OHW = (long)g.OH * g.OW;
  const long M = (long)g.N * OHW;
  const long nchunks = (M + WG_M - 1) / WG_M;

  const int a_c8 = tid % A_CG, a_r = tid / A_CG;
  const int b_c8 = tid % B_CG, b_r = tid / B_CG;
  const int aco = co0 + 8 * a_c8;
  const bool a_valid = aco < rows;
  const int a_g = a_valid ? aco / g.Cgo : 0;
  const uint16_t* a_base = P.dy[a_g] + (aco - a_g * g.Cgo);
  const int kk = k0 + 8 * b_c8;
  const bool b_valid = kk < KT;
  const KPos bp = kpos_init(b_valid ? kk : 0, g);
  const int2 btap = make_int2(g.dy[bp.t], g.dx[bp.t]);
  const uint16_t* b_base = P.x[bp.gi] + bp.cl;
  const int IHW = g.IH * g.IW;
  // deferred-BN prologue: this thread's 8 x channels are fixed -> coefficients once, in registers
  const float* bcf = b_valid ? P.xc[bp.gi] : nullptr;
  const bool brelu = (P.xrelu >> bp.gi) & 1u;
  float bsc[8], bsh[8];
  if (bcf != nullptr) { load8f(bcf + bp.cl, bsc); load8f(bcf + g.Cgi + bp.cl, bsh); }

  uint4 ra[A_V], rb[B_V];
  unsigned rbok = 0;   // in-image B rows of the staged chunk (the prologue leaves padding at 0)
  auto load = [&](long c) {
    const long mb = c * WG_M;
#pragma unroll
    for (int v = 0; v < A_V; ++v) {
      const long m = mb + a_r + A_RS * v;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (m < M && a_valid) val = *reinterpret_cast<const uint4*>(a_base + m * g.Cgo);
      ra[v] = val;
    }
    rbok = 0;
#pragma unroll
    for (int v = 0; v < B_V; ++v) {
      const long m = mb + b_r + B_RS * v;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (m < M && b_valid) {
        const int n = (int)(m / OHW);
        const int r = (int)(m - (long)n * OHW);
        const int oh = r / g.OW, ow = r - (r / g.OW) * g.OW;
        const int pix = TRANS ? in_pixel<true>(n * IHW, oh, ow, btap, g)
                              : in_pixel<false>(n * IHW, oh * g.stride, ow * g.stride, btap, g);
        if (pix >= 0) { val = *reinterpret_cast<const uint4*>(b_base + (long)pix * g.Cgi); rbok |= 1u << v; }
      }
      rb[v] = val;
    }
  };

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lg = lane >> 4;
  const int q = lr >> 2, p4 = lr & 3;   // tr-read: lane 4q+p supplies row q, cols 4p..4p+3
  const int rbase = 32 * wave + 8 * lg;

  long c = blockIdx.z;
  if (c < nchunks) load(c);
  for (; c < nchunks; c += gridDim.z) {
#pragma unroll
    for (int v = 0; v < A_V; ++v) *reinterpret_cast<uint4*>(&sA[(a_r + A_RS * v) * SA_LD + 8 * a_c8]) = ra[v];
#pragma unroll
    for (int v = 0; v < B_V; ++v) {
      uint4 val = rb[v];
      if (bcf != nullptr && ((rbok >> v) & 1u)) val = affine8(val, bsc, bsh, brelu);
      *reinterpret_cast<uint4*>(&sB[(b_r + B_RS * v) * SB_LD + 8 * b_c8]) = val;
    }
    __syncthreads();
    if (c + gridDim.z < nchunks) load(c + gridDim.z);     // next chunk in flight during the MFMAs
    uint4 fa[FI];
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const uint2 lo = tr_read(&sA[(rbase + q) * SA_LD + 16 * i + 4 * p4]);
      const uint2 hi = tr_read(&sA[(rbase + 4 + q) * SA_LD + 16 * i + 4 * p4]);
      fa[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const uint2 lo = tr_read(&sB[(rbase + q) * SB_LD + 16 * j + 4 * p4]);
      const uint2 hi = tr_read(&sB[(rbase + 4 + q) * SB_LD + 16 * j + 4 * p4]);
      const uint4 fb = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
      for (int i = 0; i < FI; ++i) acc[i][j] = mfma16x16x32(fa[i], fb, acc[i][j]);
    }
    __syncthreads();
  }

  // sequential cross-wave accumulation in LDS (fp32 tile), then one slab store per element
  float* red = reinterpret_cast<float*>(smem);
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* d = &red[(16 * i + 4 * lg + r) * K_T + 16 * j + lr];
            *d = (w == 0 ? 0.f : *d) + acc[i][j][r];
          }
    }
    __syncthreads();
  }
  // deterministic split-K: this block's partial tile goes to ITS slab (blockIdx.z) with plain stores;
  // unpack_wgrad sums the gridDim.z slabs in fixed order (no atomics, no zero-fill)
  float* slab = dw + (long)blockIdx.z * rows * KT;
  for (int e = tid; e < CO_T * K_T; e += 256) {
    const int ci = e / K_T, kj = e - (e / K_T) * K_T;
    const int co = co0 + ci, k = k0 + kj;
    if (co < rows && k < KT) slab[(long)co * KT + k] = red[e];
  }
}

// Halo-tiled weight gradient for stride-1 convs ("direct wgrad").  The gather kernel above reads
// every input pixel once per tap (a 9x im2col expansion through L2 for a 3x3); here a block stages an
// output tile of dY [TH x TW px][32 co] and the matching input HALO [(TH+eh) x (TW+ew) px][32 ci]
// in LDS ONCE, and every tap reads its shifted window of the halo with ds_read_b64_tr_b16 (each lane
// supplies its own pixel row address, so the shift is free).  Block output = dW[32 co][T taps][32 ci];
// the 4 waves own disjoint (tap, ci16) pairs, so no cross-wave reduction.  Blocks loop over pixel
// tiles (accumulating in registers) and finish by writing the block's fp32 slab (deterministic split-K).
// LDS layout: one 64-B row per pixel (32 channels, no padding); the two 32-B halves are XOR-swizzled
// by bit 3 of the pixel index.  A transposed read of 32 lanes touches pixels {b..b+3, b+8..b+11}
// (+ a tap shift): pixels p and p+8 share a bank quadrant and always sit in opposite halves, so both
// the dY and the halo reads are bank-conflict-free for every tap (a padded 72-B pitch is 2-way).
// Tile width TW in {16, 32} and TH = 256 / TW (eight 32-pixel slices); the halo row pitch HWd is
// padded to a multiple of 16 pixels, so a lane's read offsets are per-lane constants plus a
// per-slice uniform: the slice loop is only transposed reads and MFMAs.
constexpr int DW_CH = 32;               // co rows and ci channels per block

struct DwTile { int TH, TW, tw_shift, ey0, ex0, HH, HWd, HWv, tiles_y, tiles_x; float inv_hwv; };

constexpr int kDwWaves = 8;      // waves per block: each owns <= 3 (tap, ci16) pairs of a 3x3
constexpr int kDwMaxHalo = 640;  // halo pixels the staging registers cover (every T <= 9 tap set)
constexpr long kDwSplitTarget = 256;
constexpr int kDwMaxNcb = 3;
// two fragment sets (pipelined slice reads) where the registers allow it
#ifndef DWB
#define DWB(npw, ncb) ((ncb) * 2 + (npw) <= 5)
#endif     // 32-row dY sub-tiles per block, all sharing ONE staged input halo
constexpr int kDwMaxLds = 120 * 1024;
constexpr double kDwHaloCost = 0.5;   // input-halo staging per tile, in units of one co sub-tile's work
// staging elements per thread: NCB dY sub-tiles (2 slots of 128 pixels each) + the halo
constexpr int dw_stage(int ncb) { return 2 * ncb + kDwMaxHalo / (16 * kDwWaves); }

DEVI int dw_elem(int pix, int half, int sub4) {   // element offset of (pixel, 16-ch half, 4-ch sub)
  return pix * DW_CH + 16 * (half ^ ((pix >> 3) & 1)) + 4 * sub4;
}

// NCB > 1 (wide dY: horizontally fused convs, wide layers): the block owns NCB consecutive 32-row co
// sub-tiles.  The input halo is staged, and every B fragment read from LDS, ONCE per slice for all of
// them: one input pass per NCB sub-tiles instead of per sub-tile, and fewer LDS reads/writes per MFMA.
#ifndef DW_MIN_WAVES
#define DW_MIN_WAVES 1
#endif
// BWD: the dY sub-tiles are rebuilt from (dz, y) at staging time (WgradPtrs::gy, the deferred
// BN-backward prologue -- the same bwd8 as bn_act_bwd_apply, so dY is bit-identical)
template <int NPW, int NCB, bool BWD = false>
__global__ __launch_bounds__(64 * kDwWaves, DW_MIN_WAVES) void conv_wgrad_halo_kernel(WgradPtrs P, float* __restrict__ dw, ConvGeom g,
                                                              DwTile tl, int KT, long ntiles, int z0) {
  constexpr int NST = dw_stage(NCB);
  constexpr int LDT = DW_CH * NCB;                        // BWD table row length (the block's co rows)
  __shared__ float s_bt[BWD ? 5 * LDT : 1];
  extern __shared__ __attribute__((aligned(16))) uint16_t dsm[];
  constexpr int NPX = 256, NSL = 8, SUB = NPX * DW_CH;
  uint16_t* sY = dsm;                       // [NCB][256][32]  swizzled
  uint16_t* sX = dsm + NCB * SUB;           // [HH * HWd][32]  swizzled
  __shared__ int2 s_tap[kMaxTaps];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4, q = lr >> 2, p4 = lr & 3;
  const int co0 = blockIdx.y * DW_CH * NCB, ci0 = (blockIdx.z + z0) * DW_CH;   // z0: this launch's first ci chunk
  const int rows = g.Go * g.Cgo, Cip = g.Gi * g.Cgi;
  if (tid < kMaxTaps) s_tap[tid] = make_int2(g.dy[tid] - tl.ey0, g.dx[tid] - tl.ex0);
  if constexpr (BWD) {   // [5][LDT]: scale, shift (+inf: no ReLU test), k1, k2, k3 of the block's co rows
    for (int e = tid; e < LDT; e += 64 * kDwWaves) {
      const int co = co0 + e;
      const int gg = co < rows ? co / g.Cgo : 0, cl = co - gg * g.Cgo;
      const bool on = co < rows && P.gy[gg] != nullptr;
      s_bt[e] = on ? P.gs[gg][cl] : 0.f;
      s_bt[LDT + e] = (on && ((P.grelu >> gg) & 1u)) ? P.gs[gg][g.Cgo + cl] : INFINITY;
      s_bt[2 * LDT + e] = on ? P.gk[gg][cl] : 1.f;
      s_bt[3 * LDT + e] = on ? P.gk[gg][g.Cgo + cl] : 0.f;
      s_bt[4 * LDT + e] = on ? P.gk[gg][2 * g.Cgo + cl] : 0.f;
    }
  }

  // per-thread loader roles: vector vv = tid & 3 (8 channels), pixel lane vp = tid >> 2 (16 per wave)
  const int vv = tid & 3, vp = tid >> 2;
  const uint16_t* y_base[NCB];
  const uint16_t* z_base[BWD ? NCB : 1];   // BWD: the BN input y of the dY group (nullptr: plain group)
  bool y_ok[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int yco = co0 + DW_CH * cb + 8 * vv;
    y_ok[cb] = yco < rows;
    const int y_g = y_ok[cb] ? yco / g.Cgo : 0;
    y_base[cb] = P.dy[y_g] + (y_ok[cb] ? yco - y_g * g.Cgo : 0);
    if constexpr (BWD)
      z_base[cb] = (y_ok[cb] && P.gy[y_g] != nullptr) ? P.gy[y_g] + (yco - y_g * g.Cgo) : nullptr;
  }
  const int xci = ci0 + 8 * vv;
  const bool x_ok = xci < Cip;
  const int x_g = x_ok ? xci / g.Cgi : 0;
  const uint16_t* x_base = P.x[x_g] + (xci - x_g * g.Cgi);
  // deferred-BN prologue of the halo: the thread's 8 channels are fixed -> coefficients in registers
  const float* x_cf = x_ok ? P.xc[x_g] : nullptr;
  const bool x_relu = (P.xrelu >> x_g) & 1u;
  float x_sc[8], x_sh[8];
  if (x_cf != nullptr) {
    const int x_ch = xci - x_g * g.Cgi;
    load8f(x_cf + x_ch, x_sc);
    load8f(x_cf + g.Cgi + x_ch, x_sh);
  }
  __syncthreads();

  // lane pixel within a 32-pixel slice: lo = 8*lg + q, hi = lo + 4 (tile coords: row ry, column cx)
  const int plo = 8 * lg + q, phi = plo + 4;
  const int ry_lo = plo >> tl.tw_shift, cx_lo = plo & (tl.TW - 1);
  const int ry_hi = phi >> tl.tw_shift, cx_hi = phi & (tl.TW - 1);
  const int rows_per_slice = 32 >> tl.tw_shift;
  // A (dY) read offsets: slice sl adds 32*32*sl (bit 3 of the pixel is lg & 1 for every slice)
  int offA[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { offA[i][0] = dw_elem(plo, i, p4); offA[i][1] = dw_elem(phi, i, p4); }
  // B (halo) read offsets per owned pair: slice sl adds rows_per_slice*sl*HWd*32.  A pair is a (tap, full
  // 16-channel half) or -- for a half with 8 real channels (a 24-channel input's second half, an 8-channel
  // input, a 40-channel input's second chunk) -- TWO taps of that half packed into one 16-wide fragment:
  // source lanes p4 0-1 address tap 2pp, lanes 2-3 tap 2pp+1, so the transposed read puts tap 2pp's 8
  // channels in columns 0-7 and tap 2pp+1's in 8-15 (dw_pairs, the host's slot count).  Pair slots past
  // npairs read a valid address and are never stored.
  const int R = min(DW_CH, Cip - ci0);
  const int nfull = R >> 4, nfp = nfull * g.T;
  const int npairs = nfp + ((R & 15) ? (g.T + 1) >> 1 : 0);
  int offB[NPW][2];
#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    const int pr = wave + kDwWaves * j;
    int t = 0, cf = 0, sub = p4;
    if (pr < nfp) {
      t = pr / nfull;
      cf = pr - t * nfull;
    } else if (pr < npairs) {
      const int ta = 2 * (pr - nfp), tb = ta + (p4 >> 1);
      t = tb < g.T ? tb : ta;
      cf = nfull;
      sub = p4 & 1;
    }
    const int2 d = s_tap[t];
    offB[j][0] = dw_elem((ry_lo + d.x) * tl.HWd + cx_lo + d.y, cf, sub);
    offB[j][1] = dw_elem((ry_hi + d.x) * tl.HWd + cx_hi + d.y, cf, sub);
  }
  // slots holding a pair (wave-uniform): the slice loop runs only those -- a 40-channel input's second
  // chunk has 5 pairs for 24 slots
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int live = npairs > wv ? min(NPW, (npairs - wv + kDwWaves - 1) / kDwWaves) : 0;

  f32x4_t acc[NCB][2][NPW];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NPW; ++j) acc[cb][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nh = tl.HH * tl.HWv;
  // Software pipeline over the block's tiles: a tile's staging loads (NST x 16 B per thread,
  // host-checked) are issued into registers before the previous tile's MFMA phase and written to LDS
  // after it, so HBM latency hides under the MFMAs.  Slot u < 2*NCB is dY sub-tile u/2 (pixels
  // vp + 128*(u&1)); the other slots walk the halo.
  uint4 sv[NST];
  uint4 sz[BWD ? 2 * NCB : 1];   // BWD: y of the dY slots
  int sd[NST];
  unsigned sx = 0;   // staged halo slots that hold in-image pixels (get the BN prologue)
  unsigned syb = 0;  // BWD: dY slots with a loaded y (get the BN-backward prologue)
  auto stage_load = [&](long tix) {
    const int per_img = tl.tiles_y * tl.tiles_x;
    const int n = (int)(tix / per_img);
    const int rem = (int)(tix - (long)n * per_img);
    const int y0 = (rem / tl.tiles_x) * tl.TH, x0 = (rem % tl.tiles_x) * tl.TW;
    const long yoff = (long)n * g.OH * g.OW * g.Cgo;
    const uint16_t* xim = x_base + (long)n * g.IH * g.IW * g.Cgi;
    sx = 0;
    syb = 0;
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      sv[u] = make_uint4(0, 0, 0, 0);
      sd[u] = -1;
      if (u < 2 * NCB) {
        const int cb = u >> 1, e = vp + 16 * kDwWaves * (u & 1);
        const int oy = y0 + (e >> tl.tw_shift), ox = x0 + (e & (tl.TW - 1));
        sd[u] = cb * SUB + dw_elem(e, vv >> 1, 2 * (vv & 1));
        if constexpr (BWD) sz[u] = make_uint4(0, 0, 0, 0);
        if (y_ok[cb] && oy < g.OH && ox < g.OW) {
          const long po = yoff + (oy * g.OW + ox) * g.Cgo;
#ifdef DW_KO_LOAD   // (profiling knock-out builds only: no staging loads)
          if (po < 0)
#endif
          sv[u] = *reinterpret_cast<const uint4*>(y_base[cb] + po);
          if constexpr (BWD) {
            if (z_base[cb] != nullptr) {
              sz[u] = *reinterpret_cast<const uint4*>(z_base[cb] + po);
              syb |= 1u << u;
            }
          }
        }
      } else {
        const int hp = vp + 16 * kDwWaves * (u - 2 * NCB);
        if (hp < nh) {
          const int hy = fdiv(hp, tl.HWv, tl.inv_hwv), hx = hp - __mul24(hy, tl.HWv);
          const int iy = y0 + hy + tl.ey0, ix = x0 + hx + tl.ex0;
          sd[u] = NCB * SUB + dw_elem(hy * tl.HWd + hx, vv >> 1, 2 * (vv & 1));
          if (x_ok && (unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW) {
#ifdef DW_KO_LOAD
            if (iy < 0)
#endif
            sv[u] = *reinterpret_cast<const uint4*>(xim + (iy * g.IW + ix) * g.Cgi);
            sx |= 1u << u;
          }
        }
      }
    }
  };
  if ((long)blockIdx.x < ntiles) stage_load(blockIdx.x);
  for (long tix = blockIdx.x; tix < ntiles; tix += gridDim.x) {
    __syncthreads();   // previous tile's LDS reads are done
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      if (sd[u] < 0) continue;
      uint4 v = sv[u];
      if (x_cf != nullptr && ((sx >> u) & 1u)) v = affine8(v, x_sc, x_sh, x_relu);
      if constexpr (BWD) {
        if (u < 2 * NCB && ((syb >> u) & 1u)) v = bwd8(v, sz[u < 2 * NCB ? u : 0], s_bt + DW_CH * (u >> 1) + 8 * vv, LDT);
      }
      *reinterpret_cast<uint4*>(&sY[sd[u]]) = v;
    }
    __syncthreads();
    if (tix + gridDim.x < ntiles) stage_load(tix + gridDim.x);   // in flight during the MFMAs
    // Slice loop: branch-free and software-pipelined -- slice s+1's transposed reads are issued before
    // slice s's MFMAs (two fragment sets when the registers allow, DWB), so LDS latency hides under the
    // MFMAs of the same wave.  MFMAs run unconditionally: a pair slot past npairs (or a co half past
    // `rows`, whose staged dY is zero) accumulates into registers that are never stored.  Measured: the
    // per-pair / per-half branches split every read -> wait -> MFMA into its own basic block, so nothing
    // overlapped inside a wave (2 waves/SIMD: 53 % of wave cycles waiting, MFMA busy 0.19).
    // L: the wave's live pair slots (compile-time per call below)
    auto slices = [&](auto LC) {
      constexpr int L = decltype(LC)::value;
      auto frags = [&](int sl, uint4 (&fa)[NCB][2], uint4 (&fb)[L]) {
#ifdef DW_KO_LDSREAD   // (profiling knock-out: fragments from registers, no transposed LDS reads)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
          for (int i = 0; i < 2; ++i) fa[cb][i] = make_uint4(sl + cb, i, lane, (unsigned)tix);
#pragma unroll
        for (int j = 0; j < L; ++j) fb[j] = make_uint4(sl, j, lane, (unsigned)tix);
        return;
#endif
        const int sa = sl * 32 * DW_CH, sb = sl * rows_per_slice * tl.HWd * DW_CH;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const uint2 lo = tr_read(&sY[cb * SUB + sa + offA[i][0]]);
            const uint2 hi = tr_read(&sY[cb * SUB + sa + offA[i][1]]);
            fa[cb][i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
          }
#pragma unroll
        for (int j = 0; j < L; ++j) {
          const uint2 lo = tr_read(&sX[sb + offB[j][0]]);
          const uint2 hi = tr_read(&sX[sb + offB[j][1]]);
          fb[j] = make_uint4(lo.x, lo.y, hi.x, hi.y);
        }
      };
      auto mma = [&](const uint4 (&fa)[NCB][2], const uint4 (&fb)[L]) {
#pragma unroll
        for (int j = 0; j < L; ++j)
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
#ifdef DW_KO_MFMA   // (profiling knock-out: no MFMAs; the fragments stay live)
              acc[cb][i][j][0] += __uint_as_float(fa[cb][i].x ^ fb[j].y);
#else
              acc[cb][i][j] = mfma16x16x32(fa[cb][i], fb[j], acc[cb][i][j]);
#endif
            }
      };
      constexpr int NB = DWB(L, NCB) ? 2 : 1;
      uint4 fa[NB][NCB][2], fb[NB][L];
      if constexpr (NB == 2) {
        frags(0, fa[0], fb[0]);
#pragma unroll
        for (int sl = 0; sl < NSL; ++sl) {
          if (sl + 1 < NSL) frags(sl + 1, fa[(sl + 1) & 1], fb[(sl + 1) & 1]);
          mma(fa[sl & 1], fb[sl & 1]);
        }
      } else {   // register-bound variants: one set (the scheduler still hoists reads across slices)
        constexpr int UNR = L * NCB >= 9 ? 1 : NSL;   // <3,3> spills when unrolled
#pragma unroll UNR
        for (int sl = 0; sl < NSL; ++sl) {
          frags(sl, fa[0], fb[0]);
          mma(fa[0], fb[0]);
        }
      }
    };
#ifdef DW_KO_SLICES   // (profiling knock-out: staging only -- no fragment reads, no MFMAs)
    continue;
#endif
    // (one slice-loop variant: a second one -- fewer slots for waves with dead ones -- spills the <3,2> / <3,3>
    // kernels; chunks with fewer pairs get their own launch instead, conv_wgrad)
    if (live > 0) slices(std::integral_constant<int, NPW>{});
  }
  // deterministic split-K: block x writes its partial dW tile into slab x (plain stores, every needed
  // element exactly once per slab); unpack_wgrad sums the nsplit slabs in fixed order
  float* dwr = dw + (long)blockIdx.x * rows * KT;
#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    const int pr = wave + kDwWaves * j;
    if (pr >= npairs) continue;
    int t, ci;
    if (pr < nfp) {
      t = pr / nfull;
      ci = ci0 + 16 * (pr - t * nfull) + lr;
    } else {   // packed pair: columns 0-7 tap 2pp, 8-15 tap 2pp+1 (past the last tap: never stored)
      t = 2 * (pr - nfp) + (lr >> 3);
      if (t >= g.T) continue;
      ci = ci0 + 16 * nfull + (lr & 7);
    }
    if (ci >= Cip) continue;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + DW_CH * cb + 16 * i + 4 * lg + r;
          if (co < rows) dwr[(long)co * KT + t * Cip + ci] = acc[cb][i][j][r];
        }
  }
}

__global__ void pack_weight_kernel(const float* __restrict__ src, uint16_t* __restrict__ dst, int nrow, int nch,
                                   int T, int Cpk, int Kp, int t_base, int c_base, long s_row, long s_ch) {
  const long total = (long)nrow * nch * T;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int t = (int)(i % T);
    const long rc = i / T;
    const int c = (int)(rc % nch);
    const int row = (int)(rc / nch);
    dst[(long)row * Kp + (t_base + t) * Cpk + c_base + c] = f2bf(src[row * s_row + c * s_ch + t]);
  }
}

// dst[row][c][t] (+)= sum over the nrep split-K slabs of src[r][row][(t_base+t)*Cpk + c_base + c].
// 64 elements x 8 slab groups per 512-thread block: group g sums slabs g, g+8, ... in order and the
// 8 group sums are added in group order -- a fixed summation order, so bitwise deterministic, with 8x
// the loads in flight of a one-thread-per-element loop (the slabs are read straight from L2/HBM).
// Element order (row, t, c) keeps a wave's slab reads contiguous in c.
constexpr int kUnpackGroups = 8;
__global__ __launch_bounds__(64 * kUnpackGroups) void unpack_wgrad_kernel(
    const float* __restrict__ src, float* __restrict__ dst, int nrow, int nch, int T, int Cpk, int Ktot, int t_base,
    int c_base, long s_row, long s_ch, int accumulate, int nrep, long rep_stride) {
  __shared__ float part[kUnpackGroups][64];
  const long total = (long)nrow * nch * T;
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const long i = (long)blockIdx.x * 64 + lane;
  long si = 0;
  if (i < total) {
    const int c = (int)(i % nch);
    const long rt = i / nch;
    const int t = (int)(rt % T);
    const int row = (int)(rt / T);
    si = (long)row * Ktot + (t_base + t) * Cpk + c_base + c;
  }
  float v = 0.f;
  if (i < total) {
#pragma unroll 4
    for (int r = grp; r < nrep; r += kUnpackGroups) v += src[r * rep_stride + si];
  }
  part[grp][lane] = v;
  __syncthreads();
  if (grp == 0 && i < total) {
#pragma unroll
    for (int g2 = 1; g2 < kUnpackGroups; ++g2) v += part[g2][lane];
    const int c = (int)(i % nch);
    const long rt = i / nch;
    const int t = (int)(rt % T);
    const int row = (int)(rt / T);
    float* d = dst + row * s_row + c * s_ch + t;
    *d = accumulate ? *d + v : v;
  }
}

// Batched weight packing: one launch re-packs every conv weight of the model after the optimizer
// step (jobs = rows of an int64 table; blocks map to jobs through a prefix array).
constexpr int kPackPerBlock = 2048;

__global__ __launch_bounds__(256) void pack_batch_kernel(const int64_t* __restrict__ jobs, const int* __restrict__ prefix,
                                                         int njobs) {
  const int b = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {   // last job j with prefix[j] <= b
    const int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const int64_t* J = jobs + 12 * lo;
  const float* src = reinterpret_cast<const float*>(J[0]);
  uint16_t* dst = reinterpret_cast<uint16_t*>(J[1]);
  const int nch = (int)J[3], T = (int)J[4], Cpk = (int)J[5], Kp = (int)J[6];
  const int t_base = (int)J[7], c_base = (int)J[8];
  const long s_row = J[9], s_ch = J[10], total = J[11];
  const long start = (long)(b - prefix[lo]) * kPackPerBlock;
  for (long i = start + threadIdx.x; i < start + kPackPerBlock && i < total; i += 256) {
    const int t = (int)(i % T);
    const long rc = i / T;
    const int c = (int)(rc % nch);
    const int row = (int)(rc / nch);
    dst[(long)row * Kp + (t_base + t) * Cpk + c_base + c] = f2bf(src[row * s_row + c * s_ch + t]);
  }
}

// ------------------------------------------------------------------------------------------------
// Halo-tiled direct convolution (stride 1, non-TRANS): forward of every stride-1 conv and the
// data-gradient of every stride-1 conv whose (summed) input width fits the LDS tile.
// A block owns a TH x TW output-pixel tile of one image and ALL output rows.  The input tile plus its
// tap halo (all Cip channels, zero outside the image) is staged once in LDS with a pixel pitch of an
// odd number of 16-B slots, so the 16 consecutive pixels of a ds_read_b128 hit distinct banks.  Every
// 32-wide k-chunk then reads its B fragment at  pixel_base(lane) + koff[chunk][lane>>4]  -- one
// table lookup replaces the per-lane tap/bounds arithmetic of the gather kernel, and the input is read
// from HBM once per tile (halo overhead (TH+ey)(TW+ex)/(TH*TW)) instead of once per tap from L2.
// Waves split the tile's pixels (NJ 16-pixel columns each) and loop over the 16*MI-row groups.
struct HaloGeom {
  int TH, TW, tw_shift, HH, HWD, ey0, ex0, tiles_y, tiles_x, pitch, CC, nch, KS;
  int xtab;                          // deferred-BN prologue present: LDS coefficient table (3 x Cip fp32)
  int mi, pipe, nj;                  // row-group size (16*mi rows), PIPE mode, pixel columns per wave
  int st_q, st_r, st_a, st_b;        // staging cursor step of 256 elements: 256 = st_q*C8 + st_r,
                                     // st_q = st_a*HWD + st_b (non-chunked: C8 = Cip/8)
  float inv_c8, inv_hwd, inv_cgi;   // fp32 reciprocals for fdiv (staging index math)
  int split;                         // split-bank tile image (halo_phys): two copies, one per k-group parity
  int tile_elems;                    // LDS elements of the tile image (both copies when split)
};

// Split-bank tile image.  CDNA4 services a ds_read_b128 in four 16-lane groups, each mixing lanes of two
// MFMA k-groups: {0-3,12-15 | 20-27}, {4-11 | 16-19,28-31} (k-groups 0 | 1) and the same +32 (2 | 3).  With
// one image the two k-groups read (tap, channel) units at unrelated offsets and collide (PMC: 0.23-0.41
// bank-conflict rate).  Split: the tile is stored twice, copy h in the h-th 128-B half of every 256-B bank
// row (logical 16-B slot s -> row s / 8, half h, column s % 8); k-groups of parity h read copy h.  A group's
// 8 lanes per k-group read 8 consecutive pixels at an odd slot pitch -> 8 distinct columns of their half:
// conflict-free for every tap offset, at twice the tile's LDS and staging stores.
DEVI int halo_phys(int e, int smask) { return e + (e & smask); }   // smask = ~63 (split) or 0


constexpr int kHaloMaxKS = 96;   // k-steps per channel chunk (4 (tap, 8-channel) units each)
constexpr int kHaloWaves = 4;
constexpr int kHaloMaxRows = 512;
constexpr int kHaloLd = 8;       // 16-B loads in flight per thread while staging
constexpr int kHaloMaxLds = 96 * 1024;   // tile (<= halo_tile_cap() by geometry) + stats + prologue table
constexpr int kHaloTileKB = 76;          // tile + stats + prologue table cap: 2 blocks/CU with the static tables
constexpr int kPipeLd = 8;               // PIPE: 16-B vectors per thread prefetched for the next tile
constexpr int kPipeGrid = 256 * 2;       // PIPE: persistent grid, 2 blocks on each of the 256 CUs
constexpr int kPipeMaxLds = 78 * 1024;   // PIPE: tile + stats + prologue table + weights, 2 blocks/CU

// K is walked in UNITS of (tap t, 8 channels c8) -- the lane group lg of k-step ks takes unit
// 4*ks + lg.  Per unit: A offset t*Cip + 8*c8 (+ chunk base) into the packed weight row, B offset
// tapoff(t) + 8*c8 into the LDS tile.  With one chunk (CC == Cip) this is exactly the packed
// k = t*Cip + ci order, so A is read contiguously and the padding units past T*Cip hit the packed
// rows' zero padding (their B offset is a harmless in-tile address).  With CHUNKED the input channels
// are staged CC at a time (inputs too wide for one LDS tile: the data-gradient of horizontally fused
// convs reads 8 dY groups), padding units zero A, the next chunk's global loads are in flight in
// registers while the current one runs on the MFMAs, and the accumulators persist across chunks
// (single row group).

// BWD: the data-gradient staging rebuilds dY from (dz, y) per input group (ConvArgs::gy, the deferred
// BN-backward prologue: no bn_act_bwd_apply pass writes dY); never with PIPE
template <int MI, int NJ, bool CHUNKED, bool BNE = false, bool PIPE = false, bool BWD = false>
__global__ __launch_bounds__(64 * kHaloWaves, (CHUNKED || PIPE) ? 2 : ((MI <= 2 && NJ <= 4) ? 4 : 3)) void conv_halo_kernel(ConvArgs a, HaloGeom hg) {
  static_assert(!(BWD && PIPE), "BN-backward prologue: standard / chunked staging only");
  extern __shared__ uint4 halo_smem[];
  uint16_t* tile = reinterpret_cast<uint16_t*>(halo_smem);
  __shared__ int s_ua[CHUNKED ? kHaloMaxKS * 4 : 1];
  __shared__ int s_ub[kHaloMaxKS * 4];
  // input-group pointers in LDS: staging indexes them per lane.  a.x[gi] with a lane-varying gi compiles
  // to a global load of the pointer from the kernarg segment + s_waitcnt vmcnt(0) before the data load,
  // which drains every staging load in flight -- the staging loop then ran one round trip at a time (a
  // select chain over a.x[] is folded back into that load); an LDS read waits on lgkmcnt only.
  __shared__ const uint16_t* s_xp[kMaxGroups];
  __shared__ const uint16_t* s_yp[BWD ? kMaxGroups : 1];   // BWD: the groups' BN inputs y (nullable)
  // (pointers read back from LDS are generic: loads through them would be FLAT, counted in lgkmcnt too,
  // so the next pointer read's lgkmcnt wait would drain them again -- load through global pointers)
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int Cip = g.Gi * g.Cgi, C8c = hg.CC >> 3;
  const int rows = g.Go * g.Cgo;
  const int hpx = hg.HH * hg.HWD;
  if (tid < kMaxGroups) {
    s_xp[tid] = a.x[tid];
    if constexpr (BWD) s_yp[tid] = a.gy[tid];
  }
  if (g.Gi > 1) __syncthreads();   // block-uniform; Gi == 1 staging never reads s_xp / s_yp
  // per-wave (sum, sum^2) rows after the tile: [kHaloWaves][2][rows] fp32
  float* s_stat = reinterpret_cast<float*>(tile + hg.tile_elems);
  const int smask = hg.split ? ~63 : 0;                  // split-bank image (halo_phys)
  const int hcopy = hg.split ? ((lg & 1) << 6) : 0;      // this lane's copy: k-group parity
  auto st_tile = [&](int e, const uint4& val) {
    uint4* tp = reinterpret_cast<uint4*>(tile + halo_phys(e, smask));
    tp[0] = val;
    if (hg.split) tp[8] = val;   // + 128 B: the other half of the bank row
  };
  // deferred-BN prologue table after them (hg.xtab): per input channel scale, shift and the ReLU floor
  // (0 or -inf); groups without a prologue get the identity (exact on bf16 values)
  float* s_coef = s_stat + kHaloWaves * 2 * rows;
  if constexpr (BWD) {
    // BN-backward table [5][Cip]: scale, shift (+inf: no ReLU test), k1, k2, k3; plain groups get the
    // identity (dy = dz exactly: y is never loaded for them)
    for (int c = tid; c < Cip; c += 64 * kHaloWaves) {
      const int gi = c / g.Cgi, cl = c - gi * g.Cgi;
      const bool on = a.gy[gi] != nullptr;
      const float* st = a.gs[gi];
      const float* k = a.gk[gi];
      s_coef[c] = on ? st[cl] : 0.f;
      s_coef[Cip + c] = (on && ((a.grelu >> gi) & 1u)) ? st[g.Cgi + cl] : INFINITY;
      s_coef[2 * Cip + c] = on ? k[cl] : 1.f;
      s_coef[3 * Cip + c] = on ? k[g.Cgi + cl] : 0.f;
      s_coef[4 * Cip + c] = on ? k[2 * g.Cgi + cl] : 0.f;
    }
    __syncthreads();
  } else if (!BNE && hg.xtab) {
    for (int c = tid; c < Cip; c += 64 * kHaloWaves) {
      const int gi = c / g.Cgi, cl = c - gi * g.Cgi;
      const float* cf = a.xc[gi];
      s_coef[c] = cf != nullptr ? cf[cl] : 1.f;
      s_coef[Cip + c] = cf != nullptr ? cf[g.Cgi + cl] : 0.f;
      s_coef[2 * Cip + c] = (cf != nullptr && ((a.xrelu >> gi) & 1u)) ? 0.f : -INFINITY;
    }
    __syncthreads();   // read by the first staging pass, before any other barrier
  }
  // PIPE: the packed weights live in LDS for the block's lifetime (read once, reused by every tile;
  // and with no global loads in the MFMA loop, no vmcnt wait there drains the in-flight prefetch of
  // the next tile).  Row pitch = an odd number of 16-B slots.
  uint16_t* sA = reinterpret_cast<uint16_t*>(s_coef + (hg.xtab ? 3 * Cip : 0));
  const int pitchA = (4 * hg.KS + 1) * 8;
  if (PIPE) {
    const int rowsA = ((rows + 16 * MI - 1) / (16 * MI)) * 16 * MI;
    const int per_row = 4 * hg.KS;
    for (int e = tid; e < rowsA * per_row; e += 64 * kHaloWaves) {
      const int r = e / per_row, q = e - r * per_row;
      *reinterpret_cast<uint4*>(sA + r * pitchA + q * 8) = *reinterpret_cast<const uint4*>(a.w + (long)r * g.Kp + q * 8);
    }
  }
  // per-block BN partials accumulate over the block's tiles (+= by the owning lane; published by the
  // first staging barrier)
  if (a.stat_part != nullptr)
    for (int c = tid; c < kHaloWaves * 2 * rows; c += 64 * kHaloWaves) s_stat[c] = 0.f;

  // XCD-aware bijective remap: neighbouring tiles (shared halo rows) land on one XCD's L2.
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xq = nwg / 8, xr = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + orig / 8;
  const int per_img = hg.tiles_y * hg.tiles_x;
  const int ntiles = g.N * per_img;
  const int total = hpx * C8c;
  // tile origin (set per tile; the staging lambdas read it by reference)
  int ty0 = 0, tx0 = 0;
  long img = 0;
  const uint16_t* xim0 = a.x[0];
  const uint16_t* yim0 = BWD ? a.gy[0] : nullptr;   // BWD, Gi == 1: the BN input of the one group
  auto set_tile = [&](int t, int& y0, int& x0, long& im) {
    const int n = t / per_img;
    const int trem = t - n * per_img;
    const int tyi = trem / hg.tiles_x;
    y0 = tyi * hg.TH;
    x0 = (trem - tyi * hg.tiles_x) * hg.TW;
    im = (long)n * g.IH * g.IW;
  };

  // staging: element idx -> (halo pixel, 8-channel slot of the chunk); zero outside the image.
  // 32-bit per-image offsets (one image's activations < 2^31 elements) from per-image base pointers.
  // (BWD: yv[u] = the BN input y at the same element, cc[u] = its channel in [0, Cip) or -1 outside
  // the image / for a plain group -- the zero padding and plain groups stay dz)
  auto load_batch = [&](int c0, int base, uint4* v, int* dst, uint4* yv, int* cc) {
#pragma unroll
    for (int u = 0; u < kHaloLd; ++u) {
      const int idx = base + u * 64 * kHaloWaves;
      v[u] = make_uint4(0, 0, 0, 0);
      dst[u] = -1;
      if constexpr (BWD) {
        yv[u] = make_uint4(0, 0, 0, 0);
        cc[u] = -1;
      }
      if (idx < total) {
        const int hp = fdiv(idx, C8c, hg.inv_c8), c8 = idx - __mul24(hp, C8c);
        const int hy = fdiv(hp, hg.HWD, hg.inv_hwd), hx = hp - __mul24(hy, hg.HWD);
        const int iy = ty0 + hg.ey0 + hy, ix = tx0 + hg.ex0 + hx;
        dst[u] = __mul24(hp, hg.pitch) + c8 * 8;
        if ((unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW) {
          const int ci = c0 + c8 * 8;
          const int pix = iy * g.IW + ix;
          if (g.Gi == 1) {
            v[u] = ldg4(xim0 + pix * g.Cgi + ci);
            if constexpr (BWD) {
              yv[u] = ldg4(yim0 + pix * g.Cgi + ci);
              cc[u] = ci;
            }
          } else {
            const int gi = fdiv(ci, g.Cgi, hg.inv_cgi);
            const int off = img * g.Cgi + (pix * g.Cgi + ci - __mul24(gi, g.Cgi));
            v[u] = ldg4(s_xp[gi] + off);
            if constexpr (BWD) {
              const uint16_t* yp = s_yp[gi];
              if (yp != nullptr) {
                yv[u] = ldg4(yp + off);
                cc[u] = ci;
              }
            }
          }
        }
      }
    }
  };
  auto store_batch = [&](const uint4* v, const int* dst, const uint4* yv, const int* cc) {
#pragma unroll
    for (int u = 0; u < kHaloLd; ++u) {
      if (dst[u] < 0) continue;
      uint4 val = v[u];
      if constexpr (BWD) {
        if (cc[u] >= 0) val = bwd8(val, yv[u], s_coef + cc[u], Cip);
      }
      st_tile(dst[u], val);
    }
  };
  // Deferred-BN prologue as its own pass over the staged chunk (after the barrier that published it):
  // every in-image vector is normalised (+ReLU) in place from the LDS table, the zero padding is left
  // alone.  Kept out of load/store_batch: temporaries there stay live into the MFMA loop and spill.
  auto xform_pass = [&](int c0) {
    for (int idx = tid; idx < total; idx += 64 * kHaloWaves) {
      const int hp = fdiv(idx, C8c, hg.inv_c8), c8 = idx - __mul24(hp, C8c);
      const int hy = fdiv(hp, hg.HWD, hg.inv_hwd), hx = hp - __mul24(hy, hg.HWD);
      const int iy = ty0 + hg.ey0 + hy, ix = tx0 + hg.ex0 + hx;
      if ((unsigned)iy >= (unsigned)g.IH || (unsigned)ix >= (unsigned)g.IW) continue;
      const int te = __mul24(hp, hg.pitch) + c8 * 8;
      const uint4* tp = reinterpret_cast<const uint4*>(tile + halo_phys(te, smask));
      const float* cp = s_coef + c0 + c8 * 8;
      const float4 s0 = *reinterpret_cast<const float4*>(cp), s1 = *reinterpret_cast<const float4*>(cp + 4);
      const float4 h0 = *reinterpret_cast<const float4*>(cp + Cip), h1 = *reinterpret_cast<const float4*>(cp + Cip + 4);
      const float4 l0 = *reinterpret_cast<const float4*>(cp + 2 * Cip);
      const float4 l1 = *reinterpret_cast<const float4*>(cp + 2 * Cip + 4);
      float f[8];
      unpack8(*tp, f);
      f[0] = fmaxf(fmaf(f[0], s0.x, h0.x), l0.x); f[1] = fmaxf(fmaf(f[1], s0.y, h0.y), l0.y);
      f[2] = fmaxf(fmaf(f[2], s0.z, h0.z), l0.z); f[3] = fmaxf(fmaf(f[3], s0.w, h0.w), l0.w);
      f[4] = fmaxf(fmaf(f[4], s1.x, h1.x), l1.x); f[5] = fmaxf(fmaf(f[5], s1.y, h1.y), l1.y);
      f[6] = fmaxf(fmaf(f[6], s1.z, h1.z), l1.z); f[7] = fmaxf(fmaf(f[7], s1.w, h1.w), l1.w);
      st_tile(te, pack8(f));
    }
  };

  for (int e = tid; e < hg.KS * 4; e += 64 * kHaloWaves) {
    int ua = -1, ub = 0;
    if (e < g.T * C8c) {
      const int t = e / C8c, c8 = e - t * C8c;
      ua = t * Cip + 8 * c8;
      ub = ((g.dy[t] - hg.ey0) * hg.HWD + (g.dx[t] - hg.ex0)) * hg.pitch + 8 * c8;
    }
    if (CHUNKED) s_ua[e] = ua;
    s_ub[e] = ub;
  }

  constexpr int PF = CHUNKED ? kHaloLd : (PIPE ? kPipeLd : 1);
  uint4 pv[PF];
  int pd[PF];
  uint4 pyv[(BWD && CHUNKED) ? PF : 1];
  int pcc[(BWD && CHUNKED) ? PF : 1];
  // PIPE: the whole halo tile of tile t (total <= 256*kPipeLd vectors, host-checked) is fetched into
  // registers while the block computes the previous tile -- HBM reads overlap MFMA + epilogue work
  // instead of running as serial phases.  pd[u] = LDS offset | (slot + 1) << 16 for in-image vectors,
  // the bare offset for zero padding, -1 past the tile.
  auto pipe_fetch = [&](int t) {
    int y0, x0;
    long im;
    set_tile(t, y0, x0, im);
    const uint16_t* xb = a.x[0] + im * g.Cgi;
    int c8 = tid % C8c, hp = tid / C8c;
    int hy = hp / hg.HWD, hx = hp - hy * hg.HWD;
    const int iy0 = y0 + hg.ey0, ix0 = x0 + hg.ex0;
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      pv[u] = make_uint4(0, 0, 0, 0);
      pd[u] = -1;
      if (tid + u * 64 * kHaloWaves < total) {
        const int iy = iy0 + hy, ix = ix0 + hx;
        pd[u] = __mul24(hp, hg.pitch) + c8 * 8;
        if ((unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW) {
          const int ci = c8 * 8;
          const int pix = iy * g.IW + ix;
          pd[u] |= (c8 + 1) << 16;
          if (g.Gi == 1) {
            pv[u] = ldg4(xb + pix * g.Cgi + ci);
          } else {
            const int gi = fdiv(ci, g.Cgi, hg.inv_cgi);
            pv[u] = ldg4(s_xp[gi] + im * g.Cgi + (pix * g.Cgi + ci - __mul24(gi, g.Cgi)));
          }
        }
      }
      c8 += hg.st_r;
      const int carry = c8 >= C8c ? 1 : 0;
      c8 -= carry * C8c;
      hp += hg.st_q + carry;
      hx += hg.st_b + carry;
      hy += hg.st_a;
      if (hx >= hg.HWD) { hx -= hg.HWD; ++hy; }
    }
  };
  auto pipe_store = [&]() {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (pd[u] < 0) continue;
      uint4 val = pv[u];
      const int c = (pd[u] >> 16) - 1;
      if (!BNE && hg.xtab && c >= 0) {
        const float* cp = s_coef + c * 8;
        const float4 s0 = *reinterpret_cast<const float4*>(cp), s1 = *reinterpret_cast<const float4*>(cp + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(cp + Cip);
        const float4 h1 = *reinterpret_cast<const float4*>(cp + Cip + 4);
        const float4 l0 = *reinterpret_cast<const float4*>(cp + 2 * Cip);
        const float4 l1 = *reinterpret_cast<const float4*>(cp + 2 * Cip + 4);
        float f[8];
        unpack8(val, f);
        f[0] = fmaxf(fmaf(f[0], s0.x, h0.x), l0.x); f[1] = fmaxf(fmaf(f[1], s0.y, h0.y), l0.y);
        f[2] = fmaxf(fmaf(f[2], s0.z, h0.z), l0.z); f[3] = fmaxf(fmaf(f[3], s0.w, h0.w), l0.w);
        f[4] = fmaxf(fmaf(f[4], s1.x, h1.x), l1.x); f[5] = fmaxf(fmaf(f[5], s1.y, h1.y), l1.y);
        f[6] = fmaxf(fmaf(f[6], s1.z, h1.z), l1.z); f[7] = fmaxf(fmaf(f[7], s1.w, h1.w), l1.w);
        val = pack8(f);
      }
      *reinterpret_cast<uint4*>(tile + (pd[u] & 0xffff)) = val;   // (PIPE: never split)
    }
  };
  if (PIPE) pipe_fetch(wgid);

  int pb[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int p = (wave * NJ + j) * 16 + lr;
    pb[j] = ((p >> hg.tw_shift) * hg.HWD + (p & (hg.TW - 1))) * hg.pitch;
  }

  const int n_rg = CHUNKED ? 1 : (rows + 16 * MI - 1) / (16 * MI);
  const int t_end = PIPE ? ntiles : wgid + 1;      // one tile per block unless PIPE (persistent grid)
  for (int tt = wgid; tt < t_end; tt += (PIPE ? nwg : 1)) {
  set_tile(tt, ty0, tx0, img);
  xim0 = a.x[0] + img * g.Cgi;
  if constexpr (BWD) {
    if (g.Gi == 1) yim0 = a.gy[0] + img * g.Cgi;
  }
  if (CHUNKED) {
    load_batch(0, tid, pv, pd, pyv, pcc);   // host guarantees total <= 64*kHaloWaves*kHaloLd
  } else if (PIPE) {
    if (tt != wgid) __syncthreads();   // every wave is done reading the previous tile
    pipe_store();
    __syncthreads();
    if (tt + nwg < ntiles) pipe_fetch(tt + nwg);   // next tile's HBM reads overlap this tile's work
  } else {
    // Whole-input staging, before the row-group loop so that none of its temporaries stay live into
    // the MFMA loop.  Element idx = tid + 256*k -> (halo pixel hp = (hy, hx), 8-channel slot c8) is
    // walked with an incremental cursor (one division per thread, then adds with carries: this phase
    // is VALU-issue-bound).  The deferred-BN prologue runs at LDS-store time from the coefficient
    // table, only on in-image vectors (cc[u] = slot, -1 for the zero padding).
    int c8 = tid % C8c, hp = tid / C8c;
    int hy = hp / hg.HWD, hx = hp - hy * hg.HWD;
    const int iy0 = ty0 + hg.ey0, ix0 = tx0 + hg.ex0;
    for (int base = tid; base < total; base += 64 * kHaloWaves * kHaloLd) {
      uint4 v[kHaloLd];
      uint4 yv[BWD ? kHaloLd : 1];
      int dst[kHaloLd], cc[kHaloLd];
#pragma unroll
      for (int u = 0; u < kHaloLd; ++u) {
        v[u] = make_uint4(0, 0, 0, 0);
        if constexpr (BWD) yv[u] = make_uint4(0, 0, 0, 0);
        dst[u] = -1;
        cc[u] = -1;
        if (base + u * 64 * kHaloWaves < total) {
          const int iy = iy0 + hy, ix = ix0 + hx;
          dst[u] = __mul24(hp, hg.pitch) + c8 * 8;
          if ((unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW) {
            const int ci = c8 * 8;
            const int pix = iy * g.IW + ix;
            cc[u] = c8;
            if (g.Gi == 1) {
              v[u] = ldg4(xim0 + pix * g.Cgi + ci);
              if constexpr (BWD) yv[u] = ldg4(yim0 + pix * g.Cgi + ci);
            } else {
              const int gi = fdiv(ci, g.Cgi, hg.inv_cgi);
              const int off = img * g.Cgi + (pix * g.Cgi + ci - __mul24(gi, g.Cgi));
              v[u] = ldg4(s_xp[gi] + off);
              if constexpr (BWD) {
                const uint16_t* yp = s_yp[gi];
                if (yp != nullptr) yv[u] = ldg4(yp + off);
                else cc[u] = -1;   // a plain gradient group: stored as loaded
              }
            }
          }
        }
        // advance the cursor by 256 elements
        c8 += hg.st_r;
        const int carry = c8 >= C8c ? 1 : 0;
        c8 -= carry * C8c;
        hp += hg.st_q + carry;
        hx += hg.st_b + carry;
        hy += hg.st_a;
        if (hx >= hg.HWD) { hx -= hg.HWD; ++hy; }
      }
      if constexpr (BWD) {
#pragma unroll
        for (int u = 0; u < kHaloLd; ++u) {
          if (dst[u] < 0) continue;
          uint4 val = v[u];
          if (cc[u] >= 0) val = bwd8(val, yv[u], s_coef + cc[u] * 8, Cip);
          st_tile(dst[u], val);
        }
      } else if (!BNE && hg.xtab) {
#pragma unroll
        for (int u = 0; u < kHaloLd; ++u) {
          if (dst[u] < 0) continue;
          uint4 val = v[u];
          if (cc[u] >= 0) {
            const float* cp = s_coef + cc[u] * 8;
            const float4 s0 = *reinterpret_cast<const float4*>(cp), s1 = *reinterpret_cast<const float4*>(cp + 4);
            const float4 h0 = *reinterpret_cast<const float4*>(cp + Cip);
            const float4 h1 = *reinterpret_cast<const float4*>(cp + Cip + 4);
            const float4 l0 = *reinterpret_cast<const float4*>(cp + 2 * Cip);
            const float4 l1 = *reinterpret_cast<const float4*>(cp + 2 * Cip + 4);
            float f[8];
            unpack8(val, f);
            f[0] = fmaxf(fmaf(f[0], s0.x, h0.x), l0.x); f[1] = fmaxf(fmaf(f[1], s0.y, h0.y), l0.y);
            f[2] = fmaxf(fmaf(f[2], s0.z, h0.z), l0.z); f[3] = fmaxf(fmaf(f[3], s0.w, h0.w), l0.w);
            f[4] = fmaxf(fmaf(f[4], s1.x, h1.x), l1.x); f[5] = fmaxf(fmaf(f[5], s1.y, h1.y), l1.y);
            f[6] = fmaxf(fmaf(f[6], s1.z, h1.z), l1.z); f[7] = fmaxf(fmaf(f[7], s1.w, h1.w), l1.w);
            val = pack8(f);
          }
          st_tile(dst[u], val);
        }
      } else {
#pragma unroll
        for (int u = 0; u < kHaloLd; ++u)
          if (dst[u] >= 0) st_tile(dst[u], v[u]);
      }
    }
    __syncthreads();
  }

  for (int rg = 0; rg < n_rg; ++rg) {
    const int co0 = rg * 16 * MI;
    const uint16_t* wrow[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) wrow[i] = a.w + (long)(co0 + 16 * i + lr) * g.Kp + (CHUNKED ? 0 : 8 * lg);
    f32x4_t acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    for (int ch = 0; ch < hg.nch; ++ch) {
      const int c0 = ch * hg.CC;
      if (CHUNKED) {
        if (ch > 0) __syncthreads();           // every wave is done reading the previous chunk
        store_batch(pv, pd, pyv, pcc);
        __syncthreads();
        if (ch + 1 < hg.nch) load_batch(c0 + hg.CC, tid, pv, pd, pyv, pcc);   // in flight during the MFMAs
        if (!BNE && hg.xtab) {   // prologues are forward-only, BNE data-gradient-only
          xform_pass(c0);
          __syncthreads();
        }
      }
      auto load_a = [&](uint4* A, int ks) {
        if (CHUNKED) {
          const int ua = s_ua[4 * ks + lg];
#pragma unroll
          for (int i = 0; i < MI; ++i)
            A[i] = ua >= 0 ? *reinterpret_cast<const uint4*>(wrow[i] + ua + c0) : make_uint4(0, 0, 0, 0);
        } else if (PIPE) {
#pragma unroll
          for (int i = 0; i < MI; ++i)
            A[i] = *reinterpret_cast<const uint4*>(sA + (co0 + 16 * i + lr) * pitchA + 32 * ks + 8 * lg);
        } else {
#pragma unroll
          for (int i = 0; i < MI; ++i) A[i] = *reinterpret_cast<const uint4*>(wrow[i] + 32 * ks);
        }
      };
      uint4 A[MI];
      load_a(A, 0);
      for (int ks = 0; ks < hg.KS; ++ks) {
        uint4 An[MI];
        const bool more = ks + 1 < hg.KS;
        if (more) load_a(An, ks + 1);
        const int ub = s_ub[4 * ks + lg];
        uint4 B[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) B[j] = *reinterpret_cast<const uint4*>(tile + halo_phys(pb[j] + ub, smask) + hcopy);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16x16x32(A[i], B[j], acc[i][j]);
        if (more) {
#pragma unroll
          for (int i = 0; i < MI; ++i) A[i] = An[i];
        }
      }
    }
    // epilogue: bias, bf16 round (v_cvt_pk), 8-B NHWC stores, per-row (sum, sum^2) of the stored
    // values reduced over the 16 pixel lanes with DPP row adds.
    uint16_t* yb[MI];
    float bv[MI][4], cs[MI][4], cq[MI][4];
    bool rv[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int cb = co0 + 16 * i + 4 * lg;
      const int og = cb < rows ? cb / g.Cgo : 0, cl = cb - og * g.Cgo;
      yb[i] = cb < rows ? a.y[og] + img * g.Cgo + cl : nullptr;   // per-image base
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        rv[i][r] = cb < rows && cl + r < g.Cgo_l;
        bv[i][r] = (a.bias != nullptr && rv[i][r]) ? a.bias[cl + r] : 0.f;
        cs[i][r] = 0.f; cq[i][r] = 0.f;
      }
    }
    if constexpr (BNE) {
      // BN-backward partials (Go == 1: the row IS the channel).  Row group i outer: the NJ y vectors
      // of a row group are issued together, so HBM latency is exposed once per row group, not per
      // pixel group (the stores in between would otherwise order every y load behind them).
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if (yb[i] == nullptr) continue;
        const int cb = co0 + 16 * i + 4 * lg;
        const float4 sc = *reinterpret_cast<const float4*>(a.bn_coef + cb);
        const float4 sh = *reinterpret_cast<const float4*>(a.bn_coef + g.Cgo + cb);
        const float4 mu = *reinterpret_cast<const float4*>(a.bn_coef + 2 * g.Cgo + cb);
        const bool rl = a.bn_relu != 0;
        uint2 yy[NJ];
        int pmj[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int p = (wave * NJ + j) * 16 + lr;
          const int ty = ty0 + (p >> hg.tw_shift), tx = tx0 + (p & (hg.TW - 1));
          pmj[j] = (ty < g.OH && tx < g.OW) ? (ty * g.OW + tx) * g.Cgo : -1;
          yy[j] = pmj[j] >= 0 ? *reinterpret_cast<const uint2*>(a.bn_y + img * g.Cgo + cb + pmj[j]) : make_uint2(0, 0);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if (pmj[j] < 0) continue;
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = rv[i][r] ? acc[i][j][r] + bv[i][r] : 0.f;
          const uint32_t lo = pack2(o[0], o[1]), hi = pack2(o[2], o[3]);
          *reinterpret_cast<uint2*>(yb[i] + pmj[j]) = make_uint2(lo, hi);
          const float v0 = __uint_as_float(lo << 16), v1 = __uint_as_float(lo & 0xffff0000u);
          const float v2 = __uint_as_float(hi << 16), v3 = __uint_as_float(hi & 0xffff0000u);
          const float y0 = __uint_as_float(yy[j].x << 16), y1 = __uint_as_float(yy[j].x & 0xffff0000u);
          const float y2 = __uint_as_float(yy[j].y << 16), y3 = __uint_as_float(yy[j].y & 0xffff0000u);
          const float g0 = (!rl || fmaf(y0, sc.x, sh.x) > 0.f) ? v0 : 0.f;
          const float g1 = (!rl || fmaf(y1, sc.y, sh.y) > 0.f) ? v1 : 0.f;
          const float g2 = (!rl || fmaf(y2, sc.z, sh.z) > 0.f) ? v2 : 0.f;
          const float g3 = (!rl || fmaf(y3, sc.w, sh.w) > 0.f) ? v3 : 0.f;
          cs[i][0] += g0; cs[i][1] += g1; cs[i][2] += g2; cs[i][3] += g3;
          cq[i][0] += g0 * (y0 - mu.x); cq[i][1] += g1 * (y1 - mu.y);
          cq[i][2] += g2 * (y2 - mu.z); cq[i][3] += g3 * (y3 - mu.w);
        }
      }
    } else if (a.bias == nullptr) {
      // No bias (every BN'd conv): the packed weights' padding rows are zero, so padding channels
      // accumulate exactly 0 and are stored as-is; the BN partials come from the fp32 accumulators
      // (the statistics of the stored bf16 values up to rounding noise) -- 11 instead of ~23 VALU ops
      // per 4-channel quad in this issue-bound epilogue.  Parity note: the reference's autocast BN takes
      // its statistics from the bf16 conv output itself; here they come from the fp32 values before
      // that rounding (|diff| <= 2^-9 relative per element, unbiased), so the BN normalises the stored
      // bf16 tensor with statistics of slightly different values -- a systematic, tolerance-level
      // deviation (the bias path and the GEMM kernel use the rounded values).
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int p = (wave * NJ + j) * 16 + lr;
        const int ty = ty0 + (p >> hg.tw_shift), tx = tx0 + (p & (hg.TW - 1));
        if (ty >= g.OH || tx >= g.OW) continue;
        const int pm = (ty * g.OW + tx) * g.Cgo;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          if (yb[i] == nullptr) continue;
          f32x4_t v = acc[i][j];
          if (a.accum) {   // y += conv(x) (sibling launches' data-gradients)
            const uint2 ov = *reinterpret_cast<const uint2*>(yb[i] + pm);
            v[0] += __uint_as_float(ov.x << 16); v[1] += __uint_as_float(ov.x & 0xffff0000u);
            v[2] += __uint_as_float(ov.y << 16); v[3] += __uint_as_float(ov.y & 0xffff0000u);
          }
          *reinterpret_cast<uint2*>(yb[i] + pm) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            cs[i][r] += v[r];
            cq[i][r] = fmaf(v[r], v[r], cq[i][r]);
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int p = (wave * NJ + j) * 16 + lr;
        const int ty = ty0 + (p >> hg.tw_shift), tx = tx0 + (p & (hg.TW - 1));
        if (ty >= g.OH || tx >= g.OW) continue;
        const int pm = (ty * g.OW + tx) * g.Cgo;   // OH == IH, OW == IW; within the image
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          if (yb[i] == nullptr) continue;
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = rv[i][r] ? acc[i][j][r] + bv[i][r] : 0.f;
          if (a.accum) {
            const uint2 ov = *reinterpret_cast<const uint2*>(yb[i] + pm);
            o[0] += __uint_as_float(ov.x << 16); o[1] += __uint_as_float(ov.x & 0xffff0000u);
            o[2] += __uint_as_float(ov.y << 16); o[3] += __uint_as_float(ov.y & 0xffff0000u);
          }
          const uint32_t lo = pack2(o[0], o[1]), hi = pack2(o[2], o[3]);
          *reinterpret_cast<uint2*>(yb[i] + pm) = make_uint2(lo, hi);
          const float v0 = __uint_as_float(lo << 16), v1 = __uint_as_float(lo & 0xffff0000u);
          const float v2 = __uint_as_float(hi << 16), v3 = __uint_as_float(hi & 0xffff0000u);
          cs[i][0] += v0; cs[i][1] += v1; cs[i][2] += v2; cs[i][3] += v3;
          cq[i][0] += v0 * v0; cq[i][1] += v1 * v1; cq[i][2] += v2 * v2; cq[i][3] += v3 * v3;
        }
      }
    }
    if (a.stat_part != nullptr) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int cb = co0 + 16 * i + 4 * lg;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float s = row16_sum(cs[i][r]), q = row16_sum(cq[i][r]);
          if (lr == 0 && cb + r < rows) {
            s_stat[(wave * 2 + 0) * rows + cb + r] += s;
            s_stat[(wave * 2 + 1) * rows + cb + r] += q;
          }
        }
      }
    }
  }
  }   // tile loop
  if (a.stat_part != nullptr) {
    __syncthreads();
    for (int c = tid; c < rows; c += 64 * kHaloWaves) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int wv = 0; wv < kHaloWaves; ++wv) { s += s_stat[(wv * 2 + 0) * rows + c]; q += s_stat[(wv * 2 + 1) * rows + c]; }
      a.stat_part[((long)wgid * 2 + 0) * rows + c] = s;
      a.stat_part[((long)wgid * 2 + 1) * rows + c] = q;
    }
  }
}

template <int MI, int NJ, int WPX, bool TRANS, bool PH, bool BNE = false>
void launch_igemm(const ConvArgs& a, const PhaseArgs& pa, hipStream_t s) {
  const long M = PH ? (long)a.g.N * pa.OHp * pa.OWp : (long)a.g.N * a.g.OH * a.g.OW;
  const long blocks = (long)cdiv(M, 16 * NJ * WPX) * cdiv(a.g.Go * a.g.Cgo, 16 * MI);
  hipLaunchKernelGGL((conv_igemm_kernel<MI, NJ, WPX, TRANS, PH, BNE>), dim3((unsigned)blocks), dim3(64 * WPX), 0, s, a,
                     pa);
}

template <bool TRANS, bool BNE = false>
void dispatch_igemm(const ConvArgs& a, int mi, int nj, int wpx, hipStream_t s) {
  const PhaseArgs pa{};
#define CASE(MI_, NJ_, WPX_)                                                  \
  if (mi == MI_ && nj == NJ_ && wpx == WPX_) { launch_igemm<MI_, NJ_, WPX_, TRANS, false, BNE>(a, pa, s); return; }
  CASE(1, 4, 4) CASE(2, 4, 4) CASE(3, 4, 4) CASE(4, 4, 4)
  CASE(1, 4, 2) CASE(2, 4, 2) CASE(3, 4, 2) CASE(4, 4, 2)
  CASE(1, 4, 1) CASE(2, 4, 1) CASE(3, 4, 1) CASE(4, 4, 1)
  CASE(1, 8, 4) CASE(2, 8, 4) CASE(1, 8, 2) CASE(2, 8, 2) CASE(1, 8, 1) CASE(2, 8, 1)
#undef CASE
}

void dispatch_phase(const ConvArgs& a, const PhaseArgs& pa, int mi, int wpx, hipStream_t s) {
#define CASEP(MI_, WPX_) if (mi == MI_ && wpx == WPX_) { launch_igemm<MI_, 4, WPX_, false, true>(a, pa, s); return; }
  CASEP(1, 4) CASEP(2, 4) CASEP(3, 4) CASEP(4, 4)
  CASEP(1, 2) CASEP(2, 2) CASEP(3, 2) CASEP(4, 2)
  CASEP(1, 1) CASEP(2, 1) CASEP(3, 1) CASEP(4, 1)
#undef CASEP
}

int grid1d(long total) {
  long b = (total + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

// Tile choice: co tile = 16*MI rows, MI in 1..4, minimising padded MFMA rows + per-tile re-read cost.
int conv_pick_mi(int rows) {
  int best = 1;
  long best_cost = 1L << 60;
  for (int mi = 1; mi <= 4; ++mi) {
    const int tiles = cdiv(rows, 16 * mi);
    const long cost = (long)tiles * 16 * mi + 8L * tiles;
    if (cost < best_cost) { best_cost = cost; best = mi; }
  }
  return best;
}

// packed weight rows: enough for the row-group size of every kernel variant (the halo PIPE kernels
// pick MI in {1, 3}; the others conv_pick_mi); rows past `rows` stay zero
int conv_rows_alloc(int rows) {
  int r = 0;
  for (int mi = 1; mi <= 4; ++mi) r = std::max(r, cdiv(rows, 16 * mi) * 16 * mi);
  // + one zero row of slack: the LDS-tiled GEMM's last K stage reads up to 32 elements past Kp of the
  // last real row (conv_gemm.hip stage(): times a zero B operand, but it must stay inside the buffer)
  return r + 1;
}

// PIPE (persistent, next tile prefetched in registers) runs the MI 3 / NJ 4 row groups of thin-halo 3x3
// convs (the L2 3x3s): there its 256-pixel tile is also the standard kernel's; measured slower for the
// MI <= 2 layers (which lose their 512-pixel tile) and the 1x7 / dilated halos.  MI 3 at NJ 4 leaves room
// for the kPipeLd prefetch registers at 2 blocks/CU without spilling (NJ 8 and MI 4 spill there).
static size_t pipe_a_bytes(int rows, int mi, int ks) {
  return (size_t)cdiv(rows, 16 * mi) * 16 * mi * (4 * ks + 1) * 16;
}

// Pixels per wave: 128 (NJ = 8) for narrow outputs (<= 32 rows) with plenty of pixels -- amortises the
// weight-fragment loads and doubles the MFMAs per pixel-operand load; else 64.
static int conv_pick_nj(const ConvGeom& g, int mi) {
  const long M = (long)g.N * g.OH * g.OW;
  return (mi <= 2 && M >= 256L * 1024) ? 8 : 4;
}

static int conv_pick_wpx(const ConvGeom& g, int mi, int nj) {
  const long M = (long)g.N * g.OH * g.OW;
  const long co_tiles = cdiv(g.Go * g.Cgo, 16 * mi);
  for (int wpx = 4; wpx > 1; wpx >>= 1)
    if ((long)cdiv(M, 16 * nj * wpx) * co_tiles >= 1024) return wpx;
  return 1;
}

// Halo-kernel eligibility + tile geometry.  Pixel tile = 4 waves x NJ x 16 pixels (NJ = 8 for
// MI <= 2, else 4); TW in {16, 32, 64} minimising (tiles) x (stores + halo loads).  The input is staged
// whole (one chunk, LDS <= 64 KB) or -- single row group only -- in chunks of CC channels (CC | Cip, a
// chunk's staging fits the kHaloLd registers per thread), widest CC first.
static int halo_nj(int mi, bool pipe = false) { return (mi <= 2 && !pipe) ? 8 : 4; }
static int halo_tile_elems(int HH, int HWD, int pitch, bool split) {
  const int e = HH * HWD * pitch;
  return split ? 2 * ((e + 63) / 64) * 64 : e;
}
static size_t halo_lds_bytes(int HH, int HWD, int pitch, int rows, bool split = false) {
  return (size_t)halo_tile_elems(HH, HWD, pitch, split) * 2 + (size_t)kHaloWaves * 2 * rows * 4;
}

// split-bank image policy (halo_phys): 0 never, 1 (default) where it keeps the blocks per CU of the single
// image, 2 wherever it fits the LDS cap (A/B: conv_set_halo_split)
static int g_halo_split = 1;
void conv_set_halo_split(int mode) { g_halo_split = mode; }

// LDS cap of a halo tile + its stats rows + the prologue table.  Two blocks per CU hold up to ~76 KB of
// dynamic LDS each (160 KB per CU minus the static tap tables); 64 KB measured 0.6 % slower per step
// (L3 3x3 d3 leaves the gather kernel: fwd 0.49 -> 0.28 ms).
static size_t halo_tile_cap() { return (size_t)kHaloTileKB * 1024; }

// Fallback row-group size of the halo kernel.  conv_pick_mi's MI <= 2 comes with the 512-pixel (NJ = 8)
// tile; when that tile (+ halo) does not fit the LDS cap the 256-pixel MI 3/4 tile often does, instead of
// falling back to the gather kernel (L3 5x3x3 + 3x1x1 DUCK split, 216 rows x 72 ch: 1.46 -> 0.57 ms fwd).
static int halo_fallback_mi(int rows) {
  if (conv_pick_mi(rows) > 2) return 0;
  return cdiv(rows, 48) * 48 <= cdiv(rows, 64) * 64 ? 3 : 4;
}

// bwd: a data-gradient launch with the BN-backward prologue: its [5][Cip] table instead of [3][Cip], no PIPE
static bool conv_halo_ok(const ConvGeom& g, bool trans, HaloGeom& hg, bool bwd = false) {
  if (trans || g.stride != 1 || g.OH != g.IH || g.OW != g.IW) return false;
  const int rows = g.Go * g.Cgo;
  if (rows > kHaloMaxRows || g.T > 16) return false;
  const int Cip = g.Gi * g.Cgi;
  if (Cip % 8 != 0 || g.Cgi % 8 != 0) return false;
  int ey0 = 0, ey1 = 0, ex0 = 0, ex1 = 0;
  for (int t = 0; t < g.T; ++t) {
    ey0 = std::min(ey0, g.dy[t]); ey1 = std::max(ey1, g.dy[t]);
    ex0 = std::min(ex0, g.dx[t]); ex1 = std::max(ex1, g.dx[t]);
  }
  const int C8 = Cip / 8;
  // try 0: PIPE (whole input, halo tile within the prefetch registers); try 1: the standard kernels;
  // try 2: the standard kernel with the fallback 256-pixel row group (halo_fallback_mi).  (Round 2's
  // 128-pixel NJ = 2 tile for wider inputs measured 1.3 % slower per step, profiles/r02/conv_bench_L4_small.log,
  // and is gone, as are the weights-in-LDS WL variant (neutral, profiles/r03/conv_bench_v10_wl_*) and the
  // 256-pixel NJ = 4 tiles for MI <= 2.)
  const bool pipe_ok = !bwd && conv_pick_mi(rows) == 3 && ey1 - ey0 == 2 && ex1 - ex0 == 2;
  const size_t tab = (bwd ? 20 : 12) * (size_t)Cip;   // prologue table bytes
  for (int attempt = pipe_ok ? 0 : 1; attempt < 3; ++attempt) {
  const bool pipe = attempt == 0;
  if (attempt == 2 && halo_fallback_mi(rows) == 0) continue;
  const int mi = pipe ? 3 : (attempt == 1 ? conv_pick_mi(rows) : halo_fallback_mi(rows));
  const int n_rg = cdiv(rows, 16 * mi);
  const int nj = halo_nj(mi, pipe);
  const int tp = kHaloWaves * nj * 16;
  for (int pass = 0; pass < (pipe ? 1 : 2); ++pass) {   // pass 0: whole input; 1: chunks
    if (pass == 1 && (n_rg != 1 || bwd)) break;   // BWD: no chunked staging (its y registers would spill)
    for (int d = C8; d >= 1; --d) {
      if (C8 % d != 0) continue;
      if (pass == 0 && d != C8) break;
      if (pass == 1 && d == C8) continue;
      const int pitch = 8 * ((d & 1) ? d : d + 1);   // odd number of 16-B slots per pixel
      const int ks = cdiv(g.T * d, 4);
      if (ks > kHaloMaxKS) continue;
      double best = 1e30;
      bool found = false;
      for (int tw = 16; tw <= 64; tw *= 2) {
        const int th = tp / tw;
        const int HH = th + ey1 - ey0, HWD = tw + ex1 - ex0;
        // (+ the prologue table a deferred-BN input adds: two blocks per CU must still fit)
        if (halo_lds_bytes(HH, HWD, pitch, rows) + tab > halo_tile_cap()) continue;
        if (pass == 1 && HH * HWD * d > 64 * kHaloWaves * kHaloLd) continue;
        if (pipe && HH * HWD * d > 64 * kHaloWaves * kPipeLd) continue;
        if (pipe && halo_lds_bytes(HH, HWD, pitch, rows) + tab + pipe_a_bytes(rows, mi, ks) >
                        (size_t)kPipeMaxLds) continue;
        const double tiles = (double)cdiv(g.OH, th) * cdiv(g.OW, tw);
        const double cost = tiles * ((double)tp * rows / 8.0 + 0.5 * (double)HH * HWD * C8);
        if (cost < best) {
          best = cost; found = true;
          hg.TH = th; hg.TW = tw; hg.HH = HH; hg.HWD = HWD;
        }
      }
      if (!found) continue;
      hg.ey0 = ey0; hg.ex0 = ex0;
      hg.tiles_y = cdiv(g.OH, hg.TH);
      hg.tiles_x = cdiv(g.OW, hg.TW);
      hg.pitch = pitch;
      hg.CC = 8 * d;
      hg.nch = C8 / d;
      hg.KS = ks;
      hg.mi = mi;
      hg.nj = nj;
      hg.pipe = pipe ? 1 : 0;
      hg.tw_shift = hg.TW == 16 ? 4 : (hg.TW == 32 ? 5 : 6);
      hg.inv_c8 = 1.0f / (float)d;
      {
        const int step = 64 * kHaloWaves;
        hg.st_q = step / d; hg.st_r = step % d;
        hg.st_a = hg.st_q / hg.HWD; hg.st_b = hg.st_q % hg.HWD;
      }
      hg.inv_hwd = 1.0f / (float)hg.HWD;
      hg.inv_cgi = 1.0f / (float)g.Cgi;
      hg.split = 0;
      if (!pipe && g_halo_split > 0) {
        const size_t one = halo_lds_bytes(hg.HH, hg.HWD, pitch, rows) + tab + 2048;   // + static tables
        const size_t two = halo_lds_bytes(hg.HH, hg.HWD, pitch, rows, true) + tab + 2048;
        const int reg_blocks = pass == 1 ? 2 : ((mi <= 2 && nj <= 4) ? 4 : 3);   // conv_halo_kernel's bounds
        const int per_cu = 160 * 1024;
        const bool fits = two - 2048 <= halo_tile_cap();
        const bool keeps = (int)(per_cu / two) >= std::min(reg_blocks, (int)(per_cu / one));
        hg.split = fits && (g_halo_split == 2 || keeps) ? 1 : 0;
      }
      hg.tile_elems = halo_tile_elems(hg.HH, hg.HWD, pitch, hg.split != 0);
      return true;
    }
  }
  }   // attempt
  return false;
}

static size_t halo_lds(const HaloGeom& hg, int rows) {
  return halo_lds_bytes(hg.HH, hg.HWD, hg.pitch, rows, hg.split != 0);
}

static int g_halo_mode = -1;   // -1: from MSP_CONV_HALO (default on), 0: off, 1: on

static bool halo_enabled() {
  if (g_halo_mode < 0) { const char* e = getenv("MSP_CONV_HALO"); g_halo_mode = (e == nullptr || e[0] != '0') ? 1 : 0; }
  return g_halo_mode == 1;
}

void conv_set_halo(int on) { g_halo_mode = on ? 1 : 0; }
bool conv_uses_halo(const ConvGeom& g, bool trans, bool bwd) {
  HaloGeom hg;
  if (conv_gemm_ok(g, trans)) return false;   // wide inputs: the LDS-tiled GEMM kernel (conv_gemm.hip)
  return halo_enabled() && conv_halo_ok(g, trans, hg, bwd);
}

static long halo_blocks(const ConvGeom& g, const HaloGeom& hg) {
  const long nt = (long)g.N * hg.tiles_y * hg.tiles_x;
  return hg.pipe ? std::min(nt, (long)kPipeGrid) : nt;   // PIPE: persistent grid
}

// Stat partial rows of a forward launch = its pixel-tile count, which depends on the kernel the launch
// takes: ``trans`` (a strided transposed conv, conv_igemm's flag) never takes the GEMM or halo kernel --
// sizing its rows by conv_gemm_ok(g, false) under-allocated the gather kernel's rows (out-of-bounds stat
// writes: UNet / Linknet deconvs from 64 input channels up)
long conv_stat_blocks(const ConvGeom& g, bool trans, bool bwd, bool bne) {
  HaloGeom hg;
  if (!trans && conv_gemm_ok(g, false)) return conv_gemm_stat_blocks(g);
  if (!trans && !bwd && !bne && conv_fwd_fused_ok(g)) return conv_fwd_fused_blocks(g);
  if (!trans && halo_enabled() && conv_halo_ok(g, false, hg, bwd)) return halo_blocks(g, hg);
  const int mi = conv_pick_mi(g.Go * g.Cgo);
  const int nj = conv_pick_nj(g, mi);
  const int wpx = conv_pick_wpx(g, mi, nj);
  const long M = (long)g.N * g.OH * g.OW;
  return cdiv(M, 16 * nj * wpx);
}

static int g_phase_mode = -1;   // -1: from MSP_CONV_PHASE (default on), 0: off, 1: on

static bool phase_enabled() {
  if (g_phase_mode < 0) { const char* e = getenv("MSP_CONV_PHASE"); g_phase_mode = (e == nullptr || e[0] != '0') ? 1 : 0; }
  return g_phase_mode == 1;
}

void conv_set_phase(int on) { g_phase_mode = on ? 1 : 0; }

// Strided TRANS conv as stride x stride phase launches (see PhaseArgs): each phase gathers only its
// valid taps over its output sub-grid; a phase without taps writes zeros.
static void conv_igemm_phased(const ConvArgs& a, int mi, hipStream_t s) {
  const ConvGeom& g = a.g;
  const int st = g.stride, Cip = g.Gi * g.Cgi;
  // kernel width of the packed tap table (t = r*KW + c): T over the number of distinct row offsets
  int nrow = 0;
  for (int t = 0; t < g.T; ++t) {
    bool seen = false;
    for (int u = 0; u < t; ++u) seen |= g.dy[u] == g.dy[t];
    nrow += seen ? 0 : 1;
  }
  const int KW = nrow > 0 ? g.T / nrow : 1;
  for (int py = 0; py < st; ++py)
    for (int px = 0; px < st; ++px) {
      PhaseArgs pa{};
      pa.s = st; pa.py = py; pa.px = px;
      pa.OHp = (g.OH - py + st - 1) / st;
      pa.OWp = (g.OW - px + st - 1) / st;
      if (pa.OHp <= 0 || pa.OWp <= 0) continue;
      ConvArgs b = a;
      int tv = 0;
      for (int t = 0; t < g.T; ++t) {
        const int ay = py + g.dy[t], ax = px + g.dx[t];
        if (((ay % st) + st) % st != 0 || ((ax % st) + st) % st != 0) continue;
        b.g.dy[tv] = ay / st;   // exact division
        b.g.dx[tv] = ax / st;
        pa.tA[tv] = t;
        ++tv;
      }
      b.g.T = tv;
      pa.Kloop = (tv * Cip + 31) / 32 * 32;
      ConvGeom gp = b.g;
      gp.OH = pa.OHp; gp.OW = pa.OWp;
      // wide inputs (>= 64 channels): the phase as a stride-1 conv on the LDS-DMA GEMM kernel, which stores
      // into the phase's pixels of the full output (round 6; the gather kernel stays for narrow inputs)
      if (tv > 0) {
        ConvArgs bg = b;
        bg.g.OH = pa.OHp; bg.g.OW = pa.OWp; bg.g.stride = 1;
        if (conv_gemm_phase(bg, pa.tA, KW, st, py, px, g.OH, g.OW, s) == 0) continue;
      }
      dispatch_phase(b, pa, mi, conv_pick_wpx(gp, mi, 4), s);
    }
}

int conv_igemm(const ConvArgs& a, bool trans, hipStream_t s) {
  const int mi = conv_pick_mi(a.g.Go * a.g.Cgo);
  if (trans && a.g.stride > 1 && a.stat_part == nullptr && phase_enabled()) {
    conv_igemm_phased(a, mi, s);
    return 0;
  }
  bool bwd = false;
  for (int i = 0; i < a.g.Gi; ++i) bwd |= a.gy[i] != nullptr;
  if (bwd && (trans || conv_gemm_ok(a.g, trans))) return 7;
  if (conv_gemm_ok(a.g, trans)) return conv_gemm(a, s);
  // the 17-channel level's forward convs: persistent staging / compute-wave kernel (conv_bwd.hip)
  if (!trans && !bwd && a.bn_y == nullptr && !a.accum && a.g.Gi == 1 && a.g.Go <= 2 && conv_fwd_fused_ok(a.g))
    return conv_fwd_fused(a, s);
  HaloGeom hg;
  if (halo_enabled() && conv_halo_ok(a.g, trans, hg, bwd)) {
    const unsigned blocks = (unsigned)halo_blocks(a.g, hg);
    const bool pipe = hg.pipe != 0;
    const int hmi = hg.mi;
    hg.xtab = 0;
    for (int i = 0; i < a.g.Gi; ++i) hg.xtab |= a.xc[i] != nullptr;
    if (hg.xtab && a.bn_y != nullptr) return 3;   // BN prologue (forward) and BN epilogue (dgrad) never meet
    if (bwd && hg.xtab) return 3;
    const size_t lds = halo_lds(hg, a.g.Go * a.g.Cgo) +
                       (bwd ? 5 * 4 * (size_t)a.g.Gi * a.g.Cgi : (hg.xtab ? 3 * 4 * (size_t)a.g.Gi * a.g.Cgi : 0)) +
                       (hg.pipe ? pipe_a_bytes(a.g.Go * a.g.Cgo, hg.mi, hg.KS) : 0);
    // BNE: the BN-backward epilogue is its own instantiation, so plain launches keep their registers.
    // The prologue table may take the dynamic LDS past 64 KB: opted into once per instantiation,
    // before any graph capture (the first call of every shape runs eagerly).
#define HC_LAUNCH_(K_)                                                                                       \
    {                                                                                                        \
      static bool lds_attr = false;                                                                          \
      if (!lds_attr) {                                                                                       \
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&K_), hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  kHaloMaxLds);                                                              \
        lds_attr = true;                                                                                     \
      }                                                                                                      \
      hipLaunchKernelGGL((K_), dim3(blocks), dim3(64 * kHaloWaves), lds, s, a, hg);                         \
    }
#define HB_(MI_, BNE_)                                                                                       \
    if (bwd && hmi == MI_ && bne == BNE_) {                                                                  \
      HC_LAUNCH_((conv_halo_kernel<MI_, (MI_ <= 2 ? 8 : 4), false, BNE_, false, true>))                     \
      return 0;                                                                                              \
    }
#define HC_(MI_, BNE_)                                                                                       \
    if (hmi == MI_ && bne == BNE_ && !pipe) {                                                                \
      if (hg.nch > 1) HC_LAUNCH_((conv_halo_kernel<MI_, (MI_ <= 2 ? 8 : 4), true, BNE_>))                   \
      else HC_LAUNCH_((conv_halo_kernel<MI_, (MI_ <= 2 ? 8 : 4), false, BNE_>))                             \
      return 0;                                                                                              \
    }
#define HP_(BNE_)                                                                                            \
    if (hmi == 3 && bne == BNE_ && pipe) {                                                                   \
      HC_LAUNCH_((conv_halo_kernel<3, 4, false, BNE_, true>))                                                \
      return 0;                                                                                              \
    }
    const bool bne = a.bn_y != nullptr;
    HB_(1, false) HB_(2, false) HB_(3, false) HB_(4, false) HB_(1, true) HB_(2, true) HB_(3, true) HB_(4, true)
    HC_(1, false) HC_(2, false) HC_(3, false) HC_(4, false) HC_(1, true) HC_(2, true) HC_(3, true) HC_(4, true)
    HP_(false) HP_(true)
    return 4;   // no instantiation for this row-group size
#undef HB_
#undef HP_
#undef HC_
#undef HC_LAUNCH_
  }
  const int nj = conv_pick_nj(a.g, mi);
  const int wpx = conv_pick_wpx(a.g, mi, nj);
  if (trans) dispatch_igemm<true>(a, mi, nj, wpx, s);
  else if (a.bn_y != nullptr) dispatch_igemm<false, true>(a, mi, nj, wpx, s);
  else dispatch_igemm<false>(a, mi, nj, wpx, s);
  return 0;
}

const char* conv_error_string(int rc) {
  switch (rc) {
    case 0: return "ok";
    case 1: return "conv_gemm: no instantiation for the chosen tile configuration";
    case 2: return "conv_gemm: deferred-BN input prologue on the GEMM path (materialise wide inputs first)";
    case 3: return "halo conv: a BN prologue (forward) and a BN epilogue (data-gradient) in one launch";
    case 4: return "halo conv: no instantiation for this row-group size";
    case 5: return "wgrad: no instantiation for the chosen tile configuration";
    case 6: return "wgrad (halo / gather): no instantiation for this plan";
    case 7: return "BN-backward prologue: only the stride-1 halo kernels rebuild dY (resolve the gradient first)";
  }
  return "conv: unknown error";
}

static size_t wgrad_halo_lds(const DwTile& tl, int ncb) {
  return ((size_t)256 * ncb + (size_t)tl.HH * tl.HWd) * DW_CH * 2;
}

static bool wgrad_halo_ok(const ConvGeom& g, DwTile& tl) {
  if (g.stride != 1 || g.T > 9) return false;
  int ey0 = 0, ey1 = 0, ex0 = 0, ex1 = 0;
  for (int t = 0; t < g.T; ++t) {
    ey0 = std::min(ey0, g.dy[t]); ey1 = std::max(ey1, g.dy[t]);
    ex0 = std::min(ex0, g.dx[t]); ex1 = std::max(ex1, g.dx[t]);
  }
  if (g.OH != g.IH || g.OW != g.IW) return false;
  // TW = 32 unless the image is narrow enough that 16 wastes less
  tl.TW = (cdiv(g.OW, 16) * 16 < cdiv(g.OW, 32) * 32) ? 16 : 32;
  tl.tw_shift = tl.TW == 16 ? 4 : 5;
  tl.TH = 256 / tl.TW;
  tl.ey0 = ey0; tl.ex0 = ex0;
  tl.HH = tl.TH + ey1 - ey0;
  tl.HWv = tl.TW + ex1 - ex0;
  tl.HWd = cdiv(tl.HWv, 16) * 16;
  tl.inv_hwv = 1.0f / (float)tl.HWv;
  tl.tiles_y = cdiv(g.OH, tl.TH);
  tl.tiles_x = cdiv(g.OW, tl.TW);
  if (tl.HH * tl.HWv > kDwMaxHalo) return false;   // the pipelined staging registers
  return wgrad_halo_lds(tl, 1) <= 64 * 1024;
}

// Weight-gradient launch plan.  Both kernels split the pixel reduction over blocks (split-K) and
// write one fp32 dW slab per split; unpack_wgrad sums the slabs in a fixed order -> bitwise
// deterministic weight gradients (SURVEY §5 race detection / §7.4), no atomics and no zero-fill.
// (No hipMemsetAsync anywhere in the step: inside a captured hipGraph it was measured NOT to re-run
// on replays >= 2, which left stale graph-pool bytes in the old atomic replicas.)
struct WgradPlan {
  bool halo;
  DwTile tl;
  int ncb, gx, gy, gz, k_t, co_t;
  long nsplit, ntiles;
};

// bwd: the dY groups carry the BN-backward prologue (at most 2 co sub-tiles per block: the y staging
// registers of a third spill)
static WgradPlan wgrad_plan(const ConvGeom& g, bool trans, bool bwd = false) {
  WgradPlan P{};
  const int KT = g.T * g.Gi * g.Cgi;
  const int rows = g.Go * g.Cgo;
  if (!trans && wgrad_halo_ok(g, P.tl)) {
    P.halo = true;
    P.ntiles = (long)g.N * P.tl.tiles_y * P.tl.tiles_x;
    // co sub-tiles per block: as many as the LDS budget allows (<= kDwMaxNcb)
    const int max_ncb = kDwMaxNcb;
    // The kernel's time ~ (tiles per block) x (co sub-tiles per block) + the per-tile input-halo
    // staging that NCB sub-tiles share: with the grid fixed at ~split_target blocks, cost ~ gy * ncb +
    // kDwHaloCost * gy.  Balancing matters: 4 sub-tiles (a 5-group fused conv at 24 ch) run as 2 + 2,
    // not 3 + 1 (the 3-sub-tile blocks would set the kernel time).
    const int nst = cdiv(rows, DW_CH);
    int ncb = 1;
    double best = 1e30;
    for (int c = 1; c <= std::min(bwd ? 2 : max_ncb, nst); ++c) {
      if (c > 1 && wgrad_halo_lds(P.tl, c) > (size_t)kDwMaxLds) break;
      const int gy = cdiv(nst, c);
      const double cost = (double)gy * c + kDwHaloCost * gy;
      if (cost <= best) { best = cost; ncb = c; }   // ties -> the larger NCB (fewer input passes)
    }
    P.ncb = ncb;
    P.gy = cdiv(rows, DW_CH * ncb);
    P.gz = cdiv(g.Gi * g.Cgi, DW_CH);
    // one 8-wave block per CU that software-pipelines its tiles beats more, shorter-lived blocks for a
    // single ci sub-tile (L1: 256 vs 512 blocks 0.642 vs 0.648 ms); with two ci sub-tiles (L2, 40 ch)
    // 512 blocks win (3x3 0.442 -> 0.417 ms, fused-8 2.59 -> 2.43 ms at bs128;
    // profiles/r03/conv_bench_v9_dw_split_bs128.log)
    const long target = (P.gz >= 2 ? 2 : 1) * kDwSplitTarget;   // blocks in the grid
    P.nsplit = std::max(1L, std::min(target / ((long)P.gy * P.gz), P.ntiles));
    return P;
  }
  P.halo = false;
  const long M = (long)g.N * g.OH * g.OW;
  const long nchunks = (M + WG_M - 1) / WG_M;
  P.co_t = rows <= 32 ? 32 : 64;
  // K tile 64: the 64 x 128 tile needs 149 VGPRs + 128 AGPRs (1 wave/SIMD); at 64 (2 waves/SIMD) the
  // strided weight gradients run 1.5-1.9x faster (L1 3x3 s2: 50 -> 76 TF, L3: 80 -> 155 TF; step +0.8 %,
  // profiles/r02/conv_bench_s2_wgrad_kt.log).
  P.k_t = 64;
  P.gx = cdiv(KT, P.k_t);
  P.gy = cdiv(rows, P.co_t);
  P.nsplit = std::max(1L, std::min(2048L / ((long)P.gx * P.gy), nchunks));
  return P;
}

// number of dW slabs the caller allocates ([nsplit][rows][KT] fp32) and unpack_wgrad sums
// Weight-gradient kernel choice: the LDS-tiled GEMM (conv_wgrad_gemm.hip) for wide inputs, strided and
// 1x1 convs; the halo kernel keeps the narrow stride-1 multi-tap layers (17/34-channel DUCK levels), where
// staging the input halo once per tile beats re-gathering it per tap (profiles/r03/conv_bench_v4_*.log:
// L1 3x3 with a BN prologue 0.64 ms halo vs 1.23 ms GEMM; L5 fused-5 2.21 -> 0.69 ms on the GEMM).
static bool wgrad_use_gemm(const ConvGeom& g, bool trans) {
  if (!conv_wgrad_gemm_ok(g, trans)) return false;
  if (conv_wgrad_gemm_mode() == 2) return true;
  DwTile tl;
  return g.Cgi >= 64 || g.stride > 1 || g.T == 1 || trans || !wgrad_halo_ok(g, tl);
}

int conv_wgrad_replicas(const ConvGeom& g, bool trans, bool bwd, bool pro) {
  if (wgrad_use_gemm(g, trans)) return conv_wgrad_gemm_replicas(g, pro);
  return (int)wgrad_plan(g, trans, bwd).nsplit;
}

bool conv_wgrad_uses_halo(const ConvGeom& g, bool trans) {
  return !wgrad_use_gemm(g, trans) && wgrad_plan(g, trans).halo;
}

int conv_wgrad(const uint16_t* const* dy, const uint16_t* const* x, float* dw, const ConvGeom& g, bool trans,
               const float* const* xc, unsigned xrelu, hipStream_t s, const uint16_t* const* gy,
               const float* const* gs, const float* const* gk, unsigned grelu) {
  const int KT = g.T * g.Gi * g.Cgi;
  WgradPtrs P{};
  for (int i = 0; i < g.Go; ++i) P.dy[i] = dy[i];
  for (int i = 0; i < g.Gi; ++i) P.x[i] = x[i];
  bool pro = false;
  for (int i = 0; i < g.Gi; ++i) { P.xc[i] = xc != nullptr ? xc[i] : nullptr; pro |= P.xc[i] != nullptr; }
  P.xrelu = xrelu;
  bool bwd = false;
  for (int i = 0; i < g.Go; ++i) {
    P.gy[i] = gy != nullptr ? gy[i] : nullptr;
    P.gs[i] = gs != nullptr ? gs[i] : nullptr;
    P.gk[i] = gk != nullptr ? gk[i] : nullptr;
    bwd |= P.gy[i] != nullptr;
  }
  P.grelu = grelu;
  if (bwd && !conv_wgrad_uses_halo(g, trans)) return 7;
  if (wgrad_use_gemm(g, trans)) return conv_wgrad_gemm(P, dw, g, pro, s);
  const WgradPlan W = wgrad_plan(g, trans, bwd);
  if (W.halo) {
    const size_t lds = wgrad_halo_lds(W.tl, W.ncb);
    // pair slots per wave of ci chunk z (the kernel's pair table): full 16-channel halves one tap each, a
    // half with 8 real channels two taps (24-channel L1: 14 pairs, 2 slots instead of 3; the 8-channel image:
    // 5 pairs, 1 slot).  Consecutive chunks with the same count share a launch: a 40-channel input's second
    // chunk (5 pairs) runs 1 slot per wave instead of the first chunk's 3.
    auto chunk_npw = [&](int z) {
      const int R = std::min(DW_CH, g.Gi * g.Cgi - z * DW_CH);
      return cdiv((R >> 4) * g.T + ((R & 15) ? (g.T + 1) / 2 : 0), kDwWaves);
    };
    const int ncb = W.ncb;
    // > 64 KB of dynamic LDS (gfx950 has 160 KB per CU) is opted into once per instantiation, before any
    // graph capture (the first call of every shape runs eagerly)
    auto launch = [&](int npw, int z0, int nz) -> bool {
      dim3 grid((unsigned)W.nsplit, W.gy, nz);
#define HW_(N_, C_, B_)                                                                                  \
      if (npw == N_ && ncb == C_ && bwd == B_) {                                                        \
        static bool lds_attr = false;                                                                   \
        if (!lds_attr) {                                                                                \
          (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_halo_kernel<N_, C_, B_>), \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kDwMaxLds);             \
          lds_attr = true;                                                                              \
        }                                                                                               \
        hipLaunchKernelGGL((conv_wgrad_halo_kernel<N_, C_, B_>), grid, dim3(64 * kDwWaves), lds, s, P, dw, g, \
                           W.tl, KT, W.ntiles, z0);                                                     \
        return true;                                                                                    \
      }
      HW_(1, 1, false) HW_(2, 1, false) HW_(3, 1, false) HW_(1, 2, false) HW_(2, 2, false) HW_(3, 2, false)
      HW_(1, 3, false) HW_(2, 3, false) HW_(3, 3, false)
      HW_(1, 1, true) HW_(2, 1, true) HW_(3, 1, true) HW_(1, 2, true) HW_(2, 2, true) HW_(3, 2, true)
#undef HW_
      return false;
    };
    for (int z = 0; z < W.gz;) {
      const int npw = chunk_npw(z);
      int z1 = z + 1;
      while (z1 < W.gz && chunk_npw(z1) == npw) ++z1;
      if (!launch(npw, z, z1 - z)) return 6;
      z = z1;
    }
    return 0;
  }
  dim3 grid(W.gx, W.gy, (unsigned)W.nsplit);
#define WG(CO_, K_)                                                                                  \
  if (W.co_t == CO_ && W.k_t == K_) {                                                                \
    if (trans) hipLaunchKernelGGL((conv_wgrad_kernel<CO_, K_, true>), grid, dim3(256), 0, s, P, dw, g, KT); \
    else hipLaunchKernelGGL((conv_wgrad_kernel<CO_, K_, false>), grid, dim3(256), 0, s, P, dw, g, KT);      \
    return 0;                                                                                        \
  }
  WG(32, 64) WG(64, 64)
#undef WG
  return 6;
}

void pack_weight(const float* src, uint16_t* dst, int nrow, int nch, int T, int Cpk, int Kp, int t_base, int c_base,
                 long s_row, long s_ch, hipStream_t s) {
  const long total = (long)nrow * nch * T;
  hipLaunchKernelGGL(pack_weight_kernel, dim3(grid1d(total)), dim3(256), 0, s, src, dst, nrow, nch, T, Cpk, Kp, t_base,
                     c_base, s_row, s_ch);
}

void pack_batch(const int64_t* jobs, const int* prefix, int njobs, int total_blocks, hipStream_t s) {
  if (njobs <= 0 || total_blocks <= 0) return;
  hipLaunchKernelGGL(pack_batch_kernel, dim3(total_blocks), dim3(256), 0, s, jobs, prefix, njobs);
}

int pack_per_block() { return kPackPerBlock; }

void unpack_wgrad(const float* src, float* dst, int nrow, int nch, int T, int Cpk, int Ktot, int t_base, int c_base,
                  long s_row, long s_ch, bool accumulate, int nrep, long rep_stride, hipStream_t s) {
  const long total = (long)nrow * nch * T;
  hipLaunchKernelGGL(unpack_wgrad_kernel, dim3((unsigned)((total + 63) / 64)), dim3(64 * kUnpackGroups), 0, s, src,
                     dst, nrow, nch, T, Cpk, Ktot, t_base, c_base, s_row, s_ch, accumulate ? 1 : 0, nrep, rep_stride);
}

// ------------------------------------------------------------------------------------------------
// Host-side launch-planner self-check (SURVEY §5 race detection / sanitizers): enumerates DUCKNet /
// UNet / ResNet layer geometries and verifies the invariants every kernel launch relies on -- LDS
// budgets, staging-register capacities, tile coverage, cursor-step decompositions, weight-row
// padding and grid sizes.  Pure host code (no launch, no device): built with AddressSanitizer +
// UBSan on the host side by tools/sanitize/run.sh and run on the CPU by tests/test_sanitize_cpu.py.
int conv_plan_selfcheck(int verbose) {
  int bad = 0;
  auto fail = [&](const char* what, const ConvGeom& g) {
    ++bad;
    if (verbose)
      fprintf(stderr, "plan check FAILED: %s (N=%d %dx%d Gi=%d Cgi=%d Go=%d Cgo=%d T=%d s=%d)\n", what, g.N, g.IH,
              g.IW, g.Gi, g.Cgi, g.Go, g.Cgo, g.T, g.stride);
  };
  struct K { int kh, kw, dil; };
  const K ks[] = {{3, 3, 1}, {3, 3, 2}, {3, 3, 3}, {1, 7, 1}, {7, 1, 1}, {1, 1, 1}, {2, 2, 1}, {7, 7, 1}};
  const int sizes[] = {352, 176, 88, 44, 22, 11, 7, 64, 33};
  const int chans[] = {8, 24, 40, 72, 136, 272, 544, 64, 128, 256, 512};
  long checked = 0;
  for (int hw : sizes)
    for (int cin : chans)
      for (int go : {1, 2, 8})
        for (int cout : {24, 40, 72, 136, 64})
          for (const K& k : ks)
            for (int stride : {1, 2}) {
              if (stride == 2 && k.dil != 1) continue;
              ConvGeom g{};
              g.N = 4; g.IH = hw; g.IW = hw; g.Gi = 1; g.Cgi = cin;
              const int ph = (k.kh / 2) * k.dil, pw = (k.kw / 2) * k.dil;
              g.OH = (hw + 2 * ph - k.dil * (k.kh - 1) - 1) / stride + 1;
              g.OW = (hw + 2 * pw - k.dil * (k.kw - 1) - 1) / stride + 1;
              if (g.OH < 1 || g.OW < 1) continue;
              g.Go = go; g.Cgo = cout; g.Cgo_l = cout;
              g.T = k.kh * k.kw;
              if (g.T > kMaxTaps) continue;
              for (int r = 0, t = 0; r < k.kh; ++r)
                for (int c = 0; c < k.kw; ++c, ++t) { g.dy[t] = r * k.dil - ph; g.dx[t] = c * k.dil - pw; }
              g.Kp = cdiv(g.T * cin, 32) * 32;
              g.stride = stride;
              ++checked;
              const int rows = g.Go * g.Cgo;
              HaloGeom hg{};
              if (conv_halo_ok(g, false, hg)) {
                const int C8 = cin / 8, d = hg.CC / 8;
                if (hg.nch * hg.CC != cin) fail("halo chunks do not tile the input channels", g);
                if ((long)hg.tiles_y * hg.TH < g.OH || (long)hg.tiles_x * hg.TW < g.OW) fail("halo tiles miss pixels", g);
                if (halo_lds(hg, rows) + 12 * (size_t)cin > halo_tile_cap()) fail("halo tile LDS over the cap", g);
                if (halo_lds(hg, rows) + 12 * (size_t)cin > (size_t)kHaloMaxLds) fail("halo LDS > opted-in maximum", g);
                if (hg.KS > kHaloMaxKS || hg.KS * 4 < g.T * d) fail("halo k-steps", g);
                if (((hg.pitch / 8) & 1) == 0) fail("halo pitch not an odd number of 16-B slots", g);
                if (hg.TW != (1 << hg.tw_shift)) fail("halo tw_shift", g);
                if (hg.st_q * d + hg.st_r != 64 * kHaloWaves || hg.st_a * hg.HWD + hg.st_b != hg.st_q)
                  fail("halo staging cursor step", g);
                const long total = (long)hg.HH * hg.HWD * d;
                if (hg.nch > 1 && total > 64L * kHaloWaves * kHaloLd) fail("chunk exceeds staging registers", g);
                if (hg.pipe) {
                  if (total > 64L * kHaloWaves * kPipeLd) fail("PIPE tile exceeds prefetch registers", g);
                  if (halo_lds(hg, rows) + 12 * (size_t)cin + pipe_a_bytes(rows, hg.mi, hg.KS) > (size_t)kPipeMaxLds)
                    fail("PIPE LDS budget", g);
                  if (hg.nch != 1 || C8 != d) fail("PIPE with channel chunks", g);
                }
                if (hg.nj != (hg.mi <= 2 && !hg.pipe ? 8 : 4) || (hg.pipe && hg.mi != 3))
                  fail("halo tile: no instantiation for this (MI, NJ, PIPE)", g);
                if (cdiv(rows, 16 * hg.mi) * 16 * hg.mi > conv_rows_alloc(rows)) fail("weight rows under-allocated", g);
                const long blocks = halo_blocks(g, hg);
                if (blocks < 1 || blocks > (1L << 31) - 1) fail("halo grid size", g);
                if (!conv_gemm_ok(g, false) && blocks != conv_stat_blocks(g, false, false, true))
                  fail("stat partial rows != launch grid", g);
                if (conv_fwd_fused_ok(g) && conv_stat_blocks(g) != conv_fwd_fused_blocks(g))
                  fail("fused forward stat rows != its grid", g);
              }
              if (cdiv(rows, 16 * conv_pick_mi(rows)) * 16 * conv_pick_mi(rows) > conv_rows_alloc(rows))
                fail("igemm weight rows under-allocated", g);
              const WgradPlan W = wgrad_plan(g, false);
              if (W.nsplit < 1) fail("wgrad split", g);
              if (W.halo) {
                if (W.nsplit > W.ntiles) fail("wgrad more splits than tiles", g);
                if (wgrad_halo_lds(W.tl, W.ncb) > (size_t)kDwMaxLds) fail("wgrad LDS budget", g);
                if ((long)W.tl.tiles_y * W.tl.TH < g.OH || (long)W.tl.tiles_x * W.tl.TW < g.OW) fail("wgrad tiles", g);
                if (W.tl.HH * W.tl.HWv > kDwMaxHalo) fail("wgrad halo exceeds staging registers", g);
              }
            }
  if (verbose) fprintf(stderr, "conv plan self-check: %ld geometries, %d violations\n", checked, bad);
  return bad;
}

