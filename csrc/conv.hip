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

template <int MI, int NJ, int WPX, bool TRANS>
__global__ __launch_bounds__(64 * WPX) void conv_igemm_kernel(ConvArgs a) {
  const ConvGeom& g = a.g;
  __shared__ int2 s_tap[kMaxTaps];
  __shared__ const uint16_t* s_x[kMaxGroups];
  __shared__ uint16_t* s_y[kMaxGroups];
  __shared__ float s_stat[WPX][2][16 * MI];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < kMaxTaps) s_tap[tid] = make_int2(g.dy[tid], g.dx[tid]);
  if (tid < kMaxGroups) { s_x[tid] = a.x[tid]; s_y[tid] = a.y[tid]; }
  __syncthreads();

  const long OHW = (long)g.OH * g.OW;
  const long M = (long)g.N * OHW;
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
      const int oh = r / g.OW, ow = r - (r / g.OW) * g.OW;
      pn[j] = n * IHW;
      ph[j] = TRANS ? oh : oh * g.stride;
      pw[j] = TRANS ? ow : ow * g.stride;
    } else {
      pn[j] = -1; ph[j] = 0; pw[j] = 0;
    }
  }
  const uint16_t* wrow[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) wrow[i] = a.w + (long)(co0 + 16 * i + lr) * g.Kp + 8 * lg;

  KPos kp = kpos_init(8 * lg, g);

  auto load_b = [&](uint4* B, const KPos& p) {
    const bool kval = p.t < g.T;
    const int2 d = kval ? s_tap[p.t] : make_int2(0, 0);
    const uint16_t* xb = s_x[kval ? p.gi : 0] + p.cl;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (pn[j] >= 0 && kval) {
        const int pix = in_pixel<TRANS>(pn[j], ph[j], pw[j], d, g);
        if (pix >= 0) v = *reinterpret_cast<const uint4*>(xb + (long)pix * g.Cgi);
      }
      B[j] = v;
    }
  };
  auto load_a = [&](uint4* A, int k0) {
#pragma unroll
    for (int i = 0; i < MI; ++i) A[i] = *reinterpret_cast<const uint4*>(wrow[i] + k0);
  };

  f32x4_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 A[MI], B[NJ];
  load_a(A, 0);
  load_b(B, kp);
  for (int k0 = 0; k0 < g.Kp; k0 += 32) {
    uint4 An[MI], Bn[NJ];
    const bool more = k0 + 32 < g.Kp;
    if (more) {
      kpos_advance(kp, 32, g);
      load_a(An, k0 + 32);
      load_b(Bn, kp);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16x16x32(A[i], B[j], acc[i][j]);
    if (more) {
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
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const long m = m0 + 16 * j + lr;
      if (m < M) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float o = (cl + r < g.Cgo_l) ? acc[i][j][r] + bv[r] : 0.f;
          v[r] = bf2f(f2bf(o));
          csum[i][r] += v[r];
          csq[i][r] += v[r] * v[r];
        }
        *reinterpret_cast<uint2*>(yb + m * g.Cgo) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
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
// summed through LDS, then across pixel splits with fp32 atomics into dW (zeroed by the caller).
constexpr int WG_M = 128;

typedef short s16x4_t __attribute__((ext_vector_type(4)));

DEVI uint2 tr_read(const uint16_t* p) {
  s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t __attribute__((address_space(3)))*)(p));
  union { s16x4_t s; uint2 u; } c; c.s = v; return c.u;
}

struct WgradPtrs { const uint16_t* dy[kMaxGroups]; const uint16_t* x[kMaxGroups]; };

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

  uint4 ra[A_V], rb[B_V];
  auto load = [&](long c) {
    const long mb = c * WG_M;
#pragma unroll
    for (int v = 0; v < A_V; ++v) {
      const long m = mb + a_r + A_RS * v;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (m < M && a_valid) val = *reinterpret_cast<const uint4*>(a_base + m * g.Cgo);
      ra[v] = val;
    }
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
        if (pix >= 0) val = *reinterpret_cast<const uint4*>(b_base + (long)pix * g.Cgi);
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
    for (int v = 0; v < B_V; ++v) *reinterpret_cast<uint4*>(&sB[(b_r + B_RS * v) * SB_LD + 8 * b_c8]) = rb[v];
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

  // sequential cross-wave accumulation in LDS (fp32 tile), then one atomic per element
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
  for (int e = tid; e < CO_T * K_T; e += 256) {
    const int ci = e / K_T, kj = e - (e / K_T) * K_T;
    const int co = co0 + ci, k = k0 + kj;
    if (co < rows && (co % g.Cgo) < g.Cgo_l && k < KT) atomicAdd(&dw[(long)co * KT + k], red[e]);
  }
}

// Halo-tiled weight gradient for stride-1 convs ("direct wgrad").  The gather kernel above reads
// every input pixel once per tap (a 9x im2col expansion through L2 for a 3x3); here a block stages an
// output tile of dY [TH x TW px][32 co] and the matching input HALO [(TH+eh) x (TW+ew) px][32 ci]
// in LDS ONCE, and every tap reads its shifted window of the halo with ds_read_b64_tr_b16 (each lane
// supplies its own pixel row address, so the shift is free).  Block output = dW[32 co][T taps][32 ci];
// the 4 waves own disjoint (tap, ci16) pairs, so no cross-wave reduction.  Blocks loop over pixel
// tiles (accumulating in registers) and finish with one fp32 atomic per output element.
constexpr int DW_CH = 32;               // co rows and ci channels per block
constexpr int DW_LD = DW_CH + 4;        // LDS pixel pitch (bf16 elems): 72 B, 8-B aligned

struct DwTile { int TH, TW, ey0, ex0, HH, HWd, tiles_y, tiles_x; };

constexpr int kDwLd = 8;

template <int NPW>
__global__ __launch_bounds__(256) void conv_wgrad_halo_kernel(WgradPtrs P, float* __restrict__ dw, ConvGeom g,
                                                              DwTile tl, int KT, long ntiles) {
  extern __shared__ __attribute__((aligned(16))) uint16_t dsm[];
  const int npx = tl.TH * tl.TW;
  const int nslice = (npx + 31) / 32;
  uint16_t* sY = dsm;                                    // [nslice*32 + 1][DW_LD] (last row = zeros)
  uint16_t* sX = dsm + (nslice * 32 + 1) * DW_LD;        // [HH*HWd][DW_LD]
  __shared__ int2 s_tap[kMaxTaps];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4, q = lr >> 2, p4 = lr & 3;
  const int co0 = blockIdx.y * DW_CH, ci0 = blockIdx.z * DW_CH;
  const int rows = g.Go * g.Cgo, Cip = g.Gi * g.Cgi;
  if (tid < kMaxTaps) s_tap[tid] = make_int2(g.dy[tid] - tl.ey0, g.dx[tid] - tl.ex0);
  // zero row for out-of-tile pixels
  if (tid < DW_LD) sY[nslice * 32 * DW_LD + tid] = 0;

  // per-thread loader roles: vector v = tid & 3 (8 channels), pixel = tid >> 2 (+ 64*i)
  const int vv = tid & 3, vp = tid >> 2;
  const int yco = co0 + 8 * vv;
  const bool y_ok = yco < rows;
  const int y_g = y_ok ? yco / g.Cgo : 0;
  const uint16_t* y_base = P.dy[y_g] + (yco - y_g * g.Cgo);
  const int xci = ci0 + 8 * vv;
  const bool x_ok = xci < Cip;
  const int x_g = x_ok ? xci / g.Cgi : 0;
  const uint16_t* x_base = P.x[x_g] + (xci - x_g * g.Cgi);

  f32x4_t acc[2][NPW];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NPW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int npairs = 2 * g.T;

  for (long tix = blockIdx.x; tix < ntiles; tix += gridDim.x) {
    const int per_img = tl.tiles_y * tl.tiles_x;
    const int n = (int)(tix / per_img);
    const int rem = (int)(tix - (long)n * per_img);
    const int y0 = (rem / tl.tiles_x) * tl.TH, x0 = (rem % tl.tiles_x) * tl.TW;
    __syncthreads();   // previous tile's LDS reads are done
    // ---- stage dY tile (pixels beyond the image -> 0) and the input halo (zero padding outside the
    // image); kDwLd loads in flight per thread before the LDS writes of each batch.
    const int nyp = nslice * 32, nh = tl.HH * tl.HWd;
    for (int base = vp; base < nyp + nh; base += 64 * kDwLd) {
      uint4 v[kDwLd];
      int dst[kDwLd];
#pragma unroll
      for (int u = 0; u < kDwLd; ++u) {
        const int e = base + 64 * u;
        v[u] = make_uint4(0, 0, 0, 0);
        dst[u] = -1;
        if (e < nyp) {
          const int px = e;
          const int ty = px / tl.TW, tx = px - (px / tl.TW) * tl.TW;
          const int oy = y0 + ty, ox = x0 + tx;
          dst[u] = px * DW_LD + 8 * vv;
          if (px < npx && y_ok && oy < g.OH && ox < g.OW)
            v[u] = *reinterpret_cast<const uint4*>(y_base + ((long)n * g.OH * g.OW + (long)oy * g.OW + ox) * g.Cgo);
        } else if (e < nyp + nh) {
          const int hp = e - nyp;
          const int hy = hp / tl.HWd, hx = hp - (hp / tl.HWd) * tl.HWd;
          const int iy = y0 + hy + tl.ey0, ix = x0 + hx + tl.ex0;
          dst[u] = (int)(sX - sY) + hp * DW_LD + 8 * vv;
          if (x_ok && (unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW)
            v[u] = *reinterpret_cast<const uint4*>(x_base + ((long)n * g.IH * g.IW + (long)iy * g.IW + ix) * g.Cgi);
        }
      }
#pragma unroll
      for (int u = 0; u < kDwLd; ++u) {
        if (dst[u] < 0) continue;
        *reinterpret_cast<uint2*>(&sY[dst[u]]) = make_uint2(v[u].x, v[u].y);
        *reinterpret_cast<uint2*>(&sY[dst[u] + 4]) = make_uint2(v[u].z, v[u].w);
      }
    }
    __syncthreads();
    for (int sl = 0; sl < nslice; ++sl) {
      const int plo = 32 * sl + 8 * lg + q, phi = plo + 4;
      const int ylo = plo < npx ? plo : nslice * 32, yhi = phi < npx ? phi : nslice * 32;
      uint4 fa[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint2 lo = tr_read(&sY[ylo * DW_LD + 16 * i + 4 * p4]);
        const uint2 hi = tr_read(&sY[yhi * DW_LD + 16 * i + 4 * p4]);
        fa[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
      const int plc = plo < npx ? plo : 0, phc = phi < npx ? phi : 0;
      const int lty = plc / tl.TW, ltx = plc - lty * tl.TW;
      const int hty = phc / tl.TW, htx = phc - hty * tl.TW;
#pragma unroll
      for (int j = 0; j < NPW; ++j) {
        const int pr = wave + 4 * j;
        if (pr < npairs) {
          const int t = pr >> 1, cf = pr & 1;
          const int2 d = s_tap[t];
          const int xlo = (lty + d.x) * tl.HWd + ltx + d.y;
          const int xhi = (hty + d.x) * tl.HWd + htx + d.y;
          const uint2 lo = tr_read(&sX[xlo * DW_LD + 16 * cf + 4 * p4]);
          const uint2 hi = tr_read(&sX[xhi * DW_LD + 16 * cf + 4 * p4]);
          const uint4 fb = make_uint4(lo.x, lo.y, hi.x, hi.y);
          acc[0][j] = mfma16x16x32(fa[0], fb, acc[0][j]);
          acc[1][j] = mfma16x16x32(fa[1], fb, acc[1][j]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    const int pr = wave + 4 * j;
    if (pr >= npairs) continue;
    const int t = pr >> 1, cf = pr & 1;
    const int ci = ci0 + 16 * cf + lr;
    if (ci >= Cip) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + 16 * i + 4 * lg + r;
        if (co < rows && (co % g.Cgo) < g.Cgo_l) atomicAdd(&dw[(long)co * KT + t * Cip + ci], acc[i][j][r]);
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

__global__ void unpack_wgrad_kernel(const float* __restrict__ src, float* __restrict__ dst, int nrow, int nch, int T,
                                    int Cpk, int Ktot, int t_base, int c_base, long s_row, long s_ch, int accumulate) {
  const long total = (long)nrow * nch * T;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int t = (int)(i % T);
    const long rc = i / T;
    const int c = (int)(rc % nch);
    const int row = (int)(rc / nch);
    const float v = src[(long)row * Ktot + (t_base + t) * Cpk + c_base + c];
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
struct HaloGeom { int TH, TW, HH, HWD, ey0, ex0, tiles_y, tiles_x, pitch, KC; };

constexpr int kHaloMaxKC = 64;
constexpr int kHaloWaves = 4;
constexpr int kHaloMaxRows = 512;
constexpr int kHaloLd = 8;

template <int MI, int NJ>
__global__ __launch_bounds__(64 * kHaloWaves, 3) void conv_halo_kernel(ConvArgs a, HaloGeom hg) {
  extern __shared__ uint4 halo_smem[];
  uint16_t* tile = reinterpret_cast<uint16_t*>(halo_smem);
  __shared__ int s_koff[kHaloMaxKC * 4];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int Cip = g.Gi * g.Cgi, C8 = Cip >> 3;
  const int rows = g.Go * g.Cgo;
  // per-wave (sum, sum^2) rows after the tile (+ zero slot): [kHaloWaves][2][rows] fp32
  float* s_stat = reinterpret_cast<float*>(tile + hg.HH * hg.HWD * hg.pitch + 8);

  // XCD-aware bijective remap: neighbouring tiles (shared halo rows) land on one XCD's L2.
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xq = nwg / 8, xr = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + orig / 8;
  const int per_img = hg.tiles_y * hg.tiles_x;
  const int n = wgid / per_img;
  const int trem = wgid - n * per_img;
  const int ty0 = (trem / hg.tiles_x) * hg.TH, tx0 = (trem % hg.tiles_x) * hg.TW;

  // ---- stage the halo tile: 16 B per element, kHaloLd loads in flight per thread before any LDS
  // write (a load->store loop would serialise one HBM latency per iteration).
  const int hpx = hg.HH * hg.HWD;
  const long img = (long)n * g.IH * g.IW;
  const int total = hpx * C8;
  for (int base = tid; base < total; base += 64 * kHaloWaves * kHaloLd) {
    uint4 v[kHaloLd];
    int dst[kHaloLd];
#pragma unroll
    for (int u = 0; u < kHaloLd; ++u) {
      const int idx = base + u * 64 * kHaloWaves;
      v[u] = make_uint4(0, 0, 0, 0);
      dst[u] = -1;
      if (idx < total) {
        const int hp = idx / C8, c8 = idx - hp * C8;
        const int hy = hp / hg.HWD, hx = hp - hy * hg.HWD;
        const int iy = ty0 + hg.ey0 + hy, ix = tx0 + hg.ex0 + hx;
        dst[u] = hp * hg.pitch + c8 * 8;
        if ((unsigned)iy < (unsigned)g.IH && (unsigned)ix < (unsigned)g.IW) {
          const int ci = c8 * 8, gi = ci / g.Cgi, cl = ci - gi * g.Cgi;
          v[u] = *reinterpret_cast<const uint4*>(a.x[gi] + (img + (long)iy * g.IW + ix) * g.Cgi + cl);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kHaloLd; ++u)
      if (dst[u] >= 0) *reinterpret_cast<uint4*>(tile + dst[u]) = v[u];
  }
  const int zero_off = hpx * hg.pitch;  // one zeroed 16-B slot for k beyond T*Cip
  if (tid == 0) *reinterpret_cast<uint4*>(tile + zero_off) = make_uint4(0, 0, 0, 0);
  for (int e = tid; e < hg.KC * 4; e += 64 * kHaloWaves) {
    const int kk = 32 * (e >> 2) + 8 * (e & 3);
    int off = -1;
    if (kk < g.T * Cip) {
      const int t = kk / Cip, ci = kk - t * Cip;
      off = ((g.dy[t] - hg.ey0) * hg.HWD + (g.dx[t] - hg.ex0)) * hg.pitch + ci;
    }
    s_koff[e] = off;
  }
  __syncthreads();

  int pb[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int p = (wave * NJ + j) * 16 + lr;
    const int ty = p / hg.TW, tx = p - (p / hg.TW) * hg.TW;
    pb[j] = (ty * hg.HWD + tx) * hg.pitch;
  }

  const int n_rg = (rows + 16 * MI - 1) / (16 * MI);
  for (int rg = 0; rg < n_rg; ++rg) {
    const int co0 = rg * 16 * MI;
    const uint16_t* wrow[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) wrow[i] = a.w + (long)(co0 + 16 * i + lr) * g.Kp + 8 * lg;
    f32x4_t acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    uint4 A[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) A[i] = *reinterpret_cast<const uint4*>(wrow[i]);
    for (int kc = 0; kc < hg.KC; ++kc) {
      uint4 An[MI];
      const bool more = kc + 1 < hg.KC;
      if (more) {
#pragma unroll
        for (int i = 0; i < MI; ++i) An[i] = *reinterpret_cast<const uint4*>(wrow[i] + 32 * (kc + 1));
      }
      const int ko = s_koff[kc * 4 + lg];
      uint4 B[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) B[j] = *reinterpret_cast<const uint4*>(tile + (ko >= 0 ? pb[j] + ko : zero_off));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16x16x32(A[i], B[j], acc[i][j]);
      if (more) {
#pragma unroll
        for (int i = 0; i < MI; ++i) A[i] = An[i];
      }
    }
    // epilogue: bias, bf16 round, 8-B NHWC stores, per-row (sum, sum^2) of the stored values
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      float cs[4] = {0.f, 0.f, 0.f, 0.f}, cq[4] = {0.f, 0.f, 0.f, 0.f};
      const int cb = co0 + 16 * i + 4 * lg;
      if (cb < rows) {
        const int og = cb / g.Cgo, cl = cb - (cb / g.Cgo) * g.Cgo;
        uint16_t* yb = a.y[og] + cl;
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = (a.bias != nullptr && cl + r < g.Cgo_l) ? a.bias[cl + r] : 0.f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int p = (wave * NJ + j) * 16 + lr;
          const int ty = ty0 + p / hg.TW, tx = tx0 + p % hg.TW;
          if (ty >= g.OH || tx >= g.OW) continue;
          const long pm = img + (long)ty * g.OW + tx;   // OH == IH, OW == IW
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float o = (cl + r < g.Cgo_l) ? acc[i][j][r] + bv[r] : 0.f;
            v[r] = bf2f(f2bf(o));
            cs[r] += v[r];
            cq[r] += v[r] * v[r];
          }
          *reinterpret_cast<uint2*>(yb + pm * g.Cgo) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
      }
      if (a.stat_part != nullptr) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float s = cs[r], q = cq[r];
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
          if (lr == 0 && cb + r < rows) { s_stat[(wave * 2 + 0) * rows + cb + r] = s; s_stat[(wave * 2 + 1) * rows + cb + r] = q; }
        }
      }
    }
  }
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

template <int MI, int NJ, int WPX, bool TRANS>
void launch_igemm(const ConvArgs& a, hipStream_t s) {
  const long M = (long)a.g.N * a.g.OH * a.g.OW;
  const long blocks = (long)cdiv(M, 16 * NJ * WPX) * cdiv(a.g.Go * a.g.Cgo, 16 * MI);
  hipLaunchKernelGGL((conv_igemm_kernel<MI, NJ, WPX, TRANS>), dim3((unsigned)blocks), dim3(64 * WPX), 0, s, a);
}

template <bool TRANS>
void dispatch_igemm(const ConvArgs& a, int mi, int nj, int wpx, hipStream_t s) {
#define CASE(MI_, NJ_, WPX_)                                                  \
  if (mi == MI_ && nj == NJ_ && wpx == WPX_) { launch_igemm<MI_, NJ_, WPX_, TRANS>(a, s); return; }
  CASE(1, 4, 4) CASE(2, 4, 4) CASE(3, 4, 4) CASE(4, 4, 4)
  CASE(1, 4, 2) CASE(2, 4, 2) CASE(3, 4, 2) CASE(4, 4, 2)
  CASE(1, 4, 1) CASE(2, 4, 1) CASE(3, 4, 1) CASE(4, 4, 1)
  CASE(1, 8, 4) CASE(2, 8, 4) CASE(1, 8, 2) CASE(2, 8, 2) CASE(1, 8, 1) CASE(2, 8, 1)
#undef CASE
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

int conv_rows_alloc(int rows) { const int mi = conv_pick_mi(rows); return cdiv(rows, 16 * mi) * 16 * mi; }

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
// MI <= 2, else 4); TW in {16, 32, 64} chosen to minimise (padded tile area) x (halo overhead).
static int halo_nj(int mi) { return mi <= 2 ? 8 : 4; }

static bool conv_halo_ok(const ConvGeom& g, bool trans, HaloGeom& hg) {
  if (trans || g.stride != 1 || g.OH != g.IH || g.OW != g.IW) return false;
  const int rows = g.Go * g.Cgo;
  if (rows > kHaloMaxRows || g.T > kMaxTaps) return false;
  const int Cip = g.Gi * g.Cgi;
  if (Cip % 8 != 0 || g.Cgi % 8 != 0) return false;
  const int KC = g.Kp / 32;
  if (KC > kHaloMaxKC || g.Kp % 32 != 0) return false;
  int ey0 = 0, ey1 = 0, ex0 = 0, ex1 = 0;
  for (int t = 0; t < g.T; ++t) {
    ey0 = std::min(ey0, g.dy[t]); ey1 = std::max(ey1, g.dy[t]);
    ex0 = std::min(ex0, g.dx[t]); ex1 = std::max(ex1, g.dx[t]);
  }
  const int mi = conv_pick_mi(rows);
  const int tp = kHaloWaves * halo_nj(mi) * 16;
  int c8 = Cip / 8;
  if ((c8 & 1) == 0) ++c8;
  const int pitch = 8 * c8;
  double best = 1e30;
  bool found = false;
  for (int tw = 16; tw <= 64; tw *= 2) {
    const int th = tp / tw;
    const int HH = th + ey1 - ey0, HWD = tw + ex1 - ex0;
    const size_t lds = ((size_t)HH * HWD * pitch + 8) * 2 + (size_t)kHaloWaves * 2 * rows * 4;
    if (lds > 64 * 1024) continue;
    const double tiles = (double)cdiv(g.OH, th) * cdiv(g.OW, tw);
    const double cost = tiles * ((double)tp + 0.5 * (double)HH * HWD);   // stores + halo loads
    if (cost < best) {
      best = cost; found = true;
      hg.TH = th; hg.TW = tw; hg.HH = HH; hg.HWD = HWD;
    }
  }
  if (!found) return false;
  hg.ey0 = ey0; hg.ex0 = ex0;
  hg.tiles_y = cdiv(g.OH, hg.TH);
  hg.tiles_x = cdiv(g.OW, hg.TW);
  hg.pitch = pitch;
  hg.KC = KC;
  return true;
}

static size_t halo_lds(const HaloGeom& hg, int rows) {
  return ((size_t)hg.HH * hg.HWD * hg.pitch + 8) * 2 + (size_t)kHaloWaves * 2 * rows * 4;
}

static int g_halo_mode = -1;   // -1: from MSP_CONV_HALO (default on), 0: off, 1: on

static bool halo_enabled() {
  if (g_halo_mode < 0) { const char* e = getenv("MSP_CONV_HALO"); g_halo_mode = (e == nullptr || e[0] != '0') ? 1 : 0; }
  return g_halo_mode == 1;
}

void conv_set_halo(int on) { g_halo_mode = on ? 1 : 0; }
bool conv_uses_halo(const ConvGeom& g, bool trans) {
  HaloGeom hg;
  return halo_enabled() && conv_halo_ok(g, trans, hg);
}

long conv_stat_blocks(const ConvGeom& g) {
  HaloGeom hg;
  if (halo_enabled() && conv_halo_ok(g, false, hg)) return (long)g.N * hg.tiles_y * hg.tiles_x;
  const int mi = conv_pick_mi(g.Go * g.Cgo);
  const int nj = conv_pick_nj(g, mi);
  const int wpx = conv_pick_wpx(g, mi, nj);
  const long M = (long)g.N * g.OH * g.OW;
  return cdiv(M, 16 * nj * wpx);
}

void conv_igemm(const ConvArgs& a, bool trans, hipStream_t s) {
  const int mi = conv_pick_mi(a.g.Go * a.g.Cgo);
  HaloGeom hg;
  if (halo_enabled() && conv_halo_ok(a.g, trans, hg)) {
    const unsigned blocks = (unsigned)((long)a.g.N * hg.tiles_y * hg.tiles_x);
    const size_t lds = halo_lds(hg, a.g.Go * a.g.Cgo);
#define HC_(MI_)                                                                                          \
    if (mi == MI_) {                                                                                      \
      hipLaunchKernelGGL((conv_halo_kernel<MI_, (MI_ <= 2 ? 8 : 4)>), dim3(blocks), dim3(64 * kHaloWaves), \
                         lds, s, a, hg);                                                                  \
      return;                                                                                             \
    }
    HC_(1) HC_(2) HC_(3) HC_(4)
#undef HC_
  }
  const int nj = conv_pick_nj(a.g, mi);
  const int wpx = conv_pick_wpx(a.g, mi, nj);
  if (trans) dispatch_igemm<true>(a, mi, nj, wpx, s);
  else dispatch_igemm<false>(a, mi, nj, wpx, s);
}

static bool wgrad_halo_ok(const ConvGeom& g, DwTile& tl) {
  if (g.stride != 1 || g.T > 9) return false;
  int ey0 = 0, ey1 = 0, ex0 = 0, ex1 = 0;
  for (int t = 0; t < g.T; ++t) {
    ey0 = std::min(ey0, g.dy[t]); ey1 = std::max(ey1, g.dy[t]);
    ex0 = std::min(ex0, g.dx[t]); ex1 = std::max(ex1, g.dx[t]);
  }
  if (g.OH != g.IH || g.OW != g.IW) return false;
  const int nx = cdiv(g.OW, 32);
  tl.TW = cdiv(g.OW, nx);
  tl.TH = std::max(1, std::min(g.OH, 256 / tl.TW));
  tl.ey0 = ey0; tl.ex0 = ex0;
  tl.HH = tl.TH + ey1 - ey0;
  tl.HWd = tl.TW + ex1 - ex0;
  tl.tiles_y = cdiv(g.OH, tl.TH);
  tl.tiles_x = cdiv(g.OW, tl.TW);
  const int nslice = cdiv(tl.TH * tl.TW, 32);
  const size_t lds = ((size_t)(nslice * 32 + 1) + (size_t)tl.HH * tl.HWd) * DW_LD * 2;
  return lds <= 64 * 1024;
}

void conv_wgrad(const uint16_t* const* dy, const uint16_t* const* x, float* dw, const ConvGeom& g, bool trans,
                hipStream_t s) {
  const int KT = g.T * g.Gi * g.Cgi;
  const int rows = g.Go * g.Cgo;
  WgradPtrs P{};
  for (int i = 0; i < g.Go; ++i) P.dy[i] = dy[i];
  for (int i = 0; i < g.Gi; ++i) P.x[i] = x[i];
  (void)hipMemsetAsync(dw, 0, sizeof(float) * (size_t)rows * KT, s);
  DwTile tl{};
  if (!trans && wgrad_halo_ok(g, tl)) {
    const long ntiles = (long)g.N * tl.tiles_y * tl.tiles_x;
    const int gy = cdiv(rows, DW_CH), gz = cdiv(g.Gi * g.Cgi, DW_CH);
    long nsplit = 1536 / ((long)gy * gz);
    if (nsplit < 1) nsplit = 1;
    if (nsplit > ntiles) nsplit = ntiles;
    const int nslice = cdiv(tl.TH * tl.TW, 32);
    const size_t lds = ((size_t)(nslice * 32 + 1) + (size_t)tl.HH * tl.HWd) * DW_LD * 2;
    dim3 grid((unsigned)nsplit, gy, gz);
    const int npw = cdiv(2 * g.T, 4);
#define HW_(N_) if (npw == N_) { hipLaunchKernelGGL((conv_wgrad_halo_kernel<N_>), grid, dim3(256), lds, s, P, dw, g, tl, KT, ntiles); return; }
    HW_(1) HW_(2) HW_(3) HW_(4) HW_(5)
#undef HW_
  }
  const long M = (long)g.N * g.OH * g.OW;
  const long nchunks = (M + WG_M - 1) / WG_M;
  const int co_t = rows <= 32 ? 32 : 64;
  const int k_t = KT <= 64 ? 64 : 128;
  const int gx = cdiv(KT, k_t), gy = cdiv(rows, co_t);
  long target = 2048 / ((long)gx * gy);
  if (target < 1) target = 1;
  if (target > nchunks) target = nchunks;
  dim3 grid(gx, gy, (unsigned)target);
#define WG(CO_, K_)                                                                                  \
  if (co_t == CO_ && k_t == K_) {                                                                    \
    if (trans) hipLaunchKernelGGL((conv_wgrad_kernel<CO_, K_, true>), grid, dim3(256), 0, s, P, dw, g, KT); \
    else hipLaunchKernelGGL((conv_wgrad_kernel<CO_, K_, false>), grid, dim3(256), 0, s, P, dw, g, KT);      \
    return;                                                                                          \
  }
  WG(32, 64) WG(32, 128) WG(64, 64) WG(64, 128)
#undef WG
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
                  long s_row, long s_ch, bool accumulate, hipStream_t s) {
  const long total = (long)nrow * nch * T;
  hipLaunchKernelGGL(unpack_wgrad_kernel, dim3(grid1d(total)), dim3(256), 0, s, src, dst, nrow, nch, T, Cpk, Ktot,
                     t_base, c_base, s_row, s_ch, accumulate ? 1 : 0);
}
