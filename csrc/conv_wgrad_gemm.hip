// LDS-tiled weight-gradient GEMM for CDNA4 (gfx950) on v_mfma_f32_32x32x16_bf16.
//
//   dW[co][k] = sum_m  dY[m][co] * Xcol[m][k]      m = output pixel (the reduction), k = (tap t, input channel)
//
// Reference: the convolution_backward weight gradients of every conv (models/ducknet.py,
// models/modules.py:73-85).  Replaces the register-staged halo / gather weight-gradient kernels (conv.hip).
//
// Both operands are NHWC rows (channels contiguous per pixel) while the MFMA wants 8 consecutive PIXELS
// per lane: a stage of 64 pixels of each operand is DMA'd to LDS in its natural [pixel][channel] row
// order (global_load_lds_dwordx4; the im2col gather of X is the lane's source address, the zero padding
// a 64-B zero page) and the fragments are read with ds_read_b64_tr_b16 (the CDNA4 transposed read: 4
// pixel rows x 16 channels, delivered channel-per-lane).  The 64-B chunks of each LDS row are
// XOR-swizzled (source side) so the 4 rows of a transposed read sit in 4 distinct bank quarters.
// Block tile TCO co x TK k, 2-stage counted-vmcnt pipeline (2 blocks per CU), split-K over pixel ranges:
// each block writes its fp32 partial tile to its own slab ([nsplit][rows][KT]), summed in a fixed order by
// unpack_wgrad -> bitwise-deterministic weight gradients.
// Deferred-BN inputs (the conv read BN(+ReLU)(x) without materialising it): each wave re-normalises the
// X vectors it DMA'd, in LDS, after they land (its 8 channels are fixed for the whole kernel: the
// coefficients live in registers); the zero padding stays zero.
#include <algorithm>

#include "common.h"
#include "launchers.h"

namespace {

typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint8_t lds_u8_t;

DEVI f32x16_t mfma32(const uint4& a, const uint4& b, f32x16_t c) {
#ifdef GK_KO_MFMA   // (profiling knock-out builds only: csrc/build.py MSP_BUILD_DEFINES)
  c[0] += __uint_as_float(a.x ^ b.y);
  return c;
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), as_bf16x8(b), c, 0, 0, 0);
#endif
}

__device__ __attribute__((aligned(64))) uint4 g_wg_zero_page[4];

// LDS-DMA, 16 B per lane (see conv_gemm.hip glds16: inline asm keeps the compiler from draining the
// pipeline before every ds_read)
DEVI void glds16(const void* src, uint32_t lds) {
#ifdef GK_KO_DMA
  return;
#endif
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}

DEVI uint2 tr_read(const uint8_t* p) {
#ifdef GK_KO_LDS
  return make_uint2((uint32_t)(uintptr_t)p, 1u);
#endif
  s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t __attribute__((address_space(3)))*)(p));
  union { s16x4_t s; uint2 u; } c; c.s = v; return c.u;
}

// n / d for 0 <= n < 2^31 (host-built magic number)
struct FastDiv { uint32_t mul, shr; };
DEVI uint32_t fdiv_u(uint32_t n, FastDiv f) {
  return (uint32_t)(((uint64_t)__umulhi(n, f.mul) + n) >> f.shr);
}
FastDiv make_fastdiv(uint32_t d) {
  FastDiv f{0, 0};
  if (d <= 1) return f;   // mul 0, shr 0: n
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.mul = (uint32_t)((((1ull << l) - d) << 32) / d + 1);
  f.shr = l;
  return f;
}

constexpr int kBP = 64;   // pixels per stage

// 64-B-chunk swizzle of an LDS row of R bytes (R = 64, 128 or a multiple of 256): the 4 consecutive rows
// of a transposed read land in 4 distinct quarters of the 256-B bank row
template <int R>
DEVI int chunk_swz(int row) { return R == 64 ? 0 : (R == 128 ? ((row >> 1) & 1) : (row & 3)); }

struct WgGeom {
  long M;
  int KT, n_co, n_k, stages_per_split, nstages;
  FastDiv d_ohw, d_ow;
  int kw, ty0, tys, tx0, txs;   // regular tap grid (see conv_gemm.hip TapGrid)
};

template <int WM, int WN, int FM, int FN, bool PRO>
__global__ __launch_bounds__(64 * WM * WN, 2) void conv_wgrad_gemm_kernel(WgradPtrs P, float* __restrict__ dw,
                                                                          ConvGeom g, WgGeom wg) {
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int TCO = 32 * WM * FM, TK = 32 * WN * FN;
  constexpr int RA = TCO * 2, RB = TK * 2;                 // LDS row bytes (one pixel)
  constexpr int A_BYTES = kBP * RA, B_BYTES = kBP * RB, STAGE = A_BYTES + B_BYTES;
  constexpr int A_RPI = 1024 / RA, B_RPI = 1024 / RB;      // rows per DMA instruction
  constexpr int A_INS = kBP / A_RPI / NW, B_INS = kBP / B_RPI / NW;
  static_assert((RA == 64 || RA == 128 || RA % 256 == 0) && (RB == 64 || RB == 128 || RB % 256 == 0), "row bytes");
  static_assert(RA <= 1024 && RB <= 1024 && A_INS * A_RPI * NW == kBP && B_INS * B_RPI * NW == kBP, "DMA split");
  static_assert(!PRO || B_RPI % 4 == 0, "prologue: one channel vector per lane (B rows <= 256 B)");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t sbase = (uint32_t)(uintptr_t)(lds_u8_t*)smem;

  // block -> (pixel split, co tile, k tile); blocks of one split (same pixels) share an XCD's L2
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xq = nwg / 8, xr = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + orig / 8;
  const int ntile = wg.n_co * wg.n_k;
  const int split = wgid / ntile, tile = wgid - split * ntile;
  const int co_t = tile % wg.n_co, k_t = tile / wg.n_co;
  const int co0 = co_t * TCO, k0 = k_t * TK;
  const int rows = g.Go * g.Cgo, Cip = g.Gi * g.Cgi;
  const int st0 = split * wg.stages_per_split;
  const int nst = max(0, min(wg.stages_per_split, wg.nstages - st0));
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_wg_zero_page);

  // ---- A (dY) lanes: fixed channel column per instruction, pixel row = stage base + row
  const uint16_t* a_base[A_INS];
  int a_row[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = (j * NW + wave) * A_RPI + (lane * 16) / RA;
    const int slot = ((lane * 16) % RA) / 16;
    const int col = 32 * ((slot >> 2) ^ chunk_swz<RA>(row)) + 8 * (slot & 3);
    const int co = co0 + col;
    a_row[j] = row;
    if (co < rows) {
      const int og = co / g.Cgo;
      a_base[j] = P.dy[og] + (co - og * g.Cgo);
    } else {
      a_base[j] = nullptr;
    }
  }
  // ---- B (X im2col) lanes: fixed (tap, group, channel) per instruction
  const uint16_t* b_base[B_INS];
  int b_row[B_INS], b_dy[B_INS], b_dx[B_INS];
  int b_ci = 0, b_gi = 0;   // the lane's channel vector (prologue: identical for every instruction)
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = (j * NW + wave) * B_RPI + (lane * 16) / RB;
    const int slot = ((lane * 16) % RB) / 16;
    const int col = 32 * ((slot >> 2) ^ chunk_swz<RB>(row)) + 8 * (slot & 3);
    const int k = k0 + col;
    b_row[j] = row;
    if (k < wg.KT) {
      const int t = k / Cip, rem = k - (k / Cip) * Cip;
      const int gi = rem / g.Cgi, ci = rem - gi * g.Cgi;
      const int tr = t / wg.kw, tc = t - (t / wg.kw) * wg.kw;
      b_dy[j] = wg.ty0 + tr * wg.tys;
      b_dx[j] = wg.tx0 + tc * wg.txs;
      const uint16_t* xg = P.x[0];
#pragma unroll
      for (int q = 1; q < kMaxGroups; ++q) xg = gi == q ? P.x[q] : xg;
      b_base[j] = xg + ci;
      b_ci = ci; b_gi = gi;
    } else {
      b_base[j] = nullptr; b_dy[j] = 0; b_dx[j] = 0;
    }
  }
  // deferred-BN prologue coefficients of the lane's 8 channels
  float psc[8], psh[8];
  bool prelu = false, pro_on = false;
  if constexpr (PRO) {
    const float* cf = P.xc[0];
#pragma unroll
    for (int q = 1; q < kMaxGroups; ++q) cf = b_gi == q ? P.xc[q] : cf;
    pro_on = cf != nullptr && b_base[0] != nullptr;
    prelu = (P.xrelu >> b_gi) & 1u;
#pragma unroll
    for (int e = 0; e < 8; ++e) { psc[e] = 1.f; psh[e] = 0.f; }
    if (pro_on) { load8f(cf + b_ci, psc); load8f(cf + g.Cgi + b_ci, psh); }
  }

  // stage s: pixels (st0 + s) * 64 + row.  Returns the bit mask of the lane's in-image B vectors.
  auto stage = [&](int s, uint32_t sb) -> unsigned {
    const long mb = (long)(st0 + s) * kBP;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const long m = mb + a_row[j];
      const void* src = (a_base[j] != nullptr && m < wg.M) ? (const void*)(a_base[j] + m * g.Cgo) : (const void*)zero;
      glds16(src, sb + (j * NW + wave) * 1024);
    }
    unsigned ok = 0;
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const long m = mb + b_row[j];
      const void* src = zero;
      if (b_base[j] != nullptr && m < wg.M) {
        const uint32_t mu = (uint32_t)m;
        const uint32_t n = fdiv_u(mu, wg.d_ohw);
        const uint32_t r = mu - n * (uint32_t)(g.OH * g.OW);
        const uint32_t oh = fdiv_u(r, wg.d_ow);
        const int ow = (int)(r - oh * (uint32_t)g.OW);
        const int ih = (int)oh * g.stride + b_dy[j], iw = ow * g.stride + b_dx[j];
        if ((unsigned)ih < (unsigned)g.IH && (unsigned)iw < (unsigned)g.IW) {
          src = b_base[j] + ((long)((int)n * g.IH + ih) * g.IW + iw) * g.Cgi;
          ok |= 1u << j;
        }
      }
      glds16(src, sb + A_BYTES + (j * NW + wave) * 1024);
    }
    return ok;
  };

  // ---- fragment reads (transposed): lane l -> group gq = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  // rows (pixels) 16*kstep + 8*(gq >> 1) + q (+4), columns colbase + 16*(gq & 1) + 4p
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int gq = lane >> 4, li = lane & 15, lq = li >> 2, lp = li & 3;
  auto tr_addr = [&](int R, int row, int col) -> int {   // byte offset of (row, col) in a swizzled image
    const int sw = R == 64 ? 0 : (R == 128 ? ((row >> 1) & 1) : (row & 3));
    return row * R + (((col >> 5) ^ sw) << 6) + ((col & 31) << 1);
  };
  // per-lane offsets of the two transposed reads of k-step 0; k-step s adds 16 rows
  int a_off[FM][2], b_off[FN][2];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
      a_off[i][hh] = tr_addr(RA, 8 * (gq >> 1) + 4 * hh + lq, wm * FM * 32 + i * 32 + 16 * (gq & 1) + 4 * lp);
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
      b_off[j][hh] = A_BYTES + tr_addr(RB, 8 * (gq >> 1) + 4 * hh + lq, wn * FN * 32 + j * 32 + 16 * (gq & 1) + 4 * lp);
  // (16 more rows keep the row's swizzle: 16 is a multiple of 4)

  f32x16_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // 2-stage pipeline, one barrier per stage: wait for this wave's DMAs of stage s, (re-normalise its
  // X vectors), barrier (stage s visible everywhere; every wave is past stage s - 1's reads), issue the
  // DMAs of stage s + 1 into the buffer stage s - 1 used, then the MFMAs of stage s under them.
  unsigned ok_cur = 0, ok_nxt = 0;
  if (nst > 0) ok_cur = stage(0, sbase);
  for (int s = 0; s < nst; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t cur = (s & 1) * STAGE;
    if constexpr (PRO) {
      if (pro_on) {   // the lane's own landed X vectors, in place (the zero padding stays 0)
#pragma unroll
        for (int j = 0; j < B_INS; ++j) {
          if (!((ok_cur >> j) & 1u)) continue;
          uint4* v = reinterpret_cast<uint4*>(smem + cur + A_BYTES + (j * NW + wave) * 1024 + lane * 16);
          *v = affine8(*v, psc, psh, prelu);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (s + 1 < nst) ok_nxt = stage(s + 1, sbase + ((s + 1) & 1) * STAGE);
    const uint8_t* sp = smem + cur;
#pragma unroll
    for (int ks = 0; ks < kBP / 16; ++ks) {
      uint4 af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const uint2 lo = tr_read(sp + a_off[i][0] + ks * 16 * RA);
        const uint2 hi = tr_read(sp + a_off[i][1] + ks * 16 * RA);
        af[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const uint2 lo = tr_read(sp + b_off[j][0] + ks * 16 * RB);
        const uint2 hi = tr_read(sp + b_off[j][1] + ks * 16 * RB);
        bf[j] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma32(af[i], bf[j], acc[i][j]);
    }
    ok_cur = ok_nxt;
  }

  // ---- epilogue: this split's fp32 partial tile -> its slab (plain stores, every element once)
  float* slab = dw + (long)split * rows * wg.KT;
  const int kc = k0 + wn * FN * 32 + (lane & 31);
  const int lh = lane >> 5;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int k = kc + 32 * j;
    if (k >= wg.KT) continue;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + wm * FM * 32 + i * 32 + 8 * (e >> 2) + 4 * lh + (e & 3);
        if (co < rows) slab[(long)co * wg.KT + k] = acc[i][j][e];
      }
  }
}

// the deferred-BN prologue needs one channel vector per lane: B rows of <= 256 B (TK <= 128)
constexpr bool wg_pro_ok(int wn, int fn) { return 32 * wn * fn <= 128; }

struct WgCfg { int wm, wn, fm, fn; };
// TCO x TK tiles (LDS per stage = 64 * (TCO + TK) * 2 B, two stages).  Every TK <= 128 (B rows <= 256 B):
// the deferred-BN prologue then works on every configuration, so it never changes the plan.
constexpr WgCfg kWgCfgs[] = {
    {2, 2, 2, 2},   // 128 x 128
    {1, 4, 1, 1},   //  32 x 128  (narrow dY: 17-34 channel layers)
    {2, 2, 1, 2},   //  64 x 128
    {2, 2, 2, 1},   // 128 x  64
    {1, 4, 2, 1},   //  64 x 128  (waves along k)
    {2, 2, 4, 1},   // 256 x  64
    // 8-wave tiles, one block per CU (round 5, see conv_gemm.hip kCfgs); no deferred-BN prologue (TK > 128)
    {2, 4, 4, 2},   // 256 x 256 (128 KB)
    {2, 4, 2, 2},   // 128 x 256 ( 96 KB)
    {4, 2, 2, 2},   // 256 x 128 ( 96 KB)
};
constexpr int kNumWgCfgs = sizeof(kWgCfgs) / sizeof(kWgCfgs[0]);

int g_wg_mode = -1;   // env MSP_WGRAD_GEMM: 0 off (the conv.hip kernels), 1 auto (default), 2 every eligible conv
int g_wg_cfg = -1;    // conv_wgrad_gemm_force_cfg: force a configuration (tests / A-B); -1 planner
// Grid size target for 4-wave tiles (8-wave: half): 512 (round 5 sweep, profiles/r05/wgrad_blocks_sweep.txt:
// 256 / 512 / 768 / 1024 -> R101 bs64 1371 / 1456 / 1397 / 1390, FPN-R101 1532 / 1600 / 1518 / 1498,
// DUCKNet-17 bs320 553 / 592 / 579 / 593 img/s)
constexpr long g_wg_blocks = 512;
// The planner's per-row staging cost (MAC units, wg_pick).  96 (round 5) picks the 8-wave 256-wide tiles for
// the >= 136-channel 3x3 / 1x7 layers: conv_bench levels 3-6 wgrad 25.3 -> 22.4 ms at bs320 against 24
// (profiles/r05/wgrad_stage_cost_bs320.txt)
constexpr double g_wg_stage_cost = 96.0;

void wg_env() {
  if (g_wg_mode < 0) {
    const char* e = getenv("MSP_WGRAD_GEMM");
    g_wg_mode = e == nullptr ? 1 : (e[0] == '0' ? 0 : (e[0] == '2' ? 2 : 1));
  }
}

int wg_pick(int rows, int KT, bool pro) {
  if (g_wg_cfg >= 0 && (!pro || wg_pro_ok(kWgCfgs[g_wg_cfg].wn, kWgCfgs[g_wg_cfg].fn))) return g_wg_cfg;
  int best = 0;
  double best_cost = 1e30;
  for (int c = 0; c < kNumWgCfgs; ++c) {
    if (pro && !wg_pro_ok(kWgCfgs[c].wn, kWgCfgs[c].fn)) continue;
    const int tco = 32 * kWgCfgs[c].wm * kWgCfgs[c].fm, tk = 32 * kWgCfgs[c].wn * kWgCfgs[c].fn;
    const double nt = (double)cdiv(rows, tco) * cdiv(KT, tk);
    // padded MFMA work + operand staging per tile (in MAC units of one 64-pixel stage)
    const double cost = nt * ((double)tco * tk + g_wg_stage_cost * (tco + tk));
    if (cost < best_cost) { best_cost = cost; best = c; }
  }
  return best;
}

bool wg_tap_grid(const ConvGeom& g, WgGeom& w) {
  for (int kw = 1; kw <= g.T; ++kw) {
    if (g.T % kw != 0) continue;
    const int kh = g.T / kw;
    w.kw = kw; w.ty0 = g.dy[0]; w.tx0 = g.dx[0];
    w.tys = kh > 1 ? g.dy[kw] - g.dy[0] : 0;
    w.txs = kw > 1 ? g.dx[1] - g.dx[0] : 0;
    bool ok = true;
    for (int t = 0; t < g.T && ok; ++t) ok = g.dy[t] == w.ty0 + (t / kw) * w.tys && g.dx[t] == w.tx0 + (t % kw) * w.txs;
    if (ok) return true;
  }
  return false;
}

struct WgPlan { int cfg; WgGeom w; long blocks; int nsplit; };

WgPlan wg_plan(const ConvGeom& g, bool pro) {
  WgPlan p{};
  p.cfg = wg_pick(g.Go * g.Cgo, g.T * g.Gi * g.Cgi, pro);
  const WgCfg& c = kWgCfgs[p.cfg];
  WgGeom& w = p.w;
  (void)wg_tap_grid(g, w);
  w.M = (long)g.N * g.OH * g.OW;
  w.KT = g.T * g.Gi * g.Cgi;
  w.n_co = cdiv(g.Go * g.Cgo, 32 * c.wm * c.fm);
  w.n_k = cdiv(w.KT, 32 * c.wn * c.fn);
  w.nstages = (int)((w.M + kBP - 1) / kBP);
  const long ntile = (long)w.n_co * w.n_k;
  // grid target: two rounds of resident blocks -- 8-wave tiles hold one block per CU (96-128 KB of LDS), so
  // half the 4-wave configs' target: every extra split is one more fp32 dW slab for unpack_wgrad to sum
  // (round 5: with the 1024 target the 8-wave tiles doubled smp-Unet R101's unpack time, 2.2 -> 5.1 ms/step)
  const long target = c.wm * c.wn >= 8 ? g_wg_blocks / 2 : g_wg_blocks;
  long ns = std::max(1L, std::min((long)w.nstages, target / std::max(1L, ntile)));
  w.stages_per_split = (int)((w.nstages + ns - 1) / ns);
  ns = (w.nstages + w.stages_per_split - 1) / w.stages_per_split;   // no empty splits
  p.nsplit = (int)ns;
  p.blocks = ns * ntile;
  w.d_ohw = make_fastdiv((uint32_t)(g.OH * g.OW));
  w.d_ow = make_fastdiv((uint32_t)g.OW);
  return p;
}

template <int WM, int WN, int FM, int FN>
int launch_wg(const WgradPtrs& P, float* dw, const ConvGeom& g, const WgPlan& p, bool pro, hipStream_t s) {
  constexpr int LDS = 2 * kBP * (32 * WM * FM + 32 * WN * FN) * 2;
  static bool attr[2] = {false, false};
  if (pro) {
    if constexpr (!wg_pro_ok(WN, FN)) {
      return 1;
    } else {
    if (!attr[1]) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_gemm_kernel<WM, WN, FM, FN, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
      attr[1] = true;
    }
    hipLaunchKernelGGL((conv_wgrad_gemm_kernel<WM, WN, FM, FN, true>), dim3((unsigned)p.blocks), dim3(64 * WM * WN),
                       LDS, s, P, dw, g, p.w);
    return 0;
    }
  }
  if (!attr[0]) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_gemm_kernel<WM, WN, FM, FN, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr[0] = true;
  }
  hipLaunchKernelGGL((conv_wgrad_gemm_kernel<WM, WN, FM, FN, false>), dim3((unsigned)p.blocks), dim3(64 * WM * WN), LDS,
                     s, P, dw, g, p.w);
  return 0;
}


}  // namespace

// Eligibility: forward-geometry weight gradients (not the transposed-conv form) on a regular tap grid
// with 8-aligned channel groups (with or without a deferred-BN prologue on x).
bool conv_wgrad_gemm_ok(const ConvGeom& g, bool trans) {
  wg_env();
  if (!g_wg_mode || trans || g.Cgi % 8 != 0 || g.Cgo % 8 != 0) return false;
  WgGeom w{};
  if (!wg_tap_grid(g, w)) return false;
  const long M = (long)g.N * g.OH * g.OW;
  return M < (1L << 31) - 2 * kBP;
}

int conv_wgrad_gemm_replicas(const ConvGeom& g, bool pro) {
  wg_env();
  return wg_plan(g, pro).nsplit;
}

void conv_wgrad_gemm_set(int mode) { wg_env(); g_wg_mode = mode < 0 ? 0 : (mode > 2 ? 2 : mode); }
int conv_wgrad_gemm_mode() { wg_env(); return g_wg_mode; }
void conv_wgrad_gemm_force_cfg(int cfg) { wg_env(); g_wg_cfg = (cfg >= 0 && cfg < kNumWgCfgs) ? cfg : -1; }
int conv_wgrad_gemm_num_cfgs() { return kNumWgCfgs; }

int conv_wgrad_gemm(const WgradPtrs& P, float* dw, const ConvGeom& g, bool prologue, hipStream_t s) {
  const WgPlan p = wg_plan(g, prologue);
  switch (p.cfg) {
    case 0: return launch_wg<2, 2, 2, 2>(P, dw, g, p, prologue, s);
    case 1: return launch_wg<1, 4, 1, 1>(P, dw, g, p, prologue, s);
    case 2: return launch_wg<2, 2, 1, 2>(P, dw, g, p, prologue, s);
    case 3: return launch_wg<2, 2, 2, 1>(P, dw, g, p, prologue, s);
    case 4: return launch_wg<1, 4, 2, 1>(P, dw, g, p, prologue, s);
    case 5: return launch_wg<2, 2, 4, 1>(P, dw, g, p, prologue, s);
    case 6: return launch_wg<2, 4, 4, 2>(P, dw, g, p, prologue, s);
    case 7: return launch_wg<2, 4, 2, 2>(P, dw, g, p, prologue, s);
    case 8: return launch_wg<4, 2, 2, 2>(P, dw, g, p, prologue, s);
  }
  return 1;
}
