// LDS-tiled implicit-GEMM convolution for CDNA4 (gfx950): the wide-channel forward and stride-1
// data-gradient path (input width >= 64 channels), on v_mfma_f32_32x32x16_bf16.
//
// Replaces the register-direct gather kernel (conv.hip conv_igemm_kernel) for the MFMA-friendly layers of
// the reference's convolutions (3x3 d1/d2/d3, 1x7/7x1, 1x1, 3x3 s2, 2x2 s2 at 68..544
// channels; reference models/ducknet.py:95-96,144-149,160-178, models/modules.py:73-85).
//
// GEMM view:  D[co][m] = sum_k  W[co][k] * X[k][m]      m = output pixel, k = (tap t, input channel c)
//   block tile  TCO co-rows x TPX pixels, K staged 64 at a time (one 128-B row per co / pixel);
//   WM x WN waves, each owns FM x FN 32x32 accumulator tiles.
// Staging: both operands go global -> LDS with global_load_lds_dwordx4 (LDS-DMA; no VGPR round trip).
// One wave-instruction fills 8 rows x 128 B; the per-lane SOURCE address is free, so
//   * the im2col gather of X is just the lane's source address (tap shift + bounds check; the zero
//     padding and the K / M tails read a 64-B zero page),
//   * the LDS image is XOR-swizzled on the source side (16-B slot ^= (row >> 1) & 7): the 16 rows of a
//     ds_read_b128 lane group then sit on 16 distinct bank slots -> conflict-free fragment reads.
// Pipeline: 2 LDS stages; the DMA of stage k+1 is issued before the MFMAs of stage k, one
// vmcnt(0) + barrier per stage.
// Epilogue: bias / accumulate / bf16 round, 8-B NHWC stores into the row's output group, and the
// per-channel BatchNorm partials (sum, sum^2 of the stored values -- or, for the data-gradient of a
// BN output, the BN-backward partials) reduced across lanes and waves in LDS, one row per pixel tile.
#include <algorithm>

#include "common.h"
#include "launchers.h"

namespace {

typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void_t;

DEVI f32x16_t mfma32(const uint4& a, const uint4& b, f32x16_t c) {
#ifdef GK_KO_MFMA   // (profiling knock-out builds only: csrc/build.py MSP_BUILD_DEFINES)
  c[0] += __uint_as_float(a.x ^ b.y);
  return c;
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), as_bf16x8(b), c, 0, 0, 0);
#endif
}

// Output store.  (Round 5 tried global_store ... sc1 here, to keep the output stream out of the XCD's L2: the
// L4 fused-8 forward and data-gradient got 5-25 % SLOWER and their L2 read misses rose, so plain stores.)
DEVI void st_stream8(uint16_t* p, uint32_t lo, uint32_t hi) {
#ifdef GK_KO_STORE   // (profiling knock-out: no output stores; a never-true test keeps the math alive)
  if (lo == 0x7fc17fc1u && hi == 0x12345678u) *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
#else
  *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
#endif
}

// 64 zero bytes in global memory: the DMA source of every padding / out-of-range vector
__device__ __attribute__((aligned(64))) uint4 g_zero_page[4];

// LDS-DMA of 16 B per lane: LDS[lds + 16*lane] = *src (lds wave-uniform, in an SGPR via M0).  Inline asm
// on purpose: with the builtin the compiler drains every DMA in flight (vmcnt(0)) before ANY later
// ds_read, since it cannot prove the read does not alias the DMA's destination -- that would serialise
// the software pipeline.  Here the pipeline's own counted vmcnt waits + barriers order the DMAs
// against the reads; nothing else in the main loop touches the vector-memory counter.
DEVI void glds16(const void* src, uint32_t lds) {
#ifdef GK_KO_DMA
  return;
#endif
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}

typedef __attribute__((address_space(3))) uint8_t lds_u8_t;


struct KPos { int t, gi, cl; };

DEVI KPos kpos_init(int k, int Cgi, int Gi) {
  const int Cip = Gi * Cgi;
  KPos p;
  p.t = k / Cip;
  const int rem = k - p.t * Cip;
  p.gi = rem / Cgi;
  p.cl = rem - p.gi * Cgi;
  return p;
}

DEVI void kpos_advance(KPos& p, int by, int Cgi, int Gi) {
  p.cl += by;
  while (p.cl >= Cgi) {
    p.cl -= Cgi;
    if (++p.gi == Gi) { p.gi = 0; ++p.t; }
  }
}

struct GemmGeom {
  long M, OHW;
  int n_co, nk;
  // phase output map (the phase-decomposed strided data-gradient, conv_gemm_phase): GEMM pixel m of the
  // OHp x OWp phase grid stores at (py + ps*oh, px + ps*ow) of the full OH x OW output; ps = 0: identity
  int ps, py, px, OWp;
  long OHWp, OW, OHWf;
  long apitch;   // packed weight row pitch (= Kp; a phase launch walks K = its own taps, rows keep the full pitch)
};

// BK = k per stage (64 or 32): one staged row (co or pixel) is BK bf16 = ROWB bytes, one DMA instruction
// (64 lanes x 16 B) fills RPI rows.  BK 32 halves the bytes per stage, so the same LDS holds twice the
// stages in flight (the round-5 knock-outs showed the BK-64 kernel bound by LDS-DMA latency at one stage
// in flight, profiles/r05/gemm_knockouts_bs320.txt).
template <int WM, int WN, int FM, int FN, int NS, int BK>
struct GemmCfg {
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int TCO = 32 * WM * FM, TPX = 32 * WN * FN;
  static constexpr int ROWB = BK * 2, SLOTS = BK / 8, RPI = 1024 / ROWB;
  static constexpr int A_BYTES = TCO * ROWB, B_BYTES = TPX * ROWB, STAGE = A_BYTES + B_BYTES;
  static constexpr int A_INS = TCO / RPI / NW, B_INS = TPX / RPI / NW;   // DMA instructions per wave per stage
  // (the epilogue's stats scratch reuses the stages)
  static constexpr int LDS = NS * STAGE;
  static_assert(BK == 64 || BK == 32, "stage width");
  static_assert(TCO % (RPI * NW) == 0 && TPX % (RPI * NW) == 0, "tile rows must split evenly over the waves");
  static_assert(2 * WN * TCO * 4 <= NS * STAGE, "stats scratch must fit in the staging LDS");
  static_assert(NS >= 2 && NS <= 5 && (NS - 2) * (A_INS + B_INS) < 64, "pipeline depth / vmcnt range");
  static_assert(NW % 2 == 0, "one logical k slot per lane across the wave's DMA instructions");
  // XOR swizzle of the 16-B slots of a row (source side of the DMA, undone by the fragment reads): the 16
  // rows of a ds_read_b128 lane group land on 16 distinct bank slots.  BK 64: 128-B rows, slot ^= (row >> 1)
  // & 7; BK 32: 64-B rows (four per 256-B bank row), slot ^= (row >> 2) & 3.
  static DEVI int swz(int row) { return BK == 64 ? ((row >> 1) & 7) : ((row >> 2) & 3); }
};

// Regular tap grid (every conv this path takes): tap t = (r, c), r = t / kw, c = t % kw, offset
// (dy, dx) = (y0 + r * ys, x0 + c * xs) -- forward taps (r*dil - pad) and data-gradient taps (pad - r*dil)
// alike.  Kept as scalars so that the DMA address generation reads NO memory: an LDS or global read
// between two LDS-DMAs makes the compiler drain every DMA in flight (vmcnt(0)) before it.
struct TapGrid {
  int kw, y0, ys, x0, xs;
  // packed-weight tap of grid tap (tr, tc): (ar0 + tr*ars)*akw + ac0 + tc*acs -- the identity (= tr*kw + tc)
  // except for a phase launch, whose taps are a strided subset of the packed data-gradient taps
  int akw, ar0, ars, ac0, acs;
};

// OCC: the minimum blocks per CU the register allocation must allow (2: the planner's tiles; 3-4: the
// small-LDS BK-32 tiles, round 6 occupancy A/B)
template <int WM, int WN, int FM, int FN, int NS, int BK, bool BNE, int OCC = 2>
__global__ __launch_bounds__(64 * WM * WN, OCC) void conv_gemm_kernel(ConvArgs a, GemmGeom gg, TapGrid tg) {
  using C = GemmCfg<WM, WN, FM, FN, NS, BK>;
  constexpr int kRowB = C::ROWB, RPI = C::RPI;
  const ConvGeom& g = a.g;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t sbase = (uint32_t)(uintptr_t)(lds_u8_t*)smem;   // LDS byte address of the stages

  // XCD-aware bijective remap: the co tiles of one pixel tile (which share its B operand) and
  // neighbouring pixel tiles (which share input rows through the tap halo) run on one XCD's L2
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xq = nwg / 8, xr = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + orig / 8;
  const int co_t = wgid % gg.n_co;
  const long px_t = wgid / gg.n_co;
  const int co0 = co_t * C::TCO;
  const long px0 = px_t * C::TPX;
  const int rows = g.Go * g.Cgo;
  const int Cgi = g.Cgi, Gi = g.Gi;
  const int IHW = g.IH * g.IW;

  // ---- DMA roles: instruction j of this wave fills tile rows RPI*(j*NW + wave) .. +RPI-1; lane -> row
  // lane / SLOTS, physical 16-B slot lane % SLOTS = logical slot ^ swz(row).  With NW even, swz(row) does
  // not depend on j, so a lane's LOGICAL slot ls -- its k offset 8*ls inside the stage -- is the same for
  // every instruction j of the wave.
  const int ls = (lane % C::SLOTS) ^ C::swz(RPI * wave + lane / C::SLOTS);
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_page);
  // A (packed weights): a fixed row pointer per instruction; the stage adds its k base.  Rows past the
  // layer read row 0 (their outputs are never stored) and the K tail of the last stage reads past Kp into
  // the next row / the allocation's slack (packed_weight_slack): finite values times a zero B operand.
  const uint16_t* a_src[C::A_INS];
#pragma unroll
  for (int j = 0; j < C::A_INS; ++j) {
    const int co = co0 + RPI * (j * C::NW + wave) + lane / C::SLOTS;
    a_src[j] = a.w + (long)(co < rows ? co : 0) * gg.apitch + 8 * ls;
#ifdef GK_KO_AMISS   // (profiling knock-out: every A row reads row 0 -- L2-resident)
    a_src[j] = a.w + 8 * ls;
#endif
  }
  // B (im2col of the input): per instruction the pixel's input origin (element offset, taps excluded) and
  // a bitmask of the taps that land inside the image -- both fixed for the whole K walk.
  long b_pix[C::B_INS];
  uint32_t b_vm[C::B_INS];
#pragma unroll
  for (int j = 0; j < C::B_INS; ++j) {
    const long m = px0 + RPI * (j * C::NW + wave) + lane / C::SLOTS;
    b_pix[j] = 0;
    b_vm[j] = 0u;
    if (m < gg.M) {
      const int n = (int)(m / gg.OHW);
      const int r = (int)(m - (long)n * gg.OHW);
      const int oh = r / g.OW, ow = r - (r / g.OW) * g.OW;
      const int ih0 = oh * g.stride, iw0 = ow * g.stride;
      b_pix[j] = ((long)n * IHW + (long)ih0 * g.IW + iw0) * Cgi;
#ifdef GK_KO_BMISS   // (profiling knock-out: every pixel reads the tile's first rows -- L2-resident)
      b_pix[j] = ((long)(ih0 % 4) * g.IW + (iw0 % 8)) * Cgi;
#endif
      uint32_t vm = 0u;
      int tr = 0, tc = 0;
      for (int t = 0; t < g.T; ++t) {
        const int ih = ih0 + tg.y0 + tr * tg.ys, iw = iw0 + tg.x0 + tc * tg.xs;
        if ((unsigned)ih < (unsigned)g.IH && (unsigned)iw < (unsigned)g.IW) vm |= 1u << t;
        if (++tc == tg.kw) { tc = 0; ++tr; }
      }
      b_vm[j] = vm;
    }
  }
  // K walk, uniform (SGPRs): the stage's first k = (tap t0 = (tr0, tc0), group g0, channel cl0); toff0 = the
  // element offset of tap t0 from the pixel origin.  Cgi >= 64 >= the stage width, so the slots of a row
  // cross at most one (group | tap) boundary: a lane at slot ls >= (Cgi - cl0) / 8 is in the next one.
  const long dcol = (long)tg.xs * Cgi, drow = ((long)tg.ys * g.IW - (long)tg.kw * tg.xs) * Cgi;
  int t0, tr0, tc0, g0, cl0;
  long toff0;
  auto walk_to = [&](int k) {   // uniform walk state at k (a multiple of BK)
    const int Cip = Gi * Cgi;
    t0 = k / Cip;
    const int rem = k - t0 * Cip;
    g0 = rem / Cgi;
    cl0 = rem - g0 * Cgi;
    tr0 = t0 / tg.kw;
    tc0 = t0 - tr0 * tg.kw;
    toff0 = ((long)(tg.y0 + tr0 * tg.ys) * g.IW + (tg.x0 + tc0 * tg.xs)) * Cgi;
  };
  walk_to(0);
  auto gptr = [&](int q) {   // group pointer from the kernel arguments (scalars), no memory read
    const uint16_t* xb = a.x[0];
#pragma unroll
    for (int u = 1; u < kMaxGroups; ++u) xb = q == u ? a.x[u] : xb;
    return xb;
  };

  const int Cip_ = Gi * Cgi;
  auto stage = [&](int kt, uint32_t sb) {
    const int kb = kt * BK;
    // the (group | tap) after the current one
    int g1 = g0 + 1, t1 = t0, tr1 = tr0, tc1 = tc0;
    long toff1 = toff0;
    if (g1 == Gi) {
      g1 = 0;
      ++t1;
      toff1 += dcol;
      if (++tc1 == tg.kw) { tc1 = 0; ++tr1; toff1 += drow; }
    }
    const int rem0 = Cgi - cl0;
    const bool nx = 8 * ls >= rem0;   // (per lane)
    // A: packed column of the lane's k -- contiguous, shifted by the tap remap of a phase launch (uniform
    // per tap; past the last tap the contiguous continuation: finite weights times a zero B operand)
    const int dA0 = ((tg.ar0 + tr0 * tg.ars) * tg.akw + tg.ac0 + tc0 * tg.acs - t0) * Cip_;
    const int dA1 = t1 < g.T ? ((tg.ar0 + tr1 * tg.ars) * tg.akw + tg.ac0 + tc1 * tg.acs - t1) * Cip_ : dA0;
    const int ka = kb + (nx ? dA1 : dA0);
#pragma unroll
    for (int j = 0; j < C::A_INS; ++j) glds16(a_src[j] + ka, sb + (RPI * (j * C::NW + wave)) * kRowB);
    const int t = nx ? t1 : t0;
    const uint16_t* base = (nx ? gptr(g1) : gptr(g0)) + (nx ? toff1 + (8 * ls - rem0) : toff0 + (cl0 + 8 * ls));
    const bool tin = t < 32;
#pragma unroll
    for (int j = 0; j < C::B_INS; ++j) {
      const bool ok = tin && ((b_vm[j] >> t) & 1u);
      glds16(ok ? (const void*)(base + b_pix[j]) : (const void*)zero,
             sb + C::A_BYTES + (RPI * (j * C::NW + wave)) * kRowB);
    }
    // advance the walk by BK (at most one boundary: Cgi >= 64)
    cl0 += BK;
    if (cl0 >= Cgi) { cl0 -= Cgi; g0 = g1; t0 = t1; tr0 = tr1; tc0 = tc1; toff0 = toff1; }
  };

  // ---- fragment reads: lane (r = lane & 31, h = lane >> 5) takes 8 k at logical slot 2s + h of row r
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int key = C::swz(lr);   // == swz(row) for every fragment row (bases are multiples of 32)
  constexpr int KS = BK / 16;    // MFMA k-steps per stage
  int soff[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) soff[s] = (((2 * s + lh) ^ key) << 4);
  const int a_row0 = (wm * FM * 32 + lr) * kRowB;
  const int b_row0 = C::A_BYTES + (wn * FN * 32 + lr) * kRowB;

  f32x16_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // ---- software pipeline over NS LDS stages: the DMA of stage kt + NS - 1 is issued right after the
  // barrier that retires stage kt, so NS - 1 stages of loads stay in flight under the MFMAs.  Each wave
  // waits only for ITS OWN DMAs of stage kt (counted vmcnt: every wave issues exactly INS per stage),
  // then the barrier makes every wave's landed data visible (and frees the buffer stage kt - 1 used).
  constexpr int INS = C::A_INS + C::B_INS;
  const int nk = gg.nk;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) stage(p, sbase + p * C::STAGE);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1 - kt, NS - 2);   // stages issued after kt and still allowed in flight
    if (NS >= 5 && ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * INS) : "memory");
    else if (NS >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * INS) : "memory");
    else if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NS - 1 < nk) stage(kt + NS - 1, sbase + ((kt + NS - 1) % NS) * C::STAGE);
    const uint8_t* cur = smem + (kt % NS) * C::STAGE;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      uint4 af[FM], bfr[FN];
#pragma unroll
#ifdef GK_KO_LDS
      for (int i = 0; i < FM; ++i) af[i] = make_uint4(kt + i, s, lane, 0);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = make_uint4(kt, j + s, 0, lane);
#else
      for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const uint4*>(cur + a_row0 + i * 32 * kRowB + soff[s]);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = *reinterpret_cast<const uint4*>(cur + b_row0 + j * 32 * kRowB + soff[s]);
#endif
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma32(af[i], bfr[j], acc[i][j]);
    }
  }
  __syncthreads();   // every wave is done with the stages before the epilogue reuses them

  // ---- epilogue.  32x32 D layout: lane holds column (pixel) lr, rows 8q + 4h + r in register 4q + r.
  float* s_st = reinterpret_cast<float*>(smem);   // [WN][2][TCO] per-pixel-wave-column channel partials
  const bool stats = a.stat_part != nullptr;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int rb = wm * FM * 32 + i * 32;   // tile-local row base of this fragment row
    uint16_t* yb[4];
    int cl4[4];
    float cs[16], cq[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cb = co0 + rb + 8 * q + 4 * lh;
      const int og = cb < rows ? cb / g.Cgo : 0;
      cl4[q] = cb - og * g.Cgo;
      uint16_t* yg = a.y[0];
#pragma unroll
      for (int t = 1; t < kMaxGroups; ++t) yg = og == t ? a.y[t] : yg;
      yb[q] = cb < rows ? yg + cl4[q] : nullptr;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) { cs[e] = 0.f; cq[e] = 0.f; }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      long m = px0 + wn * FN * 32 + j * 32 + lr;
      if (m >= gg.M) continue;
      if (gg.ps) {   // phase launch: the phase-grid pixel's place in the full output
        const long n = m / gg.OHWp, r = m - n * gg.OHWp;
        const long oh = r / gg.OWp, ow = r - oh * gg.OWp;
        m = n * gg.OHWf + (gg.py + gg.ps * oh) * gg.OW + gg.px + gg.ps * ow;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (yb[q] == nullptr) continue;
        uint16_t* yp = yb[q] + m * g.Cgo;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][4 * q + r];
        if (a.bias != nullptr) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = cl4[q] + r < g.Cgo_l ? v[r] + a.bias[cl4[q] + r] : 0.f;
        }
        if (!BNE && a.accum) {   // y += conv(x): sibling launches' data-gradients into one tensor
          const uint2 ov = *reinterpret_cast<const uint2*>(yp);
          v[0] += __uint_as_float(ov.x << 16); v[1] += __uint_as_float(ov.x & 0xffff0000u);
          v[2] += __uint_as_float(ov.y << 16); v[3] += __uint_as_float(ov.y & 0xffff0000u);
        }
        const uint32_t lo = pack2(v[0], v[1]), hi = pack2(v[2], v[3]);
        st_stream8(yp, lo, hi);
        // statistics of the STORED (bf16-rounded) values, as a BN reading this tensor sees them
        const float w4[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                             __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
        if constexpr (BNE) {   // BN-backward partials of the BN whose output this data-gradient is (Go == 1)
          const int cb = cl4[q];
          const uint2 yy = *reinterpret_cast<const uint2*>(a.bn_y + m * g.Cgo + cb);
          const float4 sc = *reinterpret_cast<const float4*>(a.bn_coef + cb);
          const float4 sh = *reinterpret_cast<const float4*>(a.bn_coef + g.Cgo + cb);
          const float4 mu = *reinterpret_cast<const float4*>(a.bn_coef + 2 * g.Cgo + cb);
          const float y4[4] = {__uint_as_float(yy.x << 16), __uint_as_float(yy.x & 0xffff0000u),
                               __uint_as_float(yy.y << 16), __uint_as_float(yy.y & 0xffff0000u)};
          const float s4[4] = {sc.x, sc.y, sc.z, sc.w}, h4[4] = {sh.x, sh.y, sh.z, sh.w};
          const float m4[4] = {mu.x, mu.y, mu.z, mu.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gr = (!a.bn_relu || fmaf(y4[r], s4[r], h4[r]) > 0.f) ? w4[r] : 0.f;
            cs[4 * q + r] += gr;
            cq[4 * q + r] = fmaf(gr, y4[r] - m4[r], cq[4 * q + r]);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            cs[4 * q + r] += w4[r];
            cq[4 * q + r] = fmaf(w4[r], w4[r], cq[4 * q + r]);
          }
        }
      }
    }
    if (stats) {
      // sum over the 32 pixel lanes of each half: DPP row sums (16 lanes) + one swap of the row pair
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float s = row16_sum(cs[e]), q = row16_sum(cq[e]);
        s += __shfl_xor(s, 16, 64);
        q += __shfl_xor(q, 16, 64);
        if (lr == 0) {
          const int row = rb + 8 * (e >> 2) + 4 * lh + (e & 3);
          s_st[(wn * 2 + 0) * C::TCO + row] = s;
          s_st[(wn * 2 + 1) * C::TCO + row] = q;
        }
      }
    }
  }
  if (stats) {
    __syncthreads();
    // one partial row per 128 pixels (kGemmTPX): a 256-pixel tile writes two; rows past the layer's
    // pixel count (an empty tail half) are not written
    constexpr int HALVES = C::TPX / 128, WPH = WN / HALVES;   // waves per 128-pixel half
    static_assert(C::TPX % 128 == 0 && WN % HALVES == 0, "128-pixel stat rows");
    const long nrow = (gg.M + 127) / 128;
    for (int e = tid; e < HALVES * C::TCO; e += C::NT) {
      const int hb = e / C::TCO, c = e - hb * C::TCO;
      const int co = co0 + c;
      const long srow = px0 / 128 + hb;
      if (co >= rows || srow >= nrow) continue;
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < WPH; ++w) {
        const int wv = hb * WPH + w;
        s += s_st[(wv * 2 + 0) * C::TCO + c];
        q += s_st[(wv * 2 + 1) * C::TCO + c];
      }
      a.stat_part[(srow * 2 + 0) * rows + co] = s;
      a.stat_part[(srow * 2 + 1) * rows + co] = q;
    }
  }
}

// ---- configurations ------------------------------------------------------------------------------
// (WM, WN, FM, FN): TCO = 32*WM*FM co rows x TPX = 32*WN*FN pixels per block
struct CfgId { int wm, wn, fm, fn, ns, bk; };
// Two LDS stages everywhere: two blocks per CU (8 waves) measured 1.5-2x faster than one block with
// a third stage (profiles/r03/gemm_cfg_sweep_bs128.log); the tile height is the main lever (B-operand
// reuse), so the planner picks the tallest tile whose row padding stays small.
constexpr CfgId kCfgs[] = {
    {2, 2, 3, 2, 2, 64},   // 192 x 128 (80 KB)
    {2, 2, 2, 2, 2, 64},   // 128 x 128 (64 KB)
    {1, 4, 3, 1, 2, 64},   //  96 x 128 (56 KB)
    {1, 4, 5, 1, 2, 64},   // 160 x 128 (72 KB)
    {2, 2, 1, 2, 2, 64},   //  64 x 128 (48 KB)
    // round 5: 32-wide stages, 3-4 of them in flight at two blocks per CU (8-wave 256 x 256 tiles at one
    // block per CU measured slower: profiles/r05/gemm_cfg_sweep_bs320.txt)
    {2, 2, 2, 2, 4, 32},   // 128 x 128, 4 stages (64 KB)
    {2, 2, 3, 2, 4, 32},   // 192 x 128, 4 stages (80 KB)
    {2, 2, 4, 2, 3, 32},   // 256 x 128, 3 stages (72 KB)
    {2, 2, 2, 2, 5, 32},   // 128 x 128, 5 stages (80 KB)
    // round 6: a small-LDS tile at four blocks per CU -- the planner's pick for short-K launches (see
    // gemm_pick_cfg; 192 x 128 / 128 x 128 3-stage / 64 x 128 tiles at 3-4 blocks per CU measured slower at
    // every level 3-6 shape: profiles/r06/gemm_occupancy_bs320.txt)
    {2, 2, 2, 2, 2, 32},   // 128 x 128, 2 stages (32 KB), 4 blocks / CU
    // (8-wave 128 x 256 tiles at 3 x 64-wide stages, one block per CU, measured 15-35 % slower than the
    // planner's tiles at every level 3-6 shape: profiles/r05/gemm_cfg_8wave_3stage_bs320.txt)
};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);
constexpr int kPlannerCfgs = 5;   // the planner's row-tile candidates (5-8: conv_gemm_force_cfg A/B only)
constexpr int kOccCfg = 9;        // the four-blocks-per-CU tile (short K)
constexpr int kGemmTPX = 128;   // stat partial rows = pixel tiles of 128 (a 256-pixel tile writes two rows)

int g_gemm_mode = -1;     // env MSP_CONV_GEMM: 0 off, else on (default on)
int g_gemm_cfg = -1;      // conv_gemm_force_cfg: one configuration index (tests / A-B), -1 = planner
// (round 5's A/B knobs -- XCD-grouped block order, K rotation, a minimum-channel override -- measured
// neutral and were removed: profiles/r05/gemm_block_order_pxg_bs320.txt, gemm_krot_neutral_bs320.txt)

void gemm_env() {
  if (g_gemm_mode < 0) {
    const char* e = getenv("MSP_CONV_GEMM");
    g_gemm_mode = (e == nullptr || e[0] != '0') ? 1 : 0;
  }
}

// co-tile choice: minimise (padded MFMA rows) + (pixel-operand re-staging per extra co tile).  Then the
// occupancy rule (round 6, profiles/r06/gemm_occupancy_bs320.txt): a launch of <= 12 BK-64 stages is bound by
// its blocks' fill and drain, which two blocks per CU cannot overlap -- the 32-KB tile at four blocks per CU
// wins there (L3 3x3 / d3 / 1x7 -9..-17 %, 1x1 shortcuts -11..-34 %) unless its 128-row tile pads the rows
// more than 1.35x the planner's tile (L3 fused-2, L4 3x3: 144 / 136 rows); longer K keeps the 2-block tiles.
int gemm_pick_cfg(int rows, int nk64) {
  if (g_gemm_cfg >= 0) return g_gemm_cfg;
  int best = 0;
  double best_cost = 1e30;
  for (int c = 0; c < kPlannerCfgs; ++c) {
    const int tco = 32 * kCfgs[c].wm * kCfgs[c].fm;
    const int tiles = cdiv(rows, tco);
    const double cost = (double)tiles * (tco + 48.0);   // + the B-operand staging each co tile repeats
    if (cost < best_cost - 1e-9) { best_cost = cost; best = c; }
  }
  const int tb = 32 * kCfgs[best].wm * kCfgs[best].fm, to = 32 * kCfgs[kOccCfg].wm * kCfgs[kOccCfg].fm;
  if (nk64 <= 12 && (double)cdiv(rows, to) * to <= 1.35 * cdiv(rows, tb) * tb) return kOccCfg;
  return best;
}

// the tap table as a regular grid (see TapGrid); false if it is not one
bool tap_grid(const ConvGeom& g, TapGrid& tg) {
  for (int kw = 1; kw <= g.T; ++kw) {
    if (g.T % kw != 0) continue;
    const int kh = g.T / kw;
    tg.kw = kw; tg.y0 = g.dy[0]; tg.x0 = g.dx[0];
    tg.ys = kh > 1 ? g.dy[kw] - g.dy[0] : 0;
    tg.xs = kw > 1 ? g.dx[1] - g.dx[0] : 0;
    bool ok = true;
    for (int t = 0; t < g.T && ok; ++t)
      ok = g.dy[t] == tg.y0 + (t / kw) * tg.ys && g.dx[t] == tg.x0 + (t % kw) * tg.xs;
    if (ok) return true;
  }
  return false;
}

// phase launch of a strided data-gradient (conv_gemm_phase): the output map and the A tap remap; the
// identity for every other launch
struct GemmPhase {
  int ps = 0, py = 0, px = 0, OHf = 0, OWf = 0;
  long apitch = 0;   // 0: g.Kp
  int akw = 0, ar0 = 0, ars = 1, ac0 = 0, acs = 1;   // akw 0: identity remap
};

template <int WM, int WN, int FM, int FN, int NS, int BK, bool BNE, int OCC = 2>
void launch_gemm(const ConvArgs& a, const GemmPhase& ph, hipStream_t s) {
  using C = GemmCfg<WM, WN, FM, FN, NS, BK>;
  const ConvGeom& g = a.g;
  GemmGeom gg;
  gg.OHW = (long)g.OH * g.OW;
  gg.M = (long)g.N * gg.OHW;
  gg.n_co = cdiv(g.Go * g.Cgo, C::TCO);
  gg.nk = cdiv(g.Kp, BK);
  gg.ps = ph.ps; gg.py = ph.py; gg.px = ph.px; gg.OWp = g.OW;
  gg.OHWp = gg.OHW; gg.OW = ph.OWf; gg.OHWf = (long)ph.OHf * ph.OWf;
  gg.apitch = ph.apitch > 0 ? ph.apitch : g.Kp;
  const long blocks = (long)cdiv(gg.M, C::TPX) * gg.n_co;
  static bool attr = false;
  if (!attr) {   // > 64 KB dynamic LDS: opted into once per instantiation, before any graph capture
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_gemm_kernel<WM, WN, FM, FN, NS, BK, BNE, OCC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  TapGrid tg;
  (void)tap_grid(g, tg);   // conv_gemm_ok checked it
  if (ph.akw > 0) {
    tg.akw = ph.akw; tg.ar0 = ph.ar0; tg.ars = ph.ars; tg.ac0 = ph.ac0; tg.acs = ph.acs;
  } else {
    tg.akw = tg.kw; tg.ar0 = 0; tg.ars = 1; tg.ac0 = 0; tg.acs = 1;
  }
  hipLaunchKernelGGL((conv_gemm_kernel<WM, WN, FM, FN, NS, BK, BNE, OCC>), dim3((unsigned)blocks), dim3(C::NT), C::LDS, s, a, gg,
                     tg);
}

template <bool BNE>
int dispatch_gemm(const ConvArgs& a, int cfg, const GemmPhase& ph, hipStream_t s) {
  switch (cfg) {
    case 0: launch_gemm<2, 2, 3, 2, 2, 64, BNE>(a, ph, s); return 0;
    case 1: launch_gemm<2, 2, 2, 2, 2, 64, BNE>(a, ph, s); return 0;
    case 2: launch_gemm<1, 4, 3, 1, 2, 64, BNE>(a, ph, s); return 0;
    case 3: launch_gemm<1, 4, 5, 1, 2, 64, BNE>(a, ph, s); return 0;
    case 4: launch_gemm<2, 2, 1, 2, 2, 64, BNE>(a, ph, s); return 0;
    case 5: launch_gemm<2, 2, 2, 2, 4, 32, BNE>(a, ph, s); return 0;
    case 6: launch_gemm<2, 2, 3, 2, 4, 32, BNE>(a, ph, s); return 0;
    case 7: launch_gemm<2, 2, 4, 2, 3, 32, BNE>(a, ph, s); return 0;
    case 8: launch_gemm<2, 2, 2, 2, 5, 32, BNE>(a, ph, s); return 0;
    case 9: launch_gemm<2, 2, 2, 2, 2, 32, BNE, 4>(a, ph, s); return 0;
  }
  return 1;
}

}  // namespace

// (no transposed indexing -- phase-decomposed elsewhere -- and no deferred-BN input prologue: the callers
// materialise wide deferred inputs, one normalise pass beats a per-k-step transform)
// min_c: the narrowest input group the DMA K walk takes -- a stage may cross one (group | tap) boundary, so
// Cgi >= the stage width: 64 for every tile, 32 with the 32-wide-stage tiles (gemm_tile_for)
static bool gemm_geom_ok(const ConvGeom& g, int min_c) {
  if (g.Cgi < min_c || g.Cgi % 8 != 0 || g.T > 30) return false;   // (T <= 30: the per-pixel tap bitmask)
  TapGrid tg;
  if (!tap_grid(g, tg)) return false;
  const long M = (long)g.N * g.OH * g.OW;
  return M >= 1 && (long)cdiv(M, kGemmTPX) * cdiv(g.Go * g.Cgo, 64) < (1L << 31);
}

// Eligibility: a forward (or stride-1 data-gradient) conv whose every input group is >= 64 channels wide --
// or >= 32 for a STRIDED forward (the 40-channel level's 3x3 s2 downsampling conv), which runs a 32-wide
// stage tile; narrower stride-1 convs keep the fused narrow / halo kernels
bool conv_gemm_ok(const ConvGeom& g, bool trans) {
  gemm_env();
  if (!g_gemm_mode || trans) return false;
  return gemm_geom_ok(g, g.stride > 1 ? 32 : 64);
}

// the tile of a launch: the planner's (or the forced) tile, moved to the 32-wide-stage tile when the input
// groups are narrower than its 64-wide stages
static int gemm_tile_for(const ConvGeom& g) {
  const int cfg = gemm_pick_cfg(g.Go * g.Cgo, cdiv(g.Kp, 64));
  return (g.Cgi < 64 && kCfgs[cfg].bk == 64) ? kOccCfg : cfg;
}

void conv_gemm_set(int on) { gemm_env(); g_gemm_mode = on ? 1 : 0; }
void conv_gemm_force_cfg(int cfg) { gemm_env(); g_gemm_cfg = (cfg >= 0 && cfg < kNumCfgs) ? cfg : -1; }
int conv_gemm_num_cfgs() { return kNumCfgs; }

long conv_gemm_stat_blocks(const ConvGeom& g) { return cdiv((long)g.N * g.OH * g.OW, kGemmTPX); }

int conv_gemm(const ConvArgs& a, hipStream_t s) {
  gemm_env();
  for (int i = 0; i < a.g.Gi; ++i)
    if (a.xc[i] != nullptr) return 2;   // no prologue on this path (see conv_gemm_ok)
  const int cfg = gemm_tile_for(a.g);
  const GemmPhase ph;
  return a.bn_y != nullptr ? dispatch_gemm<true>(a, cfg, ph, s) : dispatch_gemm<false>(a, cfg, ph, s);
}

// One phase (py, px) of a stride-s transposed conv (the strided data-gradient) as a stride-1 GEMM conv over
// the phase's output sub-grid: `a` carries the phase geometry (OH/OW = the sub-grid, taps = the phase's
// valid taps divided by s, stride 1) and the FULL packed weights; tA[v] = the packed tap of phase tap v.
// Returns 0, or 1 when the phase is not a GEMM launch (the caller runs the gather kernel): narrow input,
// irregular taps, a packed-tap subset that is not a strided grid, or no taps.
int conv_gemm_phase(const ConvArgs& a0, const int* tA, int KW, int s_, int py, int px, int OHf, int OWf,
                    hipStream_t s) {
  gemm_env();
  ConvArgs a = a0;
  ConvGeom& g = a.g;
  const long apitch = g.Kp;                            // the full packed rows
  g.Kp = (g.T * g.Gi * g.Cgi + 31) / 32 * 32;          // K of this phase's taps
  if (g.T < 1 || !g_gemm_mode || !gemm_geom_ok(g, 32) || a.bn_y != nullptr || a.stat_part != nullptr) return 1;
  for (int i = 0; i < g.Gi; ++i)
    if (a.xc[i] != nullptr || a.gy[i] != nullptr) return 1;
  TapGrid tg;
  if (!tap_grid(g, tg)) return 1;
  GemmPhase ph;
  ph.ps = s_; ph.py = py; ph.px = px; ph.OHf = OHf; ph.OWf = OWf; ph.apitch = apitch;
  const int kh = g.T / tg.kw;
  ph.akw = KW;
  ph.ar0 = tA[0] / KW; ph.ac0 = tA[0] % KW;
  ph.ars = kh > 1 ? tA[tg.kw] / KW - ph.ar0 : 0;
  ph.acs = tg.kw > 1 ? tA[1] % KW - ph.ac0 : 0;
  for (int v = 0; v < g.T; ++v)   // the packed taps must form that strided grid
    if (tA[v] != (ph.ar0 + (v / tg.kw) * ph.ars) * KW + ph.ac0 + (v % tg.kw) * ph.acs) return 1;
  const int cfg = gemm_tile_for(g);
  return dispatch_gemm<false>(a, cfg, ph, s) == 0 ? 0 : 2;
}

