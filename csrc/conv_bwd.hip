// Fused backward of a narrow stride-1 convolution: data-gradient AND weight-gradient from ONE staging of
// dY and x (the 17-channel DUCKNet level, reference models/ducknet.py:95-96,144-179: Widescope /
// Midscope / Residual / Separated chains of conv-BN-ReLU at full resolution).
//
// For a chain BN1 -> conv C -> BN2 the separate kernels move 8 full-resolution tensor passes per conv:
//   bn_act_bwd_apply(BN2)  read dz2, y2, write dy2        (3)
//   dgrad(C) + BN1 partials  read dy2, y1, write dz1       (3)
//   wgrad(C)                 read dy2, y1 (x = BN1(y1))    (2)
// Here one persistent kernel stages, per pixel tile, dY = bwd(dz2, y2) (the deferred BN2 backward, bwd8 --
// bit-identical to bn_act_bwd_apply) and x = relu(BN1(y1)) (the deferred forward prologue) into LDS once,
// then runs the data-gradient MFMAs (dz1 + BN1's backward partials in the epilogue) and accumulates the
// weight-gradient MFMAs of the same tile in registers: read dz2, y2, y1, write dz1 -- 4 passes.
//
// Tile: 4 waves x NJ x 16 output pixels (TH x TW), halo = the tap extents (symmetric tap sets only: the
// forward and backward halos coincide).  LDS: the dY halo tile [HH*HWD][py] and the x halo tile
// [HH*HWD][px] (pitch = an odd number of 16-B slots: the data-gradient's ds_read_b128 lane groups hit
// distinct banks), plus per-wave BN partial rows.  Data-gradient: the halo kernel's scheme (A = packed
// dgrad weights from L2 with a one-step prefetch, B = ds_read_b128 of the dY tile at per-unit tap offsets,
// v_mfma_f32_16x16x32_bf16, 32 rows = input channels <= 32).  Weight-gradient: dW[co][t][ci] = sum_p
// dY[p][co] x[p + tap_t][ci]: K = the tile's pixels in 32-pixel chunks, both operands read transposed
// (ds_read_b64_tr_b16) from the same LDS tiles; wave w owns taps w, w+4, w+8 and all (co, ci) 16x16 blocks,
// accumulating over the block's tiles; at the end each block writes its fp32 dW slab (deterministic split-K,
// summed in fixed order by unpack_wgrad).  Channels 24..31 of a 24-wide tile read the next pixel's data:
// those rows/columns of the 16x16 blocks are never stored.
#include "common.h"
#include "launchers.h"

namespace {

constexpr int kFbProd = 4;        // staging waves: tile i + 1 into the other LDS buffer meanwhile
// Compute waves CW (template): data- then weight-gradient of tile i.  CW = 8 (round 5): two per SIMD beside
// the staging wave -- the single compute wave per SIMD of the CW = 4 layout exposed its LDS / MFMA
// latencies (with every global load knocked out the kernel still took 3.04 of 3.15 ms at the L1 3x3,
// tools/dev/fused_bwd_bench.py).  At 768 threads the register cap is 168 per wave, so each wave keeps half
// the data-gradient columns and at most 2 weight-gradient (group, tap) units (wave, wave + 8).  CW = 4 stays
// for the 256-pixel tiles (dilation 3) and the Go = 2 pair, where it measured faster (conv_bwd_fused_plan).
constexpr int fb_threads(int cw) { return 64 * (cw + kFbProd); }
#ifndef FB_LDY
#define FB_LDY 3   // dY vectors (two loads each) per staging thread and batch; two batches in flight
#endif
#ifndef FB_LDX
#define FB_LDX 3   // x vectors per staging thread and batch (4 / 4 spill at the 168-register cap of CW = 8)
#endif
#ifndef FB_LDF
#define FB_LDF 8   // forward mode: x vectors per staging thread and batch (one load each, no x tile)
#endif
constexpr int kFbMaxKS = 24;      // data-gradient k-steps (T <= 9 taps x <= 4 slots / 4)
constexpr int kFbMaxT = 9;
constexpr int kFbMaxLds = 156 * 1024;  // two dY + x buffer pairs, the data-gradient weights, the BN partials
constexpr int kFbSlack = 64;      // elements past each tile (the 24..31 channel over-read of the last pixel)

typedef short s16x4_t __attribute__((ext_vector_type(4)));
DEVI uint2 fb_tr_read(const uint16_t* p) {
  s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4_t __attribute__((address_space(3)))*)(p));
  union { s16x4_t s; uint2 u; } c; c.s = v; return c.u;
}

// deferred BN(+ReLU) prologue of 8 staged channels: max(x * scale + shift, floor); c = [scale x 8][shift x 8]
DEVI uint4 xpro8(const uint4& v, const float* c, float floor) {
  float f[8];
  unpack8(v, f);
#pragma unroll
  for (int k = 0; k < 8; ++k) f[k] = fmaxf(fmaf(f[k], c[k], c[8 + k]), floor);
  return pack8(f);
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
DEVI uint4 fb_ldg4(const uint16_t* p) {   // global_load (never FLAT: see conv.hip ldg4)
  const u32x4_t v =
      *reinterpret_cast<const __attribute__((address_space(1))) u32x4_t*>(reinterpret_cast<uintptr_t>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// CB: 16-channel blocks of the data-gradient rows and of both weight-gradient operands: 2 (<= 32 channels, the
// 17-channel level) or 3 (<= 48: the 34-channel level, CW = 4, 256-pixel tiles; 128 for the Go = 2 pair); forward mode also 5 (the
// 34-channel level's 3x3 + 1x1 pair: 2 x 40 stacked output rows)
template <int CW, int NJ, bool BWD, bool XPRO, bool BNE, bool GO2 = false, bool FWD = false, int CB = 2>
__global__ __launch_bounds__(fb_threads(CW), 1) void conv_bwd_fused_kernel(FusedBwdArgs a, FusedBwdGeom fg) {
  constexpr int kFbWaves = CW, kFbThreads = fb_threads(CW), kFbTapGroups = CW;
  extern __shared__ uint4 fb_smem[];
  constexpr int MI = CB, CH = 16 * CB;        // data-gradient rows: input channels <= CH
  constexpr int NT = (kFbMaxT + 1 + kFbTapGroups - 1) / kFbTapGroups;   // weight-gradient units per wave
  constexpr int TP = kFbWaves * NJ * 16;      // pixels per tile
  constexpr int NCH = TP / 32;                // weight-gradient k chunks per tile
  const int hpx = fg.HH * fg.HWD;
  const int pair = hpx * (fg.py + fg.px) + 2 * kFbSlack;   // elements of one dY + x buffer pair
  uint16_t* const lds0 = reinterpret_cast<uint16_t*>(fb_smem);
  const int wp = 32 * fg.KS + 8;                           // weight row pitch (elements; +16 B: bank spread)
  uint16_t* const s_w = lds0 + 2 * pair;                   // [CH rows][wp] data-gradient weights, per block
  float* s_stat = reinterpret_cast<float*>(s_w + CH * wp);   // [waves][2][CH]
  constexpr int BTS = 2 * CH;                 // rebuild-table row: two stacked dY groups of <= CH channels
  __shared__ float s_bt[BWD ? 5 * BTS : 1];   // dY rebuild table (stacked groups): scale, shift (+inf: no
                                              // ReLU), k1, k2, k3
  __shared__ float s_xt[XPRO ? 2 * CH : 1];   // x prologue: scale, shift
  __shared__ float s_bn[BNE ? 5 * CH : 1];    // BN1 backward partials: scale, shift (+inf: no ReLU), mean,
                                              // and (lds_y) 1 / prologue scale, -shift / scale - mean
  __shared__ int s_ldsy;
  __shared__ int s_ub[kFbMaxKS * 4];          // data-gradient unit -> dY tile offset
  __shared__ int s_wb[kFbMaxT];               // weight-gradient tap -> x tile offset (pixel units)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int wt = wave;   // compute waves: weight-gradient units wt, wt + CW
  const int Ci = a.Ci, Co = a.Co, T = a.T;
  constexpr int Go = GO2 ? 2 : 1;
  const int C8g = Co >> 3, C8y = Go * C8g, C8x = Ci >> 3;   // dY: Go groups of Co channels, stacked
  const int nU0 = T * C8g, nU = nU0 + (Go == 2 ? C8g : 0);   // data-gradient K units (tap, 8 channels)
  const int nWU = T + (Go == 2 ? 1 : 0);                     // weight-gradient (group, tap) units
  if constexpr (BWD) {
    for (int c = tid; c < BTS; c += kFbThreads) {
      const int g = c >= Co ? 1 : 0, cl = c - g * Co;
      const float* gs = g ? a.gs2 : a.gs;
      const float* gk = g ? a.gk2 : a.gk;
      const bool on = c < Go * Co && (g ? a.gy2 : a.gy) != nullptr;
      s_bt[c] = on ? gs[cl] : 0.f;
      s_bt[BTS + c] = (on && (g ? a.grelu2 : a.grelu)) ? gs[Co + cl] : INFINITY;
      s_bt[2 * BTS + c] = on ? gk[cl] : 0.f;
      s_bt[3 * BTS + c] = on ? gk[Co + cl] : 0.f;
      s_bt[4 * BTS + c] = on ? gk[2 * Co + cl] : 0.f;
    }
  }
  if constexpr (XPRO) {
    const int Cx = FWD ? Co : Ci;   // FWD: the prologue applies to the staged input (Co slots)
    for (int c = tid; c < CH; c += kFbThreads) {
      const bool on = c < Cx;
      s_xt[c] = on ? a.xc[c] : 0.f;
      s_xt[CH + c] = on ? a.xc[Cx + c] : 0.f;
    }
  }
  // unit e -> (tap t, stacked 8-channel slot c8): group 0 over every tap, then group 1 at its one tap t1
  auto unit = [&](int e, int& t, int& c8) {
    if (e < nU0) { t = e / C8g; c8 = e - t * C8g; }
    else { t = a.t1; c8 = C8g + (e - nU0); }
  };
  for (int e = tid; e < fg.KS * 4; e += kFbThreads) {
    const int u = a.uperm[e];   // (host-built pairing, see FusedBwdArgs::uperm)
    int ub;
    if (u >= 0) {
      int t, c8;
      unit(u, t, c8);
      // data-gradient taps = the negated forward taps
      ub = ((-a.dy[t] - fg.ey0) * fg.HWD + (-a.dx[t] - fg.ex0)) * fg.py + 8 * c8;
    } else {
      ub = 0;   // padding unit (zero weights): slot 0 of the lane's own pixel -- always staged, never garbage
    }
    s_ub[e] = ub;
  }
  if (tid < kFbMaxT) s_wb[tid] = tid < T ? (a.dy[tid] * fg.HWD + a.dx[tid]) : 0;
  // lds_y: the BN epilogue's y1 is this conv's own input (the chain case: x = y1 through the BN1 prologue),
  // so y1 at the output pixels is rebuilt from the staged x tile instead of a global load in the epilogue
  // (whose latency, twice per tile, was the critical path of the compute waves: with the MFMA loops knocked
  // out the kernel still took 87 % of its time).  For t = sc*y1 + sh: ReLU mask = x > 0, y1 - mean =
  // x / sc - sh / sc - mean (x = bf16(t): the rounding of the stored activation).  Needs sc != 0.
  if (tid == 0) s_ldsy = (BNE && XPRO && (const void*)a.bn_y == (const void*)a.x) ? 1 : 0;
  __syncthreads();
  if constexpr (BNE) {
    for (int c = tid; c < CH; c += kFbThreads) {
      const bool on = c < Ci;
      s_bn[c] = on ? a.bn_coef[c] : 0.f;
      s_bn[CH + c] = (on && a.bn_relu) ? a.bn_coef[Ci + c] : INFINITY;
      s_bn[2 * CH + c] = on ? a.bn_coef[2 * Ci + c] : 0.f;
      if constexpr (XPRO) {
        const float sc = on ? a.xc[c] : 1.f, sh = on ? a.xc[Ci + c] : 0.f;
        const float inv = 1.f / sc;
        s_bn[3 * CH + c] = inv;
        s_bn[4 * CH + c] = on ? fmaf(-sh, inv, -a.bn_coef[2 * Ci + c]) : 0.f;
        if (!(sc != 0.f) || !isfinite(inv)) s_ldsy = 0;   // (benign race: every writer stores 0)
      }
    }
  }
  {   // the data-gradient weights stay resident, in unit order: no global latency inside the k loop
    const int rowv = 4 * fg.KS;   // uint4 per row
    for (int e = tid; e < CH * rowv; e += kFbThreads) {
      const int r = e / rowv, u = e - r * rowv;
      const int pu = a.uperm[u];
      uint4 v = make_uint4(0, 0, 0, 0);
      if (pu >= 0) {
        int t, c8;
        unit(pu, t, c8);   // packed dgrad weights: k = t * (Go*Co) + stacked channel
        v = *reinterpret_cast<const uint4*>(a.wd + (long)r * a.Kp + t * (Go * Co) + 8 * c8);
      }
      *reinterpret_cast<uint4*>(s_w + r * wp + 8 * u) = v;
    }
  }
  if (BNE)
    for (int c = tid; c < kFbWaves * 2 * CH; c += kFbThreads) s_stat[c] = 0.f;
  __syncthreads();

  const int per_img = fg.tiles_y * fg.tiles_x;
  const long img_px = (long)a.H * a.W;
  auto tile_origin = [&](int tt, int& ty0, int& tx0, long& imoff) {
    const int n = tt / per_img, trem = tt - n * per_img;
    const int tyi = trem / fg.tiles_x;
    ty0 = tyi * fg.TH;
    tx0 = (trem - tyi * fg.tiles_x) * fg.TW;
    imoff = (long)n * img_px;
  };
  const bool producer = wave >= kFbWaves;   // wave-uniform role
  if (producer) {
    // ---- staging waves: a continuous software pipeline of load batches over this block's tiles ------------
    // Tile k (= blockIdx.x + k * gridDim.x) goes to LDS buffer pair k & 1.  Each batch is LDY dY vectors
    // (dz2 + y2: dY = bwd(dz2, y2), bwd8) and LDX x vectors (y1: x = relu(BN1(y1))) per thread, every load
    // issued unconditionally (out-of-image / past-the-end entries load a valid pixel and store zero / nothing),
    // so the compiler's counted vmcnt waits retire exactly the batch being written: batch q + 1 (possibly the
    // next tile's first) is in flight while batch q is transformed into LDS, and across the tile barrier.
    // (Round 4 staged one tile at a time with every batch's latency exposed: ~2.2 TB/s.)
    const int st = tid - 64 * kFbWaves;
    constexpr int NP = 64 * kFbProd;
    constexpr int LDY = FWD ? FB_LDF : FB_LDY, LDX = FB_LDX;
    // Fixed-slot staging: thread st serves ONE 8-channel slot c8 = st % C8 for the halo pixels st / C8 +
    // k * (NP / C8), k = 0, 1, ... ((NP / C8) * C8 threads per role; the others issue clamped loads and store
    // nothing).  The slot's BN coefficients then live in registers (round 5's element-order staging read 10
    // LDS vectors of bwd8 coefficients per dY vector) and the pixel cursor advances by a constant with one
    // carry; image offsets are 32-bit per image.
    const int PY = NP / C8y, PX = FWD ? 1 : NP / C8x;             // pixels per step of a role
    const int c8y = st % C8y, c8x = FWD ? 0 : st % C8x;
    const bool acty = st < PY * C8y, actx = !FWD && st < PX * C8x;
    const int jobsY = (hpx + PY - 1) / PY, jobsX = FWD ? 0 : (hpx + PX - 1) / PX;
    const int NB = max((jobsY + LDY - 1) / LDY, (jobsX + LDX - 1) / LDX);
    const int ntb = (fg.ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;   // grid <= ntiles
    const int Q = ntb * NB;
    struct Batch {
      uint4 v[LDY], w[LDY], x[LDX];
      int dy[LDY], dx[LDX];   // LDS element offset << 2 | in-image << 1; -1: nothing to store
      int buf;
    };
    struct Cursor { int hy, hx; };   // (a pixel past the halo has hy >= HH)
    struct Step { int a, b; };       // pixel step = a rows + b columns
    auto cursor0 = [&](int C8) {
      const int hp = st / C8, hy = hp / fg.HWD;
      return Cursor{hy, hp - hy * fg.HWD};
    };
    auto step_of = [&](int P) { const int a = P / fg.HWD; return Step{a, P - a * fg.HWD}; };
    auto advance = [&](Cursor& c, const Step& t) {
      c.hx += t.b;
      c.hy += t.a;
      if (c.hx >= fg.HWD) { c.hx -= fg.HWD; ++c.hy; }
    };
    const Step sy = step_of(PY), sx = FWD ? Step{} : step_of(PX);
    // this thread's slot: the dY group (GO2) and whether its dY is rebuilt (a plain gradient group is stored as
    // loaded), its coefficient registers (BWD: bwd8's [scale, shift, k1, k2, k3] x 8; the prologues: scale,
    // shift x 8) and LDS column offsets
    const bool g2y = GO2 && c8y >= C8g;
    const int cly = 8 * (c8y - (g2y ? C8g : 0));
    const uint16_t* const dzbase = g2y ? a.dz2 : a.dz;
    const uint16_t* const ybase = g2y ? a.gy2 : a.gy;
    const bool try_ = BWD && (!GO2 || ybase != nullptr);
    float cfy[BWD ? 40 : ((FWD && XPRO) ? 16 : 1)];
    if constexpr (BWD) {
#pragma unroll
      for (int r = 0; r < 5; ++r)
#pragma unroll
        for (int e = 0; e < 8; ++e) cfy[8 * r + e] = s_bt[BTS * r + 8 * c8y + e];
    } else if constexpr (FWD && XPRO) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { cfy[e] = s_xt[8 * c8y + e]; cfy[8 + e] = s_xt[CH + 8 * c8y + e]; }
    }
    float cfx[(!FWD && XPRO) ? 16 : 1];
    if constexpr (!FWD && XPRO) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { cfx[e] = s_xt[8 * c8x + e]; cfx[8 + e] = s_xt[CH + 8 * c8x + e]; }
    }
    Cursor cy{}, cx{};
    auto issue = [&](int k, int b, Batch& B) {
      int ty0, tx0;
      long imoff;
      tile_origin((int)blockIdx.x + min(k, ntb - 1) * (int)gridDim.x, ty0, tx0, imoff);
      B.buf = k & 1;
      if (b == 0) {   // (re-derived per tile rather than kept: registers)
        cy = cursor0(C8y);
        if (!FWD) cx = cursor0(C8x);
      }
      const int gy0 = ty0 + fg.ey0, gx0 = tx0 + fg.ex0;   // image row / column of halo pixel (0, 0)
      const uint16_t* const dzb = dzbase + imoff * Co;
#pragma unroll
      for (int u = 0; u < LDY; ++u) {
        const bool valid = acty && cy.hy < fg.HH;
        const int iy = gy0 + cy.hy, ix = gx0 + cy.hx;
        const bool in = valid && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
        const unsigned off = in ? (unsigned)((iy * a.W + ix) * Co + cly) : 0u;   // within the image
#ifndef FB_KO_LOADS   // (profiling knock-out builds only: csrc/build.py MSP_BUILD_DEFINES)
        B.v[u] = fb_ldg4(dzb + off);
        if (BWD) B.w[u] = fb_ldg4(try_ ? ybase + imoff * Co + off : dzb + off);
#else
        B.v[u] = make_uint4(0, 0, 0, 0);
        B.w[u] = make_uint4(0, 0, 0, 0);
#endif
        B.dy[u] = valid ? (((cy.hy * fg.HWD + cy.hx) * fg.py + 8 * c8y) << 2 | (in ? 2 : 0)) : -1;
        advance(cy, sy);
      }
#pragma unroll
      for (int u = 0; u < (FWD ? 0 : LDX); ++u) {
        const bool valid = actx && cx.hy < fg.HH;
        const int iy = gy0 + cx.hy, ix = gx0 + cx.hx;
        const bool in = valid && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
        const unsigned off = in ? (unsigned)((iy * a.W + ix) * Ci + 8 * c8x) : 0u;
#ifndef FB_KO_LOADS
        B.x[u] = fb_ldg4(a.x + imoff * Ci + off);
#else
        B.x[u] = make_uint4(0, 0, 0, 0);
#endif
        B.dx[u] = valid ? (((cx.hy * fg.HWD + cx.hx) * fg.px + 8 * c8x) << 2 | (in ? 2 : 0)) : -1;
        advance(cx, sx);
      }
    };
    const float xfloor = a.xrelu ? 0.f : -INFINITY;   // the prologue's ReLU (uniform: no per-channel table)
    auto commit = [&](const Batch& B) {
      uint16_t* const tY = lds0 + B.buf * pair;
      uint16_t* const tX = tY + hpx * fg.py + kFbSlack;
#pragma unroll
      for (int u = 0; u < LDY; ++u) {
        const int d = B.dy[u];
        if (d < 0) continue;
        uint4 val = B.v[u];
        if (BWD && try_) val = bwd8(val, B.w[u], cfy, 8);
        if (FWD && XPRO) val = xpro8(val, cfy, xfloor);   // forward: BN(+ReLU) of x
        if (!(d & 2)) val = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(tY + (d >> 2)) = val;
      }
#pragma unroll
      for (int u = 0; u < (FWD ? 0 : LDX); ++u) {
        const int d = B.dx[u];
        if (d < 0) continue;
        uint4 val = B.x[u];
        if (XPRO) val = xpro8(val, cfx, xfloor);
        if (!(d & 2)) val = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(tX + (d >> 2)) = val;
      }
    };
    Batch B0, B1;
    int k0 = 0, b0 = 0;   // batch q's tile / batch within the tile
    auto next = [&](int& k, int& b) { if (++b == NB) { b = 0; ++k; } };
    // (issues are unconditional -- past the end a clamped batch that is never committed -- so that every
    // commit's vmcnt wait is the exact count of the one batch issued after it)
    issue(0, 0, B0);
    for (int q = 0; q < Q; q += 2) {
      int k1 = k0, b1 = b0;
      next(k1, b1);
      issue(k1, b1, B1);
      commit(B0);
      if (b0 == NB - 1) __syncthreads();   // tile k0 staged
      if (q + 1 >= Q) break;
      int k2 = k1, b2 = b1;
      next(k2, b2);
      issue(k2, b2, B0);
      commit(B1);
      if (b1 == NB - 1) __syncthreads();
      k0 = k2; b0 = b2;
    }
    __syncthreads();   // the compute waves' last tile
    if (BNE || (FWD && a.stat_part != nullptr)) __syncthreads();   // (the BN partials' exchange below)
    return;
  }
  // FWD: the bias of this lane's output channels, read once (a global load in the epilogue put a vmcnt(0)
  // there, which also waited for every store of the tile before it)
  float bias4[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 16 * i + 4 * lg + r;
      bias4[i][r] = (FWD && a.bias != nullptr && c < a.Co_l) ? a.bias[c] : 0.f;
    }
  // data-gradient: the wave's NJ 16-pixel columns -> dY tile pixel offsets
  int pb[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int p = (wave * NJ + j) * 16 + lr;
    pb[j] = ((p >> fg.tw_shift) * fg.HWD + (p & (fg.TW - 1))) * fg.py;   // + s_ub: tap offset - halo origin
  }
  // weight-gradient transposed reads: lane (lr, lg) reads chunk pixels plo / phi, channels 4 p4 .. + 3 (+ 16 i)
  const int q = lr >> 2, p4 = lr & 3;
  // The chunk's 32 pixels are the MFMA's k; any bijection works when the dY and x reads share it.  One
  // ds_read_b64_tr_b16 serves 32 lanes per cycle = 8 pixels x 32 B: at an odd-16-B-slot pixel pitch (48 / 80 /
  // 112 B) 8 pixels of ONE parity cover the 256-B bank row exactly once, mixed parities collide (PMC: bank
  // conflict rate 0.39 with the consecutive mapping 8 lg + q).  So lanes 0-31 (lg 0, 1) take the even and lanes
  // 32-63 the odd pixels of each 16-pixel half, and the second 8 k of a lane come from the other half (+ 16).
  const int plo = 2 * (4 * (lg & 1) + q) + (lg >> 1), phi = plo + 16;
  // lane part of a chunk's halo pixels: element offsets in the dY / x tiles (phi may be in the next tile row)
  const int Ly = (plo >> fg.tw_shift) * fg.HWD + (plo & (fg.TW - 1));
  const int Lh = (phi >> fg.tw_shift) * fg.HWD + (phi & (fg.TW - 1));
  const int offYlo = Ly * fg.py + 4 * p4, offYhi = Lh * fg.py + 4 * p4;
  const int offXlo = Ly * fg.px + 4 * p4, offXhi = Lh * fg.px + 4 * p4;
  int swx[NT];
#pragma unroll
  for (int m = 0; m < NT; ++m) {
    const int u = wt + kFbTapGroups * m;
    swx[m] = u < nWU ? s_wb[(GO2 && u >= T) ? a.t1 : u] * fg.px : 0;
  }

  f32x4_t accw[NT][CB][CB];
#pragma unroll
  for (int m = 0; m < NT; ++m)
#pragma unroll
    for (int i = 0; i < CB; ++i)
#pragma unroll
      for (int j = 0; j < CB; ++j) accw[m][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float cs[MI][4], cq[MI][4];   // BN1 partials (BNE), over the block's tiles
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) { cs[i][r] = 0.f; cq[i][r] = 0.f; }

  __syncthreads();   // tile 0 staged
  int it = 0;
  for (int tt = blockIdx.x; tt < fg.ntiles; tt += gridDim.x, ++it) {
    uint16_t* const cur = lds0 + (it & 1) * pair;
    int ty0, tx0;
    long imoff;
    tile_origin(tt, ty0, tx0, imoff);
    const uint16_t* const tY = cur;
    const uint16_t* const tX = cur + hpx * fg.py + kFbSlack;

    // ---- data-gradient: dz1 = conv(dY, W_d) (+ BN1 backward partials) -----------------------------------
    {
      const uint16_t* wrow[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) wrow[i] = s_w + (16 * i + lr) * wp + 8 * lg;
      // BN1: this tile's y1 at the output pixels; the first row block's loads go out ahead of the k loop
      // (their latency under the MFMAs), the second's ahead of the first block's epilogue
      uint2 yy[2][NJ];   // row blocks i and i + 1 (a ring: at most two in flight)
      // per-image element offset of column j's output pixel (-1: outside the image; one image < 2^31 elements)
      auto pixi = [&](int j) -> int {   // per-image pixel index of column j (-1: outside the image)
        const int p = (wave * NJ + j) * 16 + lr;
        const int ty = ty0 + (p >> fg.tw_shift), tx = tx0 + (p & (fg.TW - 1));
        return (ty < a.H && tx < a.W) ? ty * a.W + tx : -1;
      };
      auto pix = [&](int j) -> int {
        const int pp = pixi(j);
        return pp >= 0 ? pp * Ci : -1;
      };
      // FWD: output pitch opitch; a Go = 2 pair's rows >= co_split store into the second output tensor
      const int opitch = FWD ? a.opitch : Ci;
      uint16_t* const dxo_im = a.dxo + imoff * opitch;   // this tile's image
      uint16_t* const dxo2_im = FWD && a.co_split > 0 ? a.dxo2 + imoff * opitch : nullptr;
      // accumulate (never with BNE, conv_bwd_fused): the ring prefetches the stored dx instead of y1 -- a load in the
      // epilogue itself exposed its whole latency (+0.76 ms on an L1 launch at bs320)
      const bool accum = !FWD && a.accum != 0;   // block-uniform
      const uint16_t* const bny_im = accum ? dxo_im : (BNE ? a.bn_y + imoff * Ci : nullptr);
      auto load_y = [&](int i) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int pm = pix(j);
          yy[i & 1][j] = (pm >= 0 && 16 * i + 4 * lg < Ci) ? *reinterpret_cast<const uint2*>(bny_im + pm + 16 * i + 4 * lg)
                                                       : make_uint2(0, 0);
        }
      };
      const bool lds_y = BNE && XPRO && s_ldsy != 0;   // block-uniform
      const bool ring = (BNE && !lds_y) || accum;
      if (ring) load_y(0);
      f32x4_t acc[MI][NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#ifdef FB_KO_DGRAD
      for (int ks = 0; ks < 0; ++ks) {
#else
      for (int ks = 0; ks < fg.KS; ++ks) {
#endif
        uint4 A[MI];
#pragma unroll
        for (int i = 0; i < MI; ++i) A[i] = *reinterpret_cast<const uint4*>(wrow[i] + 32 * ks);
        const int ub = s_ub[4 * ks + lg];
        uint4 B[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) B[j] = *reinterpret_cast<const uint4*>(tY + pb[j] + ub);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16x16x32(A[i], B[j], acc[i][j]);
      }
      // epilogue: dz1 (bf16, NHWC) for the in-image pixels and channels < Ci
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if (ring && i + 1 < MI) load_y(i + 1);
        const int cb = 16 * i + 4 * lg;
        if (cb >= Ci) continue;
        const bool og2 = FWD && a.co_split > 0 && cb >= a.co_split;   // (4-row blocks never straddle the split)
        uint16_t* const obase = og2 ? dxo2_im + (cb - a.co_split) : dxo_im + cb;
        float sc[4], sh[4], mu[4];
        if (BNE) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sc[r] = lds_y ? s_bn[3 * CH + cb + r] : s_bn[cb + r];
            sh[r] = s_bn[CH + cb + r];
            mu[r] = lds_y ? s_bn[4 * CH + cb + r] : s_bn[2 * CH + cb + r];
          }
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int pp = pixi(j);
          if (pp < 0) continue;
          f32x4_t v = acc[i][j];
          if (FWD) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += bias4[i][r];
          } else if (accum) {   // sibling launches' data-gradients into one tensor (the ring's prefetched dx)
            const uint2 ov = yy[i & 1][j];
            v[0] += __uint_as_float(ov.x << 16); v[1] += __uint_as_float(ov.x & 0xffff0000u);
            v[2] += __uint_as_float(ov.y << 16); v[3] += __uint_as_float(ov.y & 0xffff0000u);
          }
          const uint32_t lo = pack2(v[0], v[1]), hi = pack2(v[2], v[3]);
#ifndef FB_KO_STORE   // (profiling knock-out builds only)
          *reinterpret_cast<uint2*>(obase + pp * opitch) = make_uint2(lo, hi);
#endif
          if (FWD) {   // the output's BN statistics, of the stored (bf16) values
            const float g4[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                 __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              cs[i][r] += g4[r];
              cq[i][r] = fmaf(g4[r], g4[r], cq[i][r]);
            }
          }
          if (BNE) {
            const float g4[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                 __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
            if (lds_y) {   // y1 from the staged x tile (this output pixel's halo slot)
              const int p = (wave * NJ + j) * 16 + lr;
              const int hp = ((p >> fg.tw_shift) - fg.ey0) * fg.HWD + ((p & (fg.TW - 1)) - fg.ex0);
              const uint2 xv = *reinterpret_cast<const uint2*>(tX + hp * fg.px + cb);
              const float x4[4] = {__uint_as_float(xv.x << 16), __uint_as_float(xv.x & 0xffff0000u),
                                   __uint_as_float(xv.y << 16), __uint_as_float(xv.y & 0xffff0000u)};
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float gr = (!a.bn_relu || x4[r] > 0.f) ? g4[r] : 0.f;
                cs[i][r] += gr;
                cq[i][r] += gr * fmaf(x4[r], sc[r], mu[r]);
              }
            } else {
              const float y4[4] = {__uint_as_float(yy[i & 1][j].x << 16), __uint_as_float(yy[i & 1][j].x & 0xffff0000u),
                                   __uint_as_float(yy[i & 1][j].y << 16), __uint_as_float(yy[i & 1][j].y & 0xffff0000u)};
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float gr = fmaf(y4[r], sc[r], sh[r]) > 0.f ? g4[r] : 0.f;
                cs[i][r] += gr;
                cq[i][r] += gr * (y4[r] - mu[r]);
              }
            }
          }
        }
      }
    }

    // ---- weight-gradient: accw[m][i][j] += dY[chunk][co block i]^T x[chunk + tap][ci block j] ----------
#ifdef FB_KO_WGRAD
    for (int s = 0; s < 0; ++s) {
#else
#pragma unroll 2
    for (int s = 0; s < (FWD ? 0 : NCH); ++s) {
#endif
      // chunk s's halo pixel = a uniform part (the chunk's first tile pixel) + this lane's constant part: one
      // scalar product per chunk instead of per-lane shifts and multiplies for every operand address
      const int S = (((32 * s) >> fg.tw_shift) - fg.ey0) * fg.HWD + ((32 * s) & (fg.TW - 1)) - fg.ex0;
      const uint16_t* const y0 = tY + S * fg.py;
      const uint16_t* const x0 = tX + S * fg.px;
      uint4 fa[CB];
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        const uint2 lo = fb_tr_read(y0 + offYlo + 16 * i);
        const uint2 hi = fb_tr_read(y0 + offYhi + 16 * i);
        fa[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
#pragma unroll
      for (int m = 0; m < NT; ++m) {
        const int u = wt + kFbTapGroups * m;   // (group, tap) unit: group 0's taps, then group 1's tap t1
        if (u >= nWU) break;   // wave-uniform
        if (GO2 && u >= T) {   // the second group's dY columns; its unit is the wave's last, so fa is overwritten
#pragma unroll
          for (int i = 0; i < CB; ++i) {
            const uint2 lo = fb_tr_read(y0 + offYlo + Co + 16 * i);
            const uint2 hi = fb_tr_read(y0 + offYhi + Co + 16 * i);
            fa[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
          }
        }
        const uint16_t* const xb = x0 + swx[m];
#pragma unroll
        for (int j = 0; j < CB; ++j) {
          const uint2 lo = fb_tr_read(xb + offXlo + 16 * j);
          const uint2 hi = fb_tr_read(xb + offXhi + 16 * j);
          const uint4 fb = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
          for (int i = 0; i < CB; ++i) accw[m][i][j] = mfma16x16x32(fa[i], fb, accw[m][i][j]);
        }
      }
    }
    __syncthreads();   // tile i consumed, tile i + 1 staged
  }   // tile loop

  // ---- BN partials (BN1's backward, or FWD: the output's statistics): this block's row ------------------------
  if (BNE || (FWD && a.stat_part != nullptr)) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int cb = 16 * i + 4 * lg;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s2 = row16_sum(cs[i][r]), q2 = row16_sum(cq[i][r]);
        if (lr == 0 && cb + r < Ci) {
          s_stat[(wave * 2 + 0) * CH + cb + r] = s2;
          s_stat[(wave * 2 + 1) * CH + cb + r] = q2;
        }
      }
    }
    __syncthreads();
    for (int c = tid; c < Ci; c += 64 * kFbWaves) {   // (compute waves only: the staging waves have left)
      float s2 = 0.f, q2 = 0.f;
#pragma unroll
      for (int wv = 0; wv < kFbWaves; ++wv) { s2 += s_stat[(wv * 2 + 0) * CH + c]; q2 += s_stat[(wv * 2 + 1) * CH + c]; }
      a.stat_part[((long)blockIdx.x * 2 + 0) * Ci + c] = s2;
      a.stat_part[((long)blockIdx.x * 2 + 1) * Ci + c] = q2;
    }
  }
  if constexpr (FWD) return;
  // ---- dW slab of this block: [Go*Co][T * Ci], element (g*Co + co, t*Ci + ci) ----------------------------
  float* slab = a.dw + (long)blockIdx.x * (Go * Co) * (T * Ci);
#pragma unroll
  for (int m = 0; m < NT; ++m) {
    const int u = wt + kFbTapGroups * m;
    if (u >= nWU) break;
    const int g = (GO2 && u >= T) ? 1 : 0, t = g ? a.t1 : u;
#pragma unroll
    for (int i = 0; i < CB; ++i)
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        const int ci = 16 * j + lr;
        if (ci >= Ci) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = 16 * i + 4 * lg + r;
          if (co < Co) slab[(long)(g * Co + co) * (T * Ci) + t * Ci + ci] = accw[m][i][j][r];
        }
      }
  }
}

// K-unit order of the data-gradient: positions 4ks + {0, 1} and 4ks + {2, 3} are the two k-groups that one
// ds_read_b128 lane group mixes (MI355X_MICROARCH §LDS); a pair whose dY tile offsets are equal in 16-B slots
// mod 16 covers the 16 slots of a 256-B bank row exactly once (16 consecutive pixels at an odd slot pitch).
// Greedy: each pair takes the first free unit and a free unit of the same residue, else any free unit, else
// a padding unit (zero weights; it reads slot 0 of the lane's pixel: an offset chosen for its bank residue
// could land on a never-staged padding slot, and 0 x NaN garbage is NaN).
void fb_unit_order(FusedBwdArgs& a, const FusedBwdGeom& fg) {
  const int C8g = a.Co / 8, nU0 = a.T * C8g, nU = nU0 + (a.Go == 2 ? C8g : 0), n = 4 * fg.KS;
  int res[96];
  bool used[96] = {false};
  for (int u = 0; u < nU; ++u) {
    int t, c8;
    if (u < nU0) { t = u / C8g; c8 = u - t * C8g; } else { t = a.t1; c8 = C8g + (u - nU0); }
    const int ub = ((-a.dy[t] - fg.ey0) * fg.HWD + (-a.dx[t] - fg.ex0)) * fg.py + 8 * c8;
    res[u] = (ub / 8) & 15;
  }
  int pos = 0;
  for (int first = 0; pos < n; ) {
    while (first < nU && used[first]) ++first;
    if (first >= nU) {   // only padding left
      a.uperm[pos++] = (short)(-1);
      continue;
    }
    used[first] = true;
    a.uperm[pos++] = (short)first;
    int mate = -1;
    for (int u = first + 1; u < nU; ++u)
      if (!used[u] && res[u] == res[first]) { mate = u; break; }
    if (mate >= 0) {
      used[mate] = true;
      a.uperm[pos++] = (short)mate;
    } else {
      int u = first + 1;
      while (u < nU && used[u]) ++u;
      if (u < nU) { used[u] = true; a.uperm[pos++] = (short)u; }
      else a.uperm[pos++] = (short)(-1);
    }
  }
}

size_t fb_pair_lds(const FusedBwdGeom& fg) {
  return ((size_t)fg.HH * fg.HWD * (fg.py + fg.px) + 2 * kFbSlack) * 2;
}

size_t fb_lds(const FusedBwdGeom& fg) {
  return 2 * fb_pair_lds(fg) + (size_t)16 * fg.cb * (32 * fg.KS + 8) * 2 + (size_t)fg.cw * 2 * 16 * fg.cb * 4;
}

}  // namespace

// Plan: eligible shapes and the tile geometry (0 = not eligible).  Symmetric tap sets only (3x3 with any
// dilation, 1x7 / 7x1): the dY halo of the data-gradient and the x halo of the weight-gradient coincide.
// fwd: the forward mode (conv_fwd_fused): x staged in the dY slots, no x tile, any tap set (the halo is the
// forward taps' extent; the kernel gets the negated taps so that its data-gradient offsets walk them)
static bool fb_plan(const ConvGeom& g, FusedBwdGeom& fg, bool fwd) {
  // Go == 2: the ResidualBlock's 3x3 + 1x1 pair (the 1x1 at one tap of the 3x3's grid, FusedBwdArgs::t1) --
  // backward: two dY groups; forward: one staged input, the two groups' outputs as stacked kernel rows
  if (g.stride != 1 || g.Gi != 1 || g.Go < 1 || g.Go > 2 || g.OH != g.IH || g.OW != g.IW) return false;
  const int orows = fwd ? g.Go * g.Cgo : g.Cgo;   // the kernel's data-gradient rows (fwd: output channels)
  // <= 32 channels: 2 sixteen-channel blocks; <= 48 (the 34-channel level, the 24-channel pair's forward): 3;
  // <= 80 (forward only: the 40-channel pair's two stacked output groups): 5
  const int mc = std::max(g.Cgi, orows);
  const int cb = mc > 48 ? 5 : (mc > 32 ? 3 : 2);
  if (g.Cgi > 48 || orows > (fwd ? 80 : 48) || (cb == 5 && orows <= 64) ||
      g.Cgi % 8 || g.Cgo % 8 || g.T > kFbMaxT || g.T < 2)
    return false;
  int ey0 = 0, ey1 = 0, ex0 = 0, ex1 = 0;
  for (int t = 0; t < g.T; ++t) {
    bool mirrored = false;
    for (int u = 0; u < g.T; ++u) mirrored |= g.dy[u] == -g.dy[t] && g.dx[u] == -g.dx[t];
    if (!mirrored && !fwd) return false;
    ey0 = std::min(ey0, g.dy[t]); ey1 = std::max(ey1, g.dy[t]);
    ex0 = std::min(ex0, g.dx[t]); ex1 = std::max(ex1, g.dx[t]);
  }
  const int Gy = fwd ? 1 : g.Go;   // staged dY groups (fwd: the one input)
  const int C8g = (fwd ? g.Cgi : g.Cgo) / 8, C8y = Gy * C8g, C8x = fwd ? 0 : g.Cgi / 8;
  const int py = 8 * ((C8y & 1) ? C8y : C8y + 1), px = fwd ? 0 : 8 * ((C8x & 1) ? C8x : C8x + 1);
  const int KS = (g.T * C8g + (Gy == 2 ? C8g : 0) + 3) / 4;
  if (KS > kFbMaxKS) return false;
  double best = 1e30;
  bool found = false;
  // (128-pixel tiles: only the 34-channel level's dilated / wide halos, which fit no larger double buffer)
  for (int tp = 512; tp >= (cb == 3 && !fwd ? 128 : 256); tp /= 2) {
    if (tp == 128 && found) break;
    // (cb 3 backward: the 9 x 4 weight-gradient accumulators of 3 units need the 256-register budget of CW 4)
    // (8 compute waves for one output group, 4 for the Go = 2 pair: profiles/r05/fused_bwd_cw_and_knockouts_bs320.txt)
    // (cb 5: the 5 x NJ data-gradient accumulators exceed the 168-register cap of CW 8)
    const int cw = (tp <= 256 || (cb == 3 && !fwd) || cb == 5) ? 4 : (Gy == 1 ? 8 : 4);
    const int nj = tp / (16 * cw);
    if ((cb == 3 && !fwd && (tp == 512 || (Gy == 2 && nj != 2))) || (cb == 5 && nj != 4)) continue;   // (no instantiation)
    for (int tw = 16; tw <= 64; tw *= 2) {
      const int th = tp / tw;
      FusedBwdGeom c{};
      if (th < 1) continue;
      c.TH = th; c.TW = tw; c.tw_shift = tw == 16 ? 4 : (tw == 32 ? 5 : 6);
      c.HH = th + ey1 - ey0; c.HWD = tw + ex1 - ex0; c.ey0 = ey0; c.ex0 = ex0;
      c.py = py; c.px = px; c.KS = KS; c.nj = nj; c.cw = cw; c.cb = cb;
      if (fb_lds(c) > (size_t)kFbMaxLds) continue;
      const double tiles = (double)((g.OH + th - 1) / th) * ((g.OW + tw - 1) / tw);
      const double cost = tiles * ((double)c.HH * c.HWD * (C8y + C8x) + 0.25 * tp * (C8x + C8y));
      if (cost < best * 0.999) {
        best = cost;
        found = true;
        fg = c;
      }
    }
  }
  if (!found) return false;
  fg.inv_c8y = 1.0f / (float)C8y;
  fg.inv_c8x = fwd ? 0.f : 1.0f / (float)C8x;
  fg.inv_hwd = 1.0f / (float)fg.HWD;
  fg.tiles_y = (g.OH + fg.TH - 1) / fg.TH;
  fg.tiles_x = (g.OW + fg.TW - 1) / fg.TW;
  fg.ntiles = (long)g.N * fg.tiles_y * fg.tiles_x <= (1L << 30) ? g.N * fg.tiles_y * fg.tiles_x : 0;
  return fg.ntiles > 0;
}

bool conv_bwd_fused_plan(const ConvGeom& g, FusedBwdGeom& fg) { return fb_plan(g, fg, false); }

int conv_bwd_fused_blocks(const ConvGeom& g) {
  FusedBwdGeom fg;
  if (!conv_bwd_fused_plan(g, fg)) return 0;
  return std::min(fg.ntiles, kFusedBwdGrid);
}

int conv_bwd_fused(const FusedBwdArgs& a0, const ConvGeom& g, hipStream_t s) {
  FusedBwdGeom fg;
  if (!conv_bwd_fused_plan(g, fg)) return 8;
  FusedBwdArgs a = a0;
  a.N = g.N; a.H = g.IH; a.W = g.IW; a.Ci = g.Cgi; a.Co = g.Cgo; a.T = g.T;   // a.Kp: the dgrad packing's Kp
  a.Go = g.Go;
  if (g.Go == 2 && (a.dz2 == nullptr || a.t1 < 0 || a.t1 >= g.T)) return 8;
  if (a.accum && a.bn_y != nullptr) return 8;   // (one epilogue prefetch ring: dx or y1, not both)
  if ((a.gy != nullptr) != (a.gs != nullptr) || (a.gy2 != nullptr) != (a.gs2 != nullptr)) return 8;
  for (int t = 0; t < g.T; ++t) { a.dy[t] = g.dy[t]; a.dx[t] = g.dx[t]; }
  fb_unit_order(a, fg);
  const unsigned grid = (unsigned)std::min(fg.ntiles, kFusedBwdGrid);
  const size_t lds = fb_lds(fg);
  const bool bwd = a.gy != nullptr || a.gy2 != nullptr, xpro = a.xc != nullptr, bne = a.bn_y != nullptr;
#define FB_(CW_, NJ_, B_, X_, E_, G_, CB_)                                                                  \
  if (fg.cw == CW_ && fg.nj == NJ_ && fg.cb == CB_ && bwd == B_ && xpro == X_ && bne == E_ && (g.Go == 2) == G_) { \
    static bool lds_attr = false;                                                                            \
    if (!lds_attr) {                                                                                         \
      (void)hipFuncSetAttribute(                                                                             \
          reinterpret_cast<const void*>(&conv_bwd_fused_kernel<CW_, NJ_, B_, X_, E_, G_, false, CB_>),       \
          hipFuncAttributeMaxDynamicSharedMemorySize, kFbMaxLds);                                            \
      lds_attr = true;                                                                                       \
    }                                                                                                        \
    hipLaunchKernelGGL((conv_bwd_fused_kernel<CW_, NJ_, B_, X_, E_, G_, false, CB_>), dim3(grid),            \
                       dim3(fb_threads(CW_)), lds, s, a, fg);                                                \
    return 0;                                                                                                \
  }
#define FB4_(CW_, NJ_, B_, G_, CB_) FB_(CW_, NJ_, B_, false, false, G_, CB_) FB_(CW_, NJ_, B_, true, false, G_, CB_) \
                                    FB_(CW_, NJ_, B_, false, true, G_, CB_) FB_(CW_, NJ_, B_, true, true, G_, CB_)
  FB4_(8, 4, false, false, 2) FB4_(8, 4, true, false, 2) FB4_(8, 4, false, true, 2) FB4_(8, 4, true, true, 2)
  FB4_(4, 8, false, false, 2) FB4_(4, 8, true, false, 2) FB4_(4, 4, false, false, 2) FB4_(4, 4, true, false, 2)
  FB4_(4, 8, false, true, 2) FB4_(4, 8, true, true, 2) FB4_(4, 4, false, true, 2) FB4_(4, 4, true, true, 2)
  FB4_(4, 4, false, false, 3) FB4_(4, 4, true, false, 3) FB4_(4, 2, false, false, 3) FB4_(4, 2, true, false, 3)
  // the 34-channel level's Go = 2 pair (two stacked 40-channel dY groups: only 128-pixel tiles fit the LDS)
  FB4_(4, 2, false, true, 3) FB4_(4, 2, true, true, 3)
#undef FB4_
#undef FB_
  return 8;
}

// ---- forward mode ----------------------------------------------------------------------------------------
static int g_fwd_fused = -1;   // env MSP_CONV_FWD_FUSED: 0 off (the halo kernel), default on
static bool fwd_fused_enabled() {
  if (g_fwd_fused < 0) {
    const char* e = getenv("MSP_CONV_FWD_FUSED");
    g_fwd_fused = (e != nullptr && e[0] == '0') ? 0 : 1;
  }
  return g_fwd_fused >= 1;
}

// (tests / A-B: 0 off, 1 on, 2 on for single-output convs only -- the Go = 2 pair back on the halo kernel)
void conv_set_fwd_fused(int on) { g_fwd_fused = on == 2 ? 2 : (on ? 1 : 0); }

bool conv_fwd_fused_ok(const ConvGeom& g) {
  FusedBwdGeom fg;
  return fwd_fused_enabled() && (g.Go == 1 || g_fwd_fused == 1) && fb_plan(g, fg, true);
}

long conv_fwd_fused_blocks(const ConvGeom& g) {
  FusedBwdGeom fg;
  if (!fb_plan(g, fg, true)) return 0;
  return std::min(fg.ntiles, kFusedBwdGrid);
}

int conv_fwd_fused(const ConvArgs& ca, hipStream_t s) {
  const ConvGeom& g = ca.g;
  FusedBwdGeom fg;
  if (!fb_plan(g, fg, true) || g.Gi != 1 || g.Go > 2 || ca.bn_y != nullptr || ca.accum) return 8;
  if (g.Go == 2 && ca.bias != nullptr) return 8;   // (the pair has no bias; bias4 indexes one group)
  FusedBwdArgs a{};
  a.dz = ca.x[0];          // the staged operand (the data-gradient's dY slots)
  a.x = ca.x[0];
  a.xc = ca.xc[0];
  a.xrelu = (ca.xrelu & 1u) ? 1 : 0;
  a.wd = ca.w;             // forward packing [rows][Kp], k = t * Cgi + ci: the data-gradient's [Ci][T * Co]
  a.Kp = g.Kp;
  a.dxo = ca.y[0];
  a.dxo2 = g.Go == 2 ? ca.y[1] : nullptr;
  a.co_split = g.Go == 2 ? g.Cgo : 0;
  a.opitch = g.Cgo;
  a.stat_part = ca.stat_part;   // [blocks][2][Go * Cgo]: the stacked rows
  a.bias = ca.bias;
  a.Co_l = g.Cgo_l;
  a.N = g.N; a.H = g.IH; a.W = g.IW; a.T = g.T; a.Go = 1;
  a.Ci = g.Go * g.Cgo;     // kernel rows = output channels (a pair: both groups, stacked)
  a.Co = g.Cgi;            // staged channels = input channels
  for (int t = 0; t < g.T; ++t) { a.dy[t] = -g.dy[t]; a.dx[t] = -g.dx[t]; }
  fb_unit_order(a, fg);
  const unsigned grid = (unsigned)std::min(fg.ntiles, kFusedBwdGrid);
  const size_t lds = fb_lds(fg);
  const bool xpro = a.xc != nullptr;
#define FF_(CW_, NJ_, X_, CB_)                                                                               \
  if (fg.cw == CW_ && fg.nj == NJ_ && fg.cb == CB_ && xpro == X_) {                                           \
    static bool lds_attr = false;                                                                            \
    if (!lds_attr) {                                                                                         \
      (void)hipFuncSetAttribute(                                                                             \
          reinterpret_cast<const void*>(&conv_bwd_fused_kernel<CW_, NJ_, false, X_, false, false, true, CB_>), \
          hipFuncAttributeMaxDynamicSharedMemorySize, kFbMaxLds);                                            \
      lds_attr = true;                                                                                       \
    }                                                                                                        \
    hipLaunchKernelGGL((conv_bwd_fused_kernel<CW_, NJ_, false, X_, false, false, true, CB_>), dim3(grid),    \
                       dim3(fb_threads(CW_)), lds, s, a, fg);                                                \
    return 0;                                                                                                \
  }
  FF_(8, 4, false, 2) FF_(8, 4, true, 2) FF_(4, 8, false, 2) FF_(4, 8, true, 2) FF_(4, 4, false, 2) FF_(4, 4, true, 2)
  FF_(8, 4, false, 3) FF_(8, 4, true, 3) FF_(4, 4, false, 3) FF_(4, 4, true, 3)
  FF_(4, 4, false, 5) FF_(4, 4, true, 5)
#undef FF_
  return 8;
}
