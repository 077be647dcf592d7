// BatchNorm(+ReLU) for NHWC bf16 feature maps: training statistics, finalize (running stats with
// momentum + unbiased variance, exactly nn.BatchNorm2d / SyncBatchNorm semantics), fused
// normalize+ReLU apply, and the two-pass backward (channel reductions, then the elementwise dx).
//
// Reference ops replaced: every BatchNorm2d / SyncBatchNorm + ReLU pair of the models
// (models/modules.py:83-84, models/ducknet.py:99,120,137; SURVEY §2.5 K8-K10, K11 branch sums).
//
// Reductions are deterministic: each block writes per-channel partials ([nblk][2][Cp] fp32) and a
// second kernel sums them in a fixed order in fp64.  The cross-rank SyncBN exchange happens on the
// tiny [2][Cp] sums between `bn_reduce_partials` and `bn_finalize` (host side, RCCL all_reduce).
#include "common.h"
#include "launchers.h"

namespace {

constexpr int kBlock = 256;
constexpr int kPartUnroll = 4;   // pixels per trip of the backward partial-sum pass

struct SumInputs {
  const uint16_t* p[kMaxSumInputs];
  const float* c[kMaxSumInputs];   // deferred-BN prologue of input i (nullable; rows scale, shift; ld = Cp)
  unsigned relu;
};

// input i's two vectors of this trip, with its BN prologue (bf16-rounded like a materialised z)
DEVI void load_in2(const SumInputs& in, int i, long off0, long off1, bool ok1, int c0, int Cp, float* v0, float* v1) {
  uint4 a0 = *reinterpret_cast<const uint4*>(in.p[i] + off0);
  uint4 a1 = ok1 ? *reinterpret_cast<const uint4*>(in.p[i] + off1) : make_uint4(0, 0, 0, 0);
  if (in.c[i] != nullptr) {
    const bool relu = (in.relu >> i) & 1u;
    a0 = xform8(a0, in.c[i], Cp, c0, relu);
    if (ok1) a1 = xform8(a1, in.c[i], Cp, c0, relu);
  }
  unpack8(a0, v0);
  unpack8(a1, v1);
}

// Thread layout for per-channel reductions over NHWC: cg = tid % CG (8-channel group), r = tid / CG.
__global__ __launch_bounds__(kBlock) void sum_stats_kernel(SumInputs in, int k, uint16_t* __restrict__ out,
                                                           float* __restrict__ part, long P, int Cp) {
  __shared__ float red[2][kBlock][8];
  const int CG = Cp >> 3;
  const int R = kBlock / CG;
  const int tid = threadIdx.x;
  const int cg = tid % CG, r = tid / CG;
  float s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; q[e] = 0.f; }
  if (r < R) {
    // two pixels per trip: every input's vectors for both are issued before the sums (2k loads in flight)
    const long stride = (long)gridDim.x * R;
    for (long p = (long)blockIdx.x * R + r; p < P; p += 2 * stride) {
      const long p1 = p + stride;
      const bool ok1 = p1 < P;
      const long off0 = p * Cp + 8 * cg, off1 = p1 * Cp + 8 * cg;
      float v0[8], v1[8];
      load_in2(in, 0, off0, off1, ok1, 8 * cg, Cp, v0, v1);
      for (int i = 1; i < k; ++i) {
        float u0[8], u1[8];
        load_in2(in, i, off0, off1, ok1, 8 * cg, Cp, u0, u1);
#pragma unroll
        for (int e = 0; e < 8; ++e) { v0[e] += u0[e]; v1[e] += u1[e]; }
      }
      if (out != nullptr) {
        const uint4 pk0 = pack8(v0), pk1 = pack8(v1);
        *reinterpret_cast<uint4*>(out + off0) = pk0;
        if (ok1) *reinterpret_cast<uint4*>(out + off1) = pk1;
        unpack8(pk0, v0);  // statistics of the stored (rounded) tensor
        unpack8(pk1, v1);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {   // the out-of-range slot holds zeros: adds nothing
        s[e] += v0[e] + v1[e];
        q[e] += v0[e] * v0[e] + v1[e] * v1[e];
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
    part[((long)blockIdx.x * 2 + 0) * Cp + c] = ss;
    part[((long)blockIdx.x * 2 + 1) * Cp + c] = qq;
  }
}

// Two-stage deterministic column reduction of [nblk][2][width] partials:
//   stage 1: grid (column chunks of 64, S row splits); 256 threads = 64 columns x 4 row lanes
//   stage 2: one thread per column sums the S split results in order (fp64).
constexpr int kRedCols = 64, kRedRows = 4, kRedSplits = 64;

__global__ __launch_bounds__(256) void reduce_partials_stage1(const float* __restrict__ part, long nblk, int width,
                                                              int col_off, int Cp, double* __restrict__ tmp) {
  __shared__ double red[kRedRows][kRedCols];
  const int ncol = 2 * Cp;
  const int cl = threadIdx.x % kRedCols, rl = threadIdx.x / kRedCols;
  const int col = blockIdx.x * kRedCols + cl;
  const long per = (nblk + gridDim.y - 1) / gridDim.y;
  const long r0 = (long)blockIdx.y * per;
  const long r1 = r0 + per < nblk ? r0 + per : nblk;
  double acc = 0.0;
  if (col < ncol) {
    const int sidx = col / Cp, c = col - sidx * Cp;
    const float* src = part + (long)sidx * width + col_off + c;
#pragma unroll 8
    for (long b = r0 + rl; b < r1; b += kRedRows) acc += (double)src[b * 2 * width];
  }
  red[rl][cl] = acc;
  __syncthreads();
  if (rl == 0 && col < ncol) {
    double s = 0.0;
    for (int r = 0; r < kRedRows; ++r) s += red[r][cl];
    tmp[(long)blockIdx.y * ncol + col] = s;
  }
}

__global__ void reduce_partials_stage2(const double* __restrict__ tmp, int splits, int ncol, double* __restrict__ sums) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= ncol) return;
  double s = 0.0;
#pragma unroll 8
  for (int i = 0; i < splits; ++i) s += tmp[(long)i * ncol + col];
  sums[col] = s;
}

// sum of the S split rows of column i (fixed order -> deterministic)
// Finalize kernels: a block owns kFinCols channels; its kFinParts waves each sum a strided subset of
// the S split rows (independent loads in flight), then the parts are combined in a fixed order
// (deterministic).  Returns (sum, second-column sum) for channel c in lanes of part 0.
constexpr int kFinCols = 64, kFinParts = 4;

DEVI void split_sum2(const double* __restrict__ tmp, int S, int Cp, int c, bool valid, double& a, double& b) {
  __shared__ double red[2][kFinParts][kFinCols];
  const int cl = threadIdx.x % kFinCols, pt = threadIdx.x / kFinCols;
  double sa = 0.0, sb = 0.0;
  if (valid) {
#pragma unroll 4
    for (int k = pt; k < S; k += kFinParts) {
      sa += tmp[(long)k * 2 * Cp + c];
      sb += tmp[(long)k * 2 * Cp + Cp + c];
    }
  }
  red[0][pt][cl] = sa; red[1][pt][cl] = sb;
  __syncthreads();
  a = 0.0; b = 0.0;
#pragma unroll
  for (int i = 0; i < kFinParts; ++i) { a += red[0][i][cl]; b += red[1][i][cl]; }
}

struct FinFwd {   // forward finalize operands
  float count, momentum, eps;
  const float* gamma; const float* beta;
  float* rmean; float* rvar;
  float* scale; float* shift; float* mean; float* invstd;
};
struct FinBwd {   // backward finalize operands
  float count, pscale;
  const float* scale; const float* invstd; const float* mean;
  float* dgamma; float* dbeta; float* coef;
};

// nn.BatchNorm2d training semantics: biased variance normalises, the running variance takes the
// unbiased one, padded channels (C <= c < Cp) get zero scale/shift.
DEVI void fin_fwd_channel(int c, int C, int Cp, bool training, double sm, double sq, const FinFwd& f) {
  if (c >= Cp) return;
  if (c >= C) { f.scale[c] = 0.f; f.shift[c] = 0.f; f.mean[c] = 0.f; f.invstd[c] = 0.f; return; }
  float mean, var;
  if (training) {
    const double m = sm / f.count;
    double v = sq / f.count - m * m;
    if (v < 0) v = 0;
    mean = (float)m; var = (float)v;
    if (f.rmean != nullptr) {
      const float unbiased = f.count > 1.f ? (float)(v * f.count / (f.count - 1.f)) : (float)v;
      f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * mean;
      f.rvar[c] = (1.f - f.momentum) * f.rvar[c] + f.momentum * unbiased;
    }
  } else {
    mean = f.rmean[c]; var = f.rvar[c];
  }
  const float inv = rsqrtf(var + f.eps);
  const float gm = f.gamma != nullptr ? f.gamma[c] : 1.f;
  const float bt = f.beta != nullptr ? f.beta[c] : 0.f;
  f.scale[c] = gm * inv;
  f.shift[c] = bt - mean * gm * inv;
  f.mean[c] = mean;
  f.invstd[c] = inv;
}

// dx = k1*dzr + k2*y + k3.  SyncBN: the sums are global; dgamma/dbeta take pscale = 1/world of them so
// that the DDP-style average over ranks (sum all-reduce * 1/world) yields the mean of the per-rank
// local gradients.
DEVI void fin_bwd_channel(int c, int C, int Cp, double sdd, double sdxd, const FinBwd& f) {
  if (c >= Cp) return;
  if (c >= C) { f.coef[c] = 0.f; f.coef[Cp + c] = 0.f; f.coef[2 * Cp + c] = 0.f; return; }
  const float sd = (float)sdd, sdx = (float)sdxd;
  if (f.dgamma != nullptr) f.dgamma[c] += f.pscale * sdx * f.invstd[c];
  if (f.dbeta != nullptr) f.dbeta[c] += f.pscale * sd;
  const float k1 = f.scale[c];
  const float k2 = -k1 * f.invstd[c] * f.invstd[c] * sdx / f.count;
  const float k3 = -k1 * sd / f.count - k2 * f.mean[c];
  f.coef[c] = k1; f.coef[Cp + c] = k2; f.coef[2 * Cp + c] = k3;
}

__global__ __launch_bounds__(kFinCols * kFinParts) void bn_finalize_kernel(const double* __restrict__ tmp, int S,
                                                                            int C, int Cp, int training, FinFwd f) {
  const int c = blockIdx.x * kFinCols + (int)(threadIdx.x % kFinCols);
  double sm = 0.0, sq = 0.0;
  if (training) split_sum2(tmp, S, Cp, c, c < C, sm, sq);
  if (threadIdx.x >= kFinCols) return;
  fin_fwd_channel(c, C, Cp, training != 0, sm, sq, f);
}

// Elementwise BN passes: each thread owns ONE 8-channel group (cg = tid % CG) for all its pixels, so
// its per-channel coefficients are loaded once into registers (a per-vector reload costs 4-10x the
// 16 B of activation it serves); rows r = tid / CG of a block walk consecutive pixels (the wave's
// accesses stay contiguous), and an unroll of kUnroll pixels keeps that many loads in flight.
constexpr int kUnroll = 4;

__global__ __launch_bounds__(kBlock) void bn_act_apply_kernel(const uint16_t* __restrict__ y,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              uint16_t* __restrict__ z, long P, int CG,
                                                              int relu) {
  const int R = kBlock / CG, tid = threadIdx.x, cg = tid % CG, r = tid / CG;
  if (r >= R) return;
  float a[8], b[8];
  load8f(scale + 8 * cg, a);
  load8f(shift + 8 * cg, b);
  const long stride = (long)gridDim.x * R;
  const long Cp = 8L * CG;
  long p = (long)blockIdx.x * R + r;
  for (; p < P; p += kUnroll * stride) {
    uint4 in[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const long q = p + u * stride;
      in[u] = q < P ? *reinterpret_cast<const uint4*>(y + q * Cp + 8 * cg) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const long q = p + u * stride;
      if (q >= P) break;
      float v[8];
      unpack8(in[u], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float o = fmaf(v[e], a[e], b[e]);
        // relu 2: ReLU6 (MobileNetV2), clamped before the one bf16 rounding -- bitwise the rounded BN
        // output clamped by a separate relu6 pass (6 is exact in bf16; rounding is monotone)
        v[e] = relu == 2 ? fminf(fmaxf(o, 0.f), 6.f) : (relu ? fmaxf(o, 0.f) : o);
      }
      *reinterpret_cast<uint4*>(z + q * Cp + 8 * cg) = pack8(v);
    }
  }
}

// ResNet block tail in one pass: z = relu(o + r) with o = act_a(sa*y + ba) (the last BN of the block,
// deferred) and r = act_b(sb*x + bb) (the downsample branch's BN, deferred) or the plain identity x
// (sb == nullptr).  o and r are rounded to bf16 before the add, as their materialised tensors were:
// bitwise the bn_act_apply (x2) + add_act chain, minus its intermediate tensors.
__global__ __launch_bounds__(kBlock) void bn_add_act_kernel(const uint16_t* __restrict__ y,
                                                            const float* __restrict__ sa,
                                                            const float* __restrict__ ba, int relu_a,
                                                            const uint16_t* __restrict__ x,
                                                            const float* __restrict__ sb,
                                                            const float* __restrict__ bb, int relu_b,
                                                            uint16_t* __restrict__ z, long P, int CG, int relu) {
  const int R = kBlock / CG, tid = threadIdx.x, cg = tid % CG, r = tid / CG;
  if (r >= R) return;
  float a[8], b[8], c[8], d[8];
  load8f(sa + 8 * cg, a);
  load8f(ba + 8 * cg, b);
  const bool defb = sb != nullptr;
  if (defb) {
    load8f(sb + 8 * cg, c);
    load8f(bb + 8 * cg, d);
  }
  const float fa = relu_a ? 0.f : -INFINITY, fb = (defb && relu_b) ? 0.f : -INFINITY;
  const long stride = (long)gridDim.x * R;
  const long Cp = 8L * CG;
  long p = (long)blockIdx.x * R + r;
  for (; p < P; p += kUnroll * stride) {
    uint4 in[kUnroll], iv[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const long q = p + u * stride;
      in[u] = q < P ? *reinterpret_cast<const uint4*>(y + q * Cp + 8 * cg) : make_uint4(0, 0, 0, 0);
      iv[u] = q < P ? *reinterpret_cast<const uint4*>(x + q * Cp + 8 * cg) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const long q = p + u * stride;
      if (q >= P) break;
      float v[8], w[8];
      unpack8(in[u], v);
      unpack8(iv[u], w);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float o = bf2f(f2bf(fmaxf(fmaf(v[e], a[e], b[e]), fa)));
        const float rr = defb ? bf2f(f2bf(fmaxf(fmaf(w[e], c[e], d[e]), fb))) : w[e];
        const float t = o + rr;
        v[e] = relu ? fmaxf(t, 0.f) : t;
      }
      *reinterpret_cast<uint4*>(z + q * Cp + 8 * cg) = pack8(v);
    }
  }
}

__global__ __launch_bounds__(kBlock) void bn_act_bwd_partial_kernel(
    const uint16_t* __restrict__ dz, const uint16_t* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ mean, float* __restrict__ part, long P,
    int Cp, int relu) {
  __shared__ float red[2][kBlock][8];
  const int CG = Cp >> 3;
  const int R = kBlock / CG;
  const int tid = threadIdx.x;
  const int cg = tid % CG, r = tid / CG;
  float s[8], q[8], a[8], b[8], mu[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; q[e] = 0.f; }
  load8f(scale + 8 * cg, a);
  load8f(shift + 8 * cg, b);
  load8f(mean + 8 * cg, mu);
  if (r < R) {
    // kPartUnroll pixels' (dz, y) vectors issued before any is consumed: 2*kPartUnroll 16-B loads in
    // flight per thread (one pair per trip left the pass latency-bound at ~1 block per CU).
    const long stride = (long)gridDim.x * R;
    for (long p = (long)blockIdx.x * R + r; p < P; p += kPartUnroll * stride) {
      uint4 gin[kPartUnroll], yin[kPartUnroll];
#pragma unroll
      for (int u = 0; u < kPartUnroll; ++u) {
        const long q = p + u * stride;
        const bool ok = q < P;
        gin[u] = ok ? *reinterpret_cast<const uint4*>(dz + q * Cp + 8 * cg) : make_uint4(0, 0, 0, 0);
        yin[u] = ok ? *reinterpret_cast<const uint4*>(y + q * Cp + 8 * cg) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kPartUnroll; ++u) {
        float g[8], v[8];
        unpack8(gin[u], g);   // out-of-range slots are zero: gr = 0 adds nothing
        unpack8(yin[u], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gr = (!relu || fmaf(v[e], a[e], b[e]) > 0.f) ? g[e] : 0.f;
          s[e] += gr;
          q[e] += gr * (v[e] - mu[e]);
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
    part[((long)blockIdx.x * 2 + 0) * Cp + c] = ss;
    part[((long)blockIdx.x * 2 + 1) * Cp + c] = qq;
  }
}

// coef[3][Cp]: dy = k1*dzr + k2*y + k3  (k1 = gamma*invstd, k2 = -k1*invstd*sum(dzr*xmu)/M,
// k3 = -k1*sum(dzr)/M - k2*mean).  dgamma/dbeta are ACCUMULATED into the fp32 parameter grads.
__global__ __launch_bounds__(kFinCols * kFinParts) void bn_bwd_finalize_kernel(const double* __restrict__ tmp, int S,
                                                                                int C, int Cp, FinBwd f) {
  const int c = blockIdx.x * kFinCols + (int)(threadIdx.x % kFinCols);
  double a, b;
  split_sum2(tmp, S, Cp, c, c < C, a, b);
  if (threadIdx.x >= kFinCols) return;
  fin_bwd_channel(c, C, Cp, a, b, f);
}

// Fused column reduction + finalize (single-rank BN): grid (Cp/32 channel chunks, S row splits),
// 256 threads = 64 columns (32 channels x {sum, sum^2}) x 4 row lanes.  Every block publishes its
// fp64 column sums with agent-scope stores, drains, and bumps its chunk's arrival counter; the LAST
// arriving block of a chunk acquires, sums the S split rows in fixed order (deterministic) and
// finalizes those channels, then re-arms the counter for the next BN (kernels on a stream run in
// order, so one counter array serves every call).  Replaces stage-1 + finalize launches.
constexpr int kRfCh = 32;

template <bool BWD>
__global__ __launch_bounds__(256) void bn_reduce_finalize_kernel(const float* __restrict__ part, long nblk, int width,
                                                                 int col_off, int C, int Cp, double* __restrict__ tmp,
                                                                 unsigned* __restrict__ cnt, FinFwd ff, FinBwd fb) {
  __shared__ double red[4][64];
  __shared__ int s_last;
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int which = cl >> 5, ch = blockIdx.x * kRfCh + (cl & 31);
  const long per = (nblk + gridDim.y - 1) / gridDim.y;
  const long r0 = (long)blockIdx.y * per;
  const long r1 = r0 + per < nblk ? r0 + per : nblk;
  double acc = 0.0;
  if (ch < Cp) {
    const float* src = part + (long)which * width + col_off + ch;
#pragma unroll 8
    for (long b = r0 + rl; b < r1; b += 4) acc += (double)src[b * 2 * width];
  }
  red[rl][cl] = acc;
  __syncthreads();
  if (rl == 0 && ch < Cp) {
    const double s = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    __hip_atomic_store(&tmp[(long)blockIdx.y * 2 * Cp + which * Cp + ch], s, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains before the arrival
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(&cnt[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             gridDim.y - 1;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // last block of this chunk: 64 columns x 4 lanes sum the S rows (lane-strided, fixed order)
  const int S = gridDim.y;
  double t = 0.0;
  if (ch < Cp)
#pragma unroll 8
    for (int k = rl; k < S; k += 4) t += tmp[(long)k * 2 * Cp + which * Cp + ch];
  __syncthreads();
  red[rl][cl] = t;
  __syncthreads();
  if (threadIdx.x < 32) {
    const int c = blockIdx.x * kRfCh + threadIdx.x;
    const double a = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    const double b = red[0][32 + threadIdx.x] + red[1][32 + threadIdx.x] + red[2][32 + threadIdx.x] +
                     red[3][32 + threadIdx.x];
    if (BWD) fin_bwd_channel(c, C, Cp, a, b, fb);
    else fin_fwd_channel(c, C, Cp, true, a, b, ff);
  }
  if (threadIdx.x == 0) __hip_atomic_store(&cnt[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The apply pass of a BN whose input y is a SUM with a second (deferred) BN's output among its summands -- the
// ResidualBlock's bn(upper + relu(bn2(y2))) -- also emits bn2's backward partials: dy (this pass's stored, bf16
// output) IS bn2's incoming gradient, so (sum g2, sum g2 * (y2 - mean2)), g2 = dy * relu2'(y2), come from one more
// read of y2 instead of bn2's own partial pass over (dy, y2).  Grid and partial rows as bn_act_bwd_partial.
__global__ __launch_bounds__(kBlock) void bn_act_bwd_apply_part_kernel(
    const uint16_t* __restrict__ dz, const uint16_t* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ coef, uint16_t* __restrict__ dy,
    const uint16_t* __restrict__ y2, const float* __restrict__ scale2, const float* __restrict__ shift2,
    const float* __restrict__ mean2, int relu2, float* __restrict__ part, long P, int Cp, int relu) {
  __shared__ float red[2][kBlock][8];
  const int CG = Cp >> 3;
  const int R = kBlock / CG;
  const int tid = threadIdx.x;
  const int cg = tid % CG, r = tid / CG, c0 = 8 * cg;
  float s[8], q[8], a[8], b[8], k1[8], k2[8], k3[8], a2[8], b2[8], mu[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; q[e] = 0.f; }
  load8f(scale + c0, a); load8f(shift + c0, b);
  load8f(coef + c0, k1); load8f(coef + Cp + c0, k2); load8f(coef + 2 * Cp + c0, k3);
  load8f(scale2 + c0, a2); load8f(shift2 + c0, b2); load8f(mean2 + c0, mu);
  if (!relu)
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = INFINITY;
  if (r < R) {
    const long stride = (long)gridDim.x * R;
    for (long p = (long)blockIdx.x * R + r; p < P; p += kPartUnroll * stride) {
      uint4 gin[kPartUnroll], yin[kPartUnroll], zin[kPartUnroll];
#pragma unroll
      for (int u = 0; u < kPartUnroll; ++u) {
        const long qq = p + u * stride;
        const bool ok = qq < P;
        gin[u] = ok ? *reinterpret_cast<const uint4*>(dz + qq * Cp + c0) : make_uint4(0, 0, 0, 0);
        yin[u] = ok ? *reinterpret_cast<const uint4*>(y + qq * Cp + c0) : make_uint4(0, 0, 0, 0);
        zin[u] = ok ? *reinterpret_cast<const uint4*>(y2 + qq * Cp + c0) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kPartUnroll; ++u) {
        const long qq = p + u * stride;
        if (qq >= P) break;
        float g[8], v[8], w[8];
        unpack8(gin[u], g);
        unpack8(yin[u], v);
        unpack8(zin[u], w);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = bwd1(g[e], v[e], a[e], b[e], k1[e], k2[e], k3[e]);
        const uint4 o = pack8(g);
        *reinterpret_cast<uint4*>(dy + qq * Cp + c0) = o;
        unpack8(o, g);   // bn2 sees the stored (bf16) gradient, as its own partial pass would
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gr = (!relu2 || fmaf(w[e], a2[e], b2[e]) > 0.f) ? g[e] : 0.f;
          s[e] += gr;
          q[e] += gr * (w[e] - mu[e]);
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
    part[((long)blockIdx.x * 2 + 0) * Cp + c] = ss;
    part[((long)blockIdx.x * 2 + 1) * Cp + c] = qq;
  }
}

__global__ __launch_bounds__(kBlock) void bn_act_bwd_apply_kernel(
    const uint16_t* __restrict__ dz, const uint16_t* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ coef, uint16_t* __restrict__ dy, long P,
    int CG, int relu) {
  const int R = kBlock / CG, tid = threadIdx.x, cg = tid % CG, r = tid / CG;
  if (r >= R) return;
  const int Cp = CG * 8, c0 = 8 * cg;
  float a[8], b[8], k1[8], k2[8], k3[8];
  load8f(scale + c0, a); load8f(shift + c0, b);
  load8f(coef + c0, k1); load8f(coef + Cp + c0, k2); load8f(coef + 2 * Cp + c0, k3);
  if (!relu)   // bwd1's ReLU test passes everywhere
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = INFINITY;
  const long stride = (long)gridDim.x * R;
  long p = (long)blockIdx.x * R + r;
  for (; p < P; p += kUnroll * stride) {
    uint4 gin[kUnroll], yin[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const long q = p + u * stride;
      const bool ok = q < P;
      gin[u] = ok ? *reinterpret_cast<const uint4*>(dz + q * Cp + c0) : make_uint4(0, 0, 0, 0);
      yin[u] = ok ? *reinterpret_cast<const uint4*>(y + q * Cp + c0) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const long q = p + u * stride;
      if (q >= P) break;
      float g[8], v[8];
      unpack8(gin[u], g);
      unpack8(yin[u], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = bwd1(g[e], v[e], a[e], b[e], k1[e], k2[e], k3[e]);
      *reinterpret_cast<uint4*>(dy + q * Cp + c0) = pack8(g);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// DUCK tail backward (reference ducknet.py:151-154: out_bn(act(sum of the six branch-last BNs))):
// the backward of out_bn and of the k branch-last BNs it sums, in two passes instead of 1 + 2k.
//   dys = out_bn's data-gradient (its apply: relu'(ys) * (k1 dz + k2 ys + k3)) is never written: both
//   passes recompute it from (dz, ys) in registers -- it IS every branch BN's dz;
//   pass 1 (tail_partial): per branch i the (sum dzr_i, sum dzr_i * (y_i - mean_i)) channel partials;
//   pass 2 (tail_apply):   dy_i = k1_i dzr_i + k2_i y_i + k3_i for every branch.
// Traffic per tail: 8 + 14 tensor passes (dz, ys, k inputs; + k outputs) instead of out_bn's apply (3)
// plus k separate partial (2 each) and apply (3 each) passes that each re-read dys.
// The branch coefficients (scale, shift, mean | k1, k2, k3 per channel) sit in LDS; out_bn's in
// registers (thread-owned 8-channel group, as in the single-BN passes).
struct TailArgs {
  const uint16_t* dz;          // out_bn output gradient
  const uint16_t* ys;          // out_bn input (the branch sum)
  const float* oscale; const float* oshift; const float* ocoef;   // out_bn stats rows 0/1, coef [3][Cp]
  int orelu, k;
  const uint16_t* y[kTailMax];            // branch-last BN inputs
  const float* st[kTailMax];              // their stats [4][Cp] (scale, shift, mean, invstd)
  const float* coef[kTailMax];            // their backward coef [3][Cp] (apply pass)
  unsigned relu;                          // bit i: branch i has a ReLU
  uint16_t* dy[kTailMax];                 // branch data-gradients (apply pass; nullptr: deferred to the producer)
  uint16_t* g;                            // nullable: out_bn's data-gradient (bf16), for the deferred branches
};

// 8 consecutive floats from LDS as two 16-B reads (the caller guarantees 32-B alignment)
DEVI void lds8(const float* p, float* d) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

// dzr of out_bn for one 8-channel vector: relu'(ys) * (k1 dz + k2 ys + k3) -- the branch BNs' dz
DEVI void tail_dys(const uint4& gz, const uint4& yv, const float* a, const float* b, const float* k1,
                   const float* k2, const float* k3, bool relu, float* d) {
  float g[8], v[8];
  unpack8(gz, g);
  unpack8(yv, v);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float gr = (!relu || fmaf(v[e], a[e], b[e]) > 0.f) ? g[e] : 0.f;
    d[e] = bf2f(f2bf(k1[e] * gr + k2[e] * v[e] + k3[e]));   // rounded like the materialised dys
  }
}

// KM: compile-time branch capacity (the 2 x KM x 8 accumulators dominate the register budget; the host
// runs six branches as two KM = 3 launches, which re-read dz and ys once but double the occupancy)
template <int KM>
__global__ __launch_bounds__(kBlock) void bn_tail_partial_kernel(TailArgs t, float* __restrict__ part, long P, int Cp) {
  extern __shared__ float tsm[];          // [k][3][Cp] branch scale, shift, mean; then red[2][kBlock][8]
  float* red = tsm + t.k * 3 * Cp;
  const int CG = Cp >> 3, R = kBlock / CG, tid = threadIdx.x, cg = tid % CG, r = tid / CG, c0 = 8 * cg;
  for (int i = tid; i < t.k * 3 * Cp; i += kBlock) {
    const int b = i / (3 * Cp), rem = i - b * 3 * Cp;
    tsm[i] = t.st[b][rem];                // rows 0..2 of the branch's stats = scale, shift, mean
  }
  float a[8], sh[8], k1[8], k2[8], k3[8];
  load8f(t.oscale + c0, a); load8f(t.oshift + c0, sh);
  load8f(t.ocoef + c0, k1); load8f(t.ocoef + Cp + c0, k2); load8f(t.ocoef + 2 * Cp + c0, k3);
  float s[KM][8], q[KM][8];
#pragma unroll
  for (int i = 0; i < KM; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) { s[i][e] = 0.f; q[i][e] = 0.f; }
  __syncthreads();
  if (r < R) {
    const long stride = (long)gridDim.x * R;
    for (long p = (long)blockIdx.x * R + r; p < P; p += stride) {
      const long off = p * Cp + c0;
      const uint4 gz = *reinterpret_cast<const uint4*>(t.dz + off);
      const uint4 yv = *reinterpret_cast<const uint4*>(t.ys + off);
      uint4 yi[KM];
#pragma unroll
      for (int i = 0; i < KM; ++i)
        yi[i] = i < t.k ? *reinterpret_cast<const uint4*>(t.y[i] + off) : make_uint4(0, 0, 0, 0);
      float d[8];
      tail_dys(gz, yv, a, sh, k1, k2, k3, t.orelu != 0, d);
#pragma unroll
      for (int i = 0; i < KM; ++i) {
        if (i >= t.k) break;
        float sc[8], shf[8], mu[8], v[8];
        lds8(tsm + i * 3 * Cp + c0, sc);           // 16-B LDS reads (rows are 32-B aligned: Cp % 8 == 0)
        lds8(tsm + i * 3 * Cp + Cp + c0, shf);
        lds8(tsm + i * 3 * Cp + 2 * Cp + c0, mu);
        unpack8(yi[i], v);
        const bool rl = (t.relu >> i) & 1u;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gr = (!rl || fmaf(v[e], sc[e], shf[e]) > 0.f) ? d[e] : 0.f;
          s[i][e] += gr;
          q[i][e] += gr * (v[e] - mu[e]);
        }
      }
    }
  }
  // per branch: block column reduction -> part[i][blk][2][Cp] (fixed order: deterministic)
  const long nblk = gridDim.x;
#pragma unroll
  for (int i = 0; i < KM; ++i) {
    if (i >= t.k) break;
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[(0 * kBlock + tid) * 8 + e] = s[i][e]; red[(1 * kBlock + tid) * 8 + e] = q[i][e]; }
    __syncthreads();
    for (int c = tid; c < Cp; c += kBlock) {
      const int g = c >> 3, e = c & 7;
      float ss = 0.f, qq = 0.f;
      for (int rr = 0; rr < R; ++rr) { ss += red[(rr * CG + g) * 8 + e]; qq += red[(kBlock + rr * CG + g) * 8 + e]; }
      part[(((long)i * nblk + blockIdx.x) * 2 + 0) * Cp + c] = ss;
      part[(((long)i * nblk + blockIdx.x) * 2 + 1) * Cp + c] = qq;
    }
    __syncthreads();
  }
}

template <int KM>
__global__ __launch_bounds__(kBlock) void bn_tail_apply_kernel(TailArgs t, long P, int Cp) {
  extern __shared__ float tsm[];          // [k][5][Cp] branch scale, shift, k1, k2, k3
  const int CG = Cp >> 3, R = kBlock / CG, tid = threadIdx.x, cg = tid % CG, r = tid / CG, c0 = 8 * cg;
  for (int i = tid; i < t.k * 5 * Cp; i += kBlock) {
    const int b = i / (5 * Cp), rem = i - b * 5 * Cp;
    tsm[i] = rem < 2 * Cp ? t.st[b][rem] : t.coef[b][rem - 2 * Cp];
  }
  float a[8], sh[8], k1[8], k2[8], k3[8];
  load8f(t.oscale + c0, a); load8f(t.oshift + c0, sh);
  load8f(t.ocoef + c0, k1); load8f(t.ocoef + Cp + c0, k2); load8f(t.ocoef + 2 * Cp + c0, k3);
  __syncthreads();
  if (r >= R) return;
  // two pixels per trip: each branch's 5 coefficient rows are read from LDS once for both
  const long stride = (long)gridDim.x * R;
  for (long p = (long)blockIdx.x * R + r; p < P; p += 2 * stride) {
    const long p1 = p + stride;
    const bool ok1 = p1 < P;
    const long off0 = p * Cp + c0, off1 = p1 * Cp + c0;
    float d0[8], d1[8];
    tail_dys(*reinterpret_cast<const uint4*>(t.dz + off0), *reinterpret_cast<const uint4*>(t.ys + off0), a, sh, k1, k2,
             k3, t.orelu != 0, d0);
    tail_dys(ok1 ? *reinterpret_cast<const uint4*>(t.dz + off1) : make_uint4(0, 0, 0, 0),
             ok1 ? *reinterpret_cast<const uint4*>(t.ys + off1) : make_uint4(0, 0, 0, 0), a, sh, k1, k2, k3,
             t.orelu != 0, d1);
    if (t.g != nullptr) {   // (uniform) the deferred branches' dz: their producers rebuild dy from (g, y_i)
      *reinterpret_cast<uint4*>(t.g + off0) = pack8(d0);
      if (ok1) *reinterpret_cast<uint4*>(t.g + off1) = pack8(d1);
    }
#pragma unroll
    for (int i = 0; i < KM; ++i) {
      if (i >= t.k) break;
      if (t.dy[i] == nullptr) continue;   // (uniform) deferred branch
      const uint4 y0 = *reinterpret_cast<const uint4*>(t.y[i] + off0);
      const uint4 y1 = ok1 ? *reinterpret_cast<const uint4*>(t.y[i] + off1) : make_uint4(0, 0, 0, 0);
      const float* cf = tsm + i * 5 * Cp + c0;
      float sc[8], shf[8], c1[8], c2[8], c3[8], v0[8], v1[8], o0[8], o1[8];
      lds8(cf, sc); lds8(cf + Cp, shf); lds8(cf + 2 * Cp, c1); lds8(cf + 3 * Cp, c2); lds8(cf + 4 * Cp, c3);
      unpack8(y0, v0);
      unpack8(y1, v1);
      const bool rl = (t.relu >> i) & 1u;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g0 = (!rl || fmaf(v0[e], sc[e], shf[e]) > 0.f) ? d0[e] : 0.f;
        const float g1 = (!rl || fmaf(v1[e], sc[e], shf[e]) > 0.f) ? d1[e] : 0.f;
        o0[e] = c1[e] * g0 + c2[e] * v0[e] + c3[e];
        o1[e] = c1[e] * g1 + c2[e] * v1[e] + c3[e];
      }
      *reinterpret_cast<uint4*>(t.dy[i] + off0) = pack8(o0);
      if (ok1) *reinterpret_cast<uint4*>(t.dy[i] + off1) = pack8(o1);
    }
  }
}

// Grid of the channel-owning elementwise passes: ~kUnroll pixels per thread per loop trip, <= 8192 blocks.
int grid_rows(long P, int CG) {
  const long R = kBlock / CG;
  long b = (P + R * kUnroll - 1) / (R * kUnroll);
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

long bn_partial_blocks(long P, int Cp) {
  const int CG = Cp / 8;
  const int R = kBlock / CG;
  long b = (P + (long)R * 16 - 1) / ((long)R * 16);
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return b;
}

void sum_stats(const uint16_t* const* inputs, const float* const* coefs, unsigned relu_mask, int k, uint16_t* out,
               float* part, long P, int Cp, hipStream_t s) {
  SumInputs in{};
  for (int i = 0; i < k; ++i) {
    in.p[i] = inputs[i];
    in.c[i] = coefs != nullptr ? coefs[i] : nullptr;
  }
  in.relu = relu_mask;
  hipLaunchKernelGGL(sum_stats_kernel, dim3(bn_partial_blocks(P, Cp)), dim3(kBlock), 0, s, in, k, out, part, P, Cp);
}

int bn_reduce_splits(long nblk) {
  long sp = nblk / 32;
  if (sp > kRedSplits) sp = kRedSplits;
  if (sp < 1) sp = 1;
  return (int)sp;
}

void bn_reduce_partials(const float* part, long nblk, int width, int col_off, int Cp, double* tmp, hipStream_t s) {
  const int splits = bn_reduce_splits(nblk);
  hipLaunchKernelGGL(reduce_partials_stage1, dim3(cdiv(2 * Cp, kRedCols), splits), dim3(256), 0, s, part, nblk, width,
                     col_off, Cp, tmp);
}

void bn_collapse(const double* tmp, int S, int Cp, double* out, hipStream_t s) {
  hipLaunchKernelGGL(reduce_partials_stage2, dim3(cdiv(2 * Cp, 256)), dim3(256), 0, s, tmp, S, 2 * Cp, out);
}

void bn_finalize(const double* tmp, int S, int C, int Cp, float count, const float* gamma, const float* beta,
                 float* running_mean, float* running_var, float momentum, float eps, int training,
                 float* scale, float* shift, float* mean, float* invstd, hipStream_t s) {
  const FinFwd f{count, momentum, eps, gamma, beta, running_mean, running_var, scale, shift, mean, invstd};
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(Cp, kFinCols)), dim3(kFinCols * kFinParts), 0, s, tmp, S, C, Cp,
                     training, f);
}

int bn_rf_chunks(int Cp) { return cdiv(Cp, kRfCh); }

void bn_reduce_finalize(const float* part, long nblk, int width, int col_off, int C, int Cp, double* tmp,
                        unsigned* cnt, float count, const float* gamma, const float* beta, float* running_mean,
                        float* running_var, float momentum, float eps, float* scale, float* shift, float* mean,
                        float* invstd, hipStream_t s) {
  const FinFwd f{count, momentum, eps, gamma, beta, running_mean, running_var, scale, shift, mean, invstd};
  const FinBwd b{};
  hipLaunchKernelGGL((bn_reduce_finalize_kernel<false>), dim3(cdiv(Cp, kRfCh), bn_reduce_splits(nblk)), dim3(256), 0, s,
                     part, nblk, width, col_off, C, Cp, tmp, cnt, f, b);
}

void bn_reduce_bwd_finalize(const float* part, long nblk, int C, int Cp, double* tmp, unsigned* cnt, float count,
                            const float* scale, const float* invstd, const float* mean, float* dgamma, float* dbeta,
                            float* coef, float pscale, hipStream_t s) {
  const FinFwd f{};
  const FinBwd b{count, pscale, scale, invstd, mean, dgamma, dbeta, coef};
  hipLaunchKernelGGL((bn_reduce_finalize_kernel<true>), dim3(cdiv(Cp, kRfCh), bn_reduce_splits(nblk)), dim3(256), 0, s,
                     part, nblk, Cp, 0, C, Cp, tmp, cnt, f, b);
}

void bn_act_apply(const uint16_t* y, const float* scale, const float* shift, uint16_t* z, long P, int Cp,
                  int relu, hipStream_t s) {
  hipLaunchKernelGGL(bn_act_apply_kernel, dim3(grid_rows(P, Cp / 8)), dim3(kBlock), 0, s, y, scale, shift, z, P,
                     Cp / 8, relu);
}

void bn_add_act(const uint16_t* y, const float* sa, const float* ba, int relu_a, const uint16_t* x, const float* sb,
                const float* bb, int relu_b, uint16_t* z, long P, int Cp, int relu, hipStream_t s) {
  hipLaunchKernelGGL(bn_add_act_kernel, dim3(grid_rows(P, Cp / 8)), dim3(kBlock), 0, s, y, sa, ba, relu_a, x, sb, bb,
                     relu_b, z, P, Cp / 8, relu);
}

void bn_act_bwd_partial(const uint16_t* dz, const uint16_t* y, const float* scale, const float* shift,
                        const float* mean, float* part, long P, int Cp, int relu, hipStream_t s) {
  hipLaunchKernelGGL(bn_act_bwd_partial_kernel, dim3(bn_partial_blocks(P, Cp)), dim3(kBlock), 0, s, dz, y, scale,
                     shift, mean, part, P, Cp, relu);
}

void bn_bwd_finalize(const double* tmp, int S, int C, int Cp, float count, const float* scale, const float* invstd,
                     const float* mean, float* dgamma, float* dbeta, float* coef, float pscale, hipStream_t s) {
  const FinBwd f{count, pscale, scale, invstd, mean, dgamma, dbeta, coef};
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(cdiv(Cp, kFinCols)), dim3(kFinCols * kFinParts), 0, s, tmp, S, C, Cp,
                     f);
}

long bn_tail_blocks(long P, int Cp) { return bn_partial_blocks(P, Cp); }

static TailArgs tail_args(const uint16_t* dz, const uint16_t* ys, const float* ostats, const float* ocoef, int orelu,
                          int k, const uint16_t* const* y, const float* const* st, const float* const* coef,
                          unsigned relu, uint16_t* const* dy, int Cp) {
  TailArgs t{};
  t.dz = dz; t.ys = ys; t.oscale = ostats; t.oshift = ostats + Cp; t.ocoef = ocoef; t.orelu = orelu; t.k = k;
  for (int i = 0; i < k; ++i) {
    t.y[i] = y[i]; t.st[i] = st[i];
    t.coef[i] = coef != nullptr ? coef[i] : nullptr;
    t.dy[i] = dy != nullptr ? dy[i] : nullptr;
  }
  t.relu = relu;
  return t;
}

void bn_tail_partial(const uint16_t* dz, const uint16_t* ys, const float* ostats, const float* ocoef, int orelu, int k,
                     const uint16_t* const* y, const float* const* st, unsigned relu, float* part, long P, int Cp,
                     hipStream_t s) {
  const TailArgs t = tail_args(dz, ys, ostats, ocoef, orelu, k, y, st, nullptr, relu, nullptr, Cp);
  const size_t lds = ((size_t)k * 3 * Cp + 2 * kBlock * 8) * sizeof(float);
  if (k <= 3)
    hipLaunchKernelGGL(bn_tail_partial_kernel<3>, dim3(bn_tail_blocks(P, Cp)), dim3(kBlock), lds, s, t, part, P, Cp);
  else
    hipLaunchKernelGGL(bn_tail_partial_kernel<kTailMax>, dim3(bn_tail_blocks(P, Cp)), dim3(kBlock), lds, s, t, part, P,
                       Cp);
}

void bn_tail_apply(const uint16_t* dz, const uint16_t* ys, const float* ostats, const float* ocoef, int orelu, int k,
                   const uint16_t* const* y, const float* const* st, const float* const* coef, unsigned relu,
                   uint16_t* const* dy, long P, int Cp, hipStream_t s, uint16_t* g) {
  TailArgs t = tail_args(dz, ys, ostats, ocoef, orelu, k, y, st, coef, relu, dy, Cp);
  t.g = g;
  const size_t lds = (size_t)k * 5 * Cp * sizeof(float);
  if (k <= 3)
    hipLaunchKernelGGL(bn_tail_apply_kernel<3>, dim3(grid_rows(P, Cp / 8)), dim3(kBlock), lds, s, t, P, Cp);
  else
    hipLaunchKernelGGL(bn_tail_apply_kernel<kTailMax>, dim3(grid_rows(P, Cp / 8)), dim3(kBlock), lds, s, t, P, Cp);
}

void bn_act_bwd_apply_part(const uint16_t* dz, const uint16_t* y, const float* scale, const float* shift,
                           const float* coef, uint16_t* dy, const uint16_t* y2, const float* scale2,
                           const float* shift2, const float* mean2, int relu2, float* part, long P, int Cp, int relu,
                           hipStream_t s) {
  hipLaunchKernelGGL(bn_act_bwd_apply_part_kernel, dim3(bn_partial_blocks(P, Cp)), dim3(kBlock), 0, s, dz, y, scale,
                     shift, coef, dy, y2, scale2, shift2, mean2, relu2, part, P, Cp, relu);
}

void bn_act_bwd_apply(const uint16_t* dz, const uint16_t* y, const float* scale, const float* shift,
                      const float* coef, uint16_t* dy, long P, int Cp, int relu, hipStream_t s) {
  hipLaunchKernelGGL(bn_act_bwd_apply_kernel, dim3(grid_rows(P, Cp / 8)), dim3(kBlock), 0, s, dz, y, scale, shift,
                     coef, dy, P, Cp / 8, relu);
}
