// Fused losses over NCHW fp32 logits (one pass computes the loss partials AND the gradient).
//   ce_fwd_bwd    : nn.CrossEntropyLoss(weight, ignore_index) with mean reduction; also emits the
//                   per-pixel loss for OHEM (reference core/loss.py:6-31).
//   kd_kl_fwd_bwd : F.kl_div(log_softmax(s/T), softmax(t/T)) * T^2, elementwise-mean reduction
//                   (reference core/loss.py:42-46).
//   mse_fwd_bwd   : F.mse_loss(s, t) (KD 'mse', reference core/loss.py:47-48).
//   bce_dice_*    : binary (num_class == 1) BCE-with-logits + per-sample soft Dice on the sigmoid
//                   (SURVEY Appendix E.1): a per-sample reduction pass, then the gradient pass once the
//                   sample's Dice sums are known.
// Partials are per block ([nblk][2] = {weighted loss sum, weight sum}); the host sums them.
#include "common.h"
#include "launchers.h"

namespace {
constexpr int kBlock = 256;
constexpr int kMaxC = 64;

__global__ __launch_bounds__(kBlock) void ce_kernel(const float* __restrict__ logits, const int64_t* __restrict__ target,
                                                    const float* __restrict__ weight, float* __restrict__ grad,
                                                    float* __restrict__ pix_loss, float* __restrict__ part, int N,
                                                    int C, long HW, int ignore_index) {
  __shared__ float red[2][kBlock / 64];
  const long P = (long)N * HW;
  float ls = 0.f, ws = 0.f;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < P; i += (long)gridDim.x * kBlock) {
    const long n = i / HW, p = i - n * HW;
    const float* x = logits + n * C * HW + p;
    float* gx = grad + n * C * HW + p;
    const long t = target[i];
    if (t == ignore_index || t < 0 || t >= C) {
      for (int c = 0; c < C; ++c) gx[c * HW] = 0.f;
      if (pix_loss) pix_loss[i] = 0.f;
      continue;
    }
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, x[c * HW]);
    // full-precision exp/log (the per-pixel losses rank pixels for OHEM: fast-math ulps reorder
    // near-equal confident pixels against the torch oracle)
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += expf(x[c * HW] - m);
    const float lse = m + logf(se);
    const float l = lse - x[t * HW];
    const float w = weight ? weight[t] : 1.f;
    ls += w * l;
    ws += w;
    if (pix_loss) pix_loss[i] = l;
    const float inv = 1.f / se;
    for (int c = 0; c < C; ++c) {
      const float pc = expf(x[c * HW] - m) * inv;
      gx[c * HW] = w * (pc - (c == t ? 1.f : 0.f));
    }
  }
  ls = wave_sum(ls);
  ws = wave_sum(ws);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = ls; red[1][threadIdx.x >> 6] = ws; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int w = 0; w < kBlock / 64; ++w) { a += red[0][w]; b += red[1][w]; }
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
}

__global__ __launch_bounds__(kBlock) void kd_kl_kernel(const float* __restrict__ s, const float* __restrict__ t,
                                                       float* __restrict__ grad, float* __restrict__ part, int N,
                                                       int C, long HW, float T) {
  __shared__ float red[kBlock / 64];
  const long P = (long)N * HW;
  const float invT = 1.f / T;
  const float gscale = T / (float)((double)N * C * HW);
  float acc = 0.f;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < P; i += (long)gridDim.x * kBlock) {
    const long n = i / HW, p = i - n * HW;
    const float* xs = s + n * C * HW + p;
    const float* xt = t + n * C * HW + p;
    float ms = -INFINITY, mt = -INFINITY;
    for (int c = 0; c < C; ++c) { ms = fmaxf(ms, xs[c * HW] * invT); mt = fmaxf(mt, xt[c * HW] * invT); }
    float ss = 0.f, st = 0.f;
    for (int c = 0; c < C; ++c) { ss += __expf(xs[c * HW] * invT - ms); st += __expf(xt[c * HW] * invT - mt); }
    const float lss = ms + __logf(ss), lst = mt + __logf(st);
    for (int c = 0; c < C; ++c) {
      const float lq = xs[c * HW] * invT - lss;   // log q (student)
      const float lp = xt[c * HW] * invT - lst;   // log p (teacher)
      const float pc = __expf(lp);
      acc += pc > 0.f ? pc * (lp - lq) : 0.f;
      grad[n * C * HW + c * HW + p] = gscale * (__expf(lq) - pc);
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f;
    for (int w = 0; w < kBlock / 64; ++w) a += red[w];
    part[blockIdx.x] = a;
  }
}
__global__ __launch_bounds__(kBlock) void mse_kernel(const float* __restrict__ s, const float* __restrict__ t,
                                                     float* __restrict__ grad, float* __restrict__ part, long n) {
  __shared__ float red[kBlock / 64];
  const float gs = 2.f / (float)n;
  float acc = 0.f;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long)gridDim.x * kBlock) {
    const float d = s[i] - t[i];
    acc += d * d;
    grad[i] = gs * d;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f;
    for (int w = 0; w < kBlock / 64; ++w) a += red[w];
    part[blockIdx.x] = a;
  }
}

DEVI float sigmoidf(float x) { return 1.f / (1.f + __expf(-x)); }

// grid (splits, N): block (b, n) reduces its slice of sample n into part[n][b][4] =
// {sum BCE, sum p*t, sum p, sum t}.
__global__ __launch_bounds__(kBlock) void bce_dice_stats_kernel(const float* __restrict__ x, const float* __restrict__ t,
                                                                float* __restrict__ part, long HW) {
  __shared__ float red[4][kBlock / 64];
  const int n = blockIdx.y;
  const float* xs = x + (long)n * HW;
  const float* ts = t + (long)n * HW;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < HW; i += (long)gridDim.x * kBlock) {
    const float v = xs[i], y = ts[i];
    const float p = sigmoidf(v);
    a[0] += fmaxf(v, 0.f) - v * y + log1pf(__expf(-fabsf(v)));
    a[1] += p * y;
    a[2] += p;
    a[3] += y;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float w = wave_sum(a[k]);
    if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = w;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float v = 0.f;
    for (int w = 0; w < kBlock / 64; ++w) v += red[threadIdx.x][w];
    part[((long)n * gridDim.x + blockIdx.x) * 4 + threadIdx.x] = v;
  }
}

// d/dx of  bw * mean(BCE) + dw * (1 - mean_n (2 I_n + s) / (D_n + s)),  scaled by the upstream
// gradient *gup (a device scalar: no host sync).  coef[n] = {D_n + s, 2 I_n + s}.
__global__ __launch_bounds__(kBlock) void bce_dice_grad_kernel(const float* __restrict__ x, const float* __restrict__ t,
                                                               const float* __restrict__ coef,
                                                               const float* __restrict__ gup, float* __restrict__ grad,
                                                               int N, long HW, float bw, float dw) {
  const long total = (long)N * HW;
  const float g0 = gup[0];
  const float kb = bw / (float)total, kd = dw / (float)N;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int n = (int)(i / HW);
    const float den = coef[2 * n], num = coef[2 * n + 1];
    const float p = sigmoidf(x[i]), y = t[i];
    const float gd = -kd * p * (1.f - p) * (2.f * y * den - num) / (den * den);
    grad[i] = g0 * (kb * (p - y) + gd);
  }
}

// ---- OHEM selection on the device (reference core/loss.py:13-20): loss_hard = L[L > thr]; if fewer
// than n_min = #valid // 16 survive, loss_hard = topk(L, n_min).  Both branches are evaluated with no
// host synchronisation (graph-capturable): counts/sums above thr, and an exact radix select of the
// n_min-th largest per-pixel loss (non-negative floats order like their uint32 bits) in four 8-bit
// passes.  Ties at the k-th value take the fractional weight (n_min - #greater) / #equal each, which
// gives torch's loss value exactly (torch picks an arbitrary subset of the ties).
// State words (uint32 / fp32 bit-casts): see kOh* below.  Partials per block, reduced in fixed order.
constexpr int kOhPrefix = 0, kOhK = 1, kOhCntAbove = 2, kOhSumAbove = 3, kOhNMin = 4, kOhMode = 5, kOhSel = 6,
              kOhWGt = 7, kOhWEq = 8, kOhLoss = 9, kOhWords = 16;

__global__ __launch_bounds__(kBlock) void ohem_count_kernel(const float* __restrict__ L, const int64_t* __restrict__ tgt,
                                                            long P, float thr, int ignore_index, float* __restrict__ bpart) {
  __shared__ float red[3][kBlock / 64];
  float c = 0.f, sm = 0.f, nv = 0.f;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < P; i += (long)gridDim.x * kBlock) {
    const float l = L[i];
    if (l > thr) { c += 1.f; sm += l; }
    nv += tgt[i] != ignore_index ? 1.f : 0.f;
  }
  c = wave_sum(c); sm = wave_sum(sm); nv = wave_sum(nv);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = c; red[1][threadIdx.x >> 6] = sm; red[2][threadIdx.x >> 6] = nv; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f, d = 0.f;
    for (int w = 0; w < kBlock / 64; ++w) { a += red[0][w]; b += red[1][w]; d += red[2][w]; }
    bpart[3 * blockIdx.x] = a; bpart[3 * blockIdx.x + 1] = b; bpart[3 * blockIdx.x + 2] = d;
  }
}

// one block: fixed-order reduction of the count partials, n_min, radix-select state, histogram reset
__global__ __launch_bounds__(kBlock) void ohem_init_kernel(const float* __restrict__ bpart, int nblk,
                                                           unsigned* __restrict__ st, unsigned* __restrict__ hist) {
  if (threadIdx.x == 0) {
    double c = 0.0, sm = 0.0, nv = 0.0;
    for (int b = 0; b < nblk; ++b) { c += bpart[3 * b]; sm += bpart[3 * b + 1]; nv += bpart[3 * b + 2]; }
    const unsigned n_min = (unsigned)((long long)nv / 16);
    st[kOhPrefix] = 0u;
    st[kOhK] = n_min;
    st[kOhCntAbove] = (unsigned)c;
    st[kOhSumAbove] = __float_as_uint((float)sm);
    st[kOhNMin] = n_min;
  }
  hist[threadIdx.x] = 0u;
}

__global__ __launch_bounds__(kBlock) void ohem_hist_kernel(const float* __restrict__ L, long P, int shift,
                                                           const unsigned* __restrict__ st, unsigned* __restrict__ hist) {
  __shared__ unsigned h[256];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const unsigned prefix = st[kOhPrefix];
  const int hs = shift + 8;   // bits above this digit must equal the decided prefix
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < P; i += (long)gridDim.x * kBlock) {
    const unsigned u = __float_as_uint(L[i]);
    if (hs >= 32 || (u >> hs) == (prefix >> hs)) atomicAdd(&h[(u >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// one block: the digit of the k-th largest among the candidates; k becomes its rank inside that digit
__global__ __launch_bounds__(kBlock) void ohem_pick_kernel(int shift, unsigned* __restrict__ st, unsigned* __restrict__ hist) {
  __shared__ unsigned cnt[256];
  cnt[threadIdx.x] = hist[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned k = st[kOhK];
    unsigned above = 0u, b = 0u;
    for (int d = 255; d >= 0; --d) {
      if (above + cnt[d] >= k) { b = (unsigned)d; break; }
      above += cnt[d];
    }
    st[kOhK] = k > above ? k - above : 0u;
    st[kOhPrefix] |= b << shift;
  }
  __syncthreads();
  hist[threadIdx.x] = 0u;   // ready for the next digit
}

__global__ __launch_bounds__(kBlock) void ohem_topk_kernel(const float* __restrict__ L, long P,
                                                           const unsigned* __restrict__ st, float* __restrict__ bpart) {
  __shared__ float red[3][kBlock / 64];
  const float vk = __uint_as_float(st[kOhPrefix]);
  float sgt = 0.f, cgt = 0.f, ceq = 0.f;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < P; i += (long)gridDim.x * kBlock) {
    const float l = L[i];
    if (l > vk) { sgt += l; cgt += 1.f; }
    else if (l == vk) ceq += 1.f;
  }
  sgt = wave_sum(sgt); cgt = wave_sum(cgt); ceq = wave_sum(ceq);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = sgt; red[1][threadIdx.x >> 6] = cgt; red[2][threadIdx.x >> 6] = ceq; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f, d = 0.f;
    for (int w = 0; w < kBlock / 64; ++w) { a += red[0][w]; b += red[1][w]; d += red[2][w]; }
    bpart[3 * blockIdx.x] = a; bpart[3 * blockIdx.x + 1] = b; bpart[3 * blockIdx.x + 2] = d;
  }
}

// one thread: pick the branch, write the loss and the per-pixel backward weights
__global__ void ohem_finish_kernel(const float* __restrict__ bpart, int nblk, float thr, unsigned* __restrict__ st,
                                   float* __restrict__ loss) {
  double sgt = 0.0, cgt = 0.0, ceq = 0.0;
  for (int b = 0; b < nblk; ++b) { sgt += bpart[3 * b]; cgt += bpart[3 * b + 1]; ceq += bpart[3 * b + 2]; }
  const unsigned n_min = st[kOhNMin], c_above = st[kOhCntAbove];
  const float vk = __uint_as_float(st[kOhPrefix]);
  float l, sel, wgt, weq;
  unsigned mode;
  if (c_above >= n_min) {   // threshold branch: mean of the losses above thr
    mode = 0u;
    sel = thr;
    wgt = c_above > 0 ? 1.f / (float)c_above : 0.f;
    weq = 0.f;
    l = c_above > 0 ? __uint_as_float(st[kOhSumAbove]) * wgt : 0.f;
  } else {                  // top-k branch: the n_min largest (ties at the k-th value shared)
    mode = 1u;
    sel = vk;
    const double take_eq = (double)n_min - cgt;
    l = (float)((sgt + take_eq * (double)vk) / (double)n_min);
    wgt = 1.f / (float)n_min;
    weq = ceq > 0.0 ? (float)(take_eq / ceq) * wgt : 0.f;
  }
  st[kOhMode] = mode;
  st[kOhSel] = __float_as_uint(sel);
  st[kOhWGt] = __float_as_uint(wgt);
  st[kOhWEq] = __float_as_uint(weq);
  loss[0] = l;
}

// backward: grad_logits[n][c][p] *= g * w(L[n][p]) in place
__global__ __launch_bounds__(kBlock) void ohem_bwd_kernel(float* __restrict__ grad, const float* __restrict__ L,
                                                          const unsigned* __restrict__ st, const float* __restrict__ gup,
                                                          int N, int C, long HW) {
  const float sel = __uint_as_float(st[kOhSel]), wgt = __uint_as_float(st[kOhWGt]) * gup[0];
  const float weq = __uint_as_float(st[kOhWEq]) * gup[0];
  const long P = (long)N * HW;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < P; i += (long)gridDim.x * kBlock) {
    const float l = L[i];
    const float w = l > sel ? wgt : (l == sel ? weq : 0.f);
    const long n = i / HW, p = i - n * HW;
    float* gx = grad + n * C * HW + p;
    for (int c = 0; c < C; ++c) gx[c * HW] *= w;
  }
}
}  // namespace

long ce_blocks(long P) {
  long b = (P + kBlock * 8 - 1) / (kBlock * 8);
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return b;
}

void ce_fwd_bwd(const float* logits, const int64_t* target, const float* weight, float* grad, float* pix_loss,
                float* part, int N, int C, long HW, int ignore_index, hipStream_t s) {
  (void)kMaxC;
  hipLaunchKernelGGL(ce_kernel, dim3(ce_blocks((long)N * HW)), dim3(kBlock), 0, s, logits, target, weight, grad,
                     pix_loss, part, N, C, HW, ignore_index);
}

void kd_kl_fwd_bwd(const float* s_logits, const float* t_logits, float* grad, float* part, int N, int C, long HW,
                   float T, hipStream_t s) {
  hipLaunchKernelGGL(kd_kl_kernel, dim3(ce_blocks((long)N * HW)), dim3(kBlock), 0, s, s_logits, t_logits, grad,
                     part, N, C, HW, T);
}

void mse_fwd_bwd(const float* s_, const float* t, float* grad, float* part, long n, hipStream_t s) {
  hipLaunchKernelGGL(mse_kernel, dim3(ce_blocks(n)), dim3(kBlock), 0, s, s_, t, grad, part, n);
}

int bce_dice_splits(long HW) {
  long b = (HW + kBlock * 16 - 1) / (kBlock * 16);
  if (b > 256) b = 256;
  if (b < 1) b = 1;
  return (int)b;
}

void bce_dice_stats(const float* x, const float* t, float* part, int N, long HW, hipStream_t s) {
  hipLaunchKernelGGL(bce_dice_stats_kernel, dim3(bce_dice_splits(HW), N), dim3(kBlock), 0, s, x, t, part, HW);
}

void bce_dice_grad(const float* x, const float* t, const float* coef, const float* gup, float* grad, int N, long HW,
                   float bw, float dw, hipStream_t s) {
  hipLaunchKernelGGL(bce_dice_grad_kernel, dim3(ce_blocks((long)N * HW)), dim3(kBlock), 0, s, x, t, coef, gup, grad,
                     N, HW, bw, dw);
}

int ohem_state_words() { return kOhWords; }

void ohem_select(const float* pix_loss, const int64_t* target, long P, float thr, int ignore_index, float* bpart,
                 unsigned* state, unsigned* hist, float* loss, hipStream_t s) {
  const int nblk = (int)ce_blocks(P);
  hipLaunchKernelGGL(ohem_count_kernel, dim3(nblk), dim3(kBlock), 0, s, pix_loss, target, P, thr, ignore_index, bpart);
  hipLaunchKernelGGL(ohem_init_kernel, dim3(1), dim3(kBlock), 0, s, bpart, nblk, state, hist);
  for (int shift = 24; shift >= 0; shift -= 8) {
    hipLaunchKernelGGL(ohem_hist_kernel, dim3(nblk), dim3(kBlock), 0, s, pix_loss, P, shift, state, hist);
    hipLaunchKernelGGL(ohem_pick_kernel, dim3(1), dim3(kBlock), 0, s, shift, state, hist);
  }
  hipLaunchKernelGGL(ohem_topk_kernel, dim3(nblk), dim3(kBlock), 0, s, pix_loss, P, state, bpart);
  hipLaunchKernelGGL(ohem_finish_kernel, dim3(1), dim3(1), 0, s, bpart, nblk, thr, state, loss);
}

void ohem_backward(float* grad, const float* pix_loss, const unsigned* state, const float* gup, int N, int C, long HW,
                   hipStream_t s) {
  hipLaunchKernelGGL(ohem_bwd_kernel, dim3(ce_blocks((long)N * HW)), dim3(kBlock), 0, s, grad, pix_loss, state, gup,
                     N, C, HW);
}
