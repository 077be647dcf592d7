// Batched attention GEMMs + whole-map softmax for MAnet's position-attention block (PAB; reference hub
// models/__init__.py:8-10 -> segmentation_models_pytorch MAnet): S = center . top^T over the hw positions,
// softmax over the WHOLE flattened hw x hw map of each image (the reference's view(b, -1) quirk), then
// S . bottom -- and their backward.  The maps are small (hw = 121 at a 352 input's stride-32 level), so one
// generic MFMA kernel covers every operand transposition of the five products (forward 2, backward 3).
#include "common.h"
#include "launchers.h"

namespace {

DEVI float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

constexpr int kAtTile = 64;   // C tile (64 x 64) per 256-thread block: 2 x 2 waves of 32 x 32 (2 x 2 MFMA 16x16)
constexpr int kAtK = 32;      // k per stage (one v_mfma_f32_16x16x32_bf16)
constexpr int kAtPitch = kAtK + 8;   // LDS row pitch (elements): k-contiguous rows, +16 B against bank repeats

// C[b] (M x N) = op(A[b]) (M x K) . op(B[b]) (K x N), bf16 operands, fp32 accumulation.
// A(m, k) = transA ? A[k * lda + m] : A[m * lda + k];  B(k, n) = transB ? B[n * ldb + k] : B[k * ldb + n].
// OUT_BF16: C stored as bf16 (round to nearest even), else fp32.  Both LDS images are k-contiguous (row = m or
// n), so each MFMA operand fragment is one 16-B LDS read; the global->LDS copy transposes element-wise
// (2-B loads: these GEMMs are a few MFLOP, latency- not bandwidth-bound).
template <bool OUT_BF16>
__global__ __launch_bounds__(256) void batched_gemm_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                           void* __restrict__ Cv, int M, int N, int K, int lda, int ldb,
                                                           int ldc, long sa, long sb, long sc, int transA, int transB) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[kAtTile * kAtPitch];
  __shared__ __attribute__((aligned(16))) uint16_t sB[kAtTile * kAtPitch];
  const int b = blockIdx.z;
  const int m0 = blockIdx.y * kAtTile, n0 = blockIdx.x * kAtTile;
  const uint16_t* Ab = A + b * sa;
  const uint16_t* Bb = B + b * sb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += kAtK) {
    // 64 x 32 elements per operand: 8 per thread; consecutive threads walk the operand's contiguous axis
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = tid + 256 * e;
      int r, kk;   // LDS row (m or n) and k
      if (transA) { kk = idx / kAtTile; r = idx - kk * kAtTile; } else { r = idx / kAtK; kk = idx - r * kAtK; }
      const int gm = m0 + r, gk = k0 + kk;
      uint16_t v = 0;
      if (gm < M && gk < K) v = transA ? Ab[(long)gk * lda + gm] : Ab[(long)gm * lda + gk];
      sA[r * kAtPitch + kk] = v;
      if (transB) { r = idx / kAtK; kk = idx - r * kAtK; } else { kk = idx / kAtTile; r = idx - kk * kAtTile; }
      const int gn = n0 + r, gk2 = k0 + kk;
      uint16_t w = 0;
      if (gn < N && gk2 < K) w = transB ? Bb[(long)gn * ldb + gk2] : Bb[(long)gk2 * ldb + gn];
      sB[r * kAtPitch + kk] = w;
    }
    __syncthreads();
    uint4 fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const uint4*>(sA + (wm + 16 * i + lr) * kAtPitch + 8 * lg);
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = *reinterpret_cast<const uint4*>(sB + (wn + 16 * j + lr) * kAtPitch + 8 * lg);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16x16x32(fa[i], fb[j], acc[i][j]);
    __syncthreads();
  }
  // D fragment: lane (lr, lg) holds rows 4*lg + r, column lr of each 16 x 16 block
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + 16 * i + 4 * lg + r, gn = n0 + wn + 16 * j + lr;
        if (gm >= M || gn >= N) continue;
        const long o = b * sc + (long)gm * ldc + gn;
        if (OUT_BF16) static_cast<uint16_t*>(Cv)[o] = f2bf(acc[i][j][r]);
        else static_cast<float*>(Cv)[o] = acc[i][j][r];
      }
}

// softmax over each image's whole flattened map (n = hw * hw values): P = exp(S - max) / sum, bf16 out.
// One 1024-thread block per image; fp32 max / sum in LDS.
__global__ __launch_bounds__(1024) void softmax_all_kernel(const float* __restrict__ S, uint16_t* __restrict__ P, long n) {
  __shared__ float red[32];
  const float* s = S + blockIdx.x * n;
  uint16_t* p = P + blockIdx.x * n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float mx = -INFINITY;
  for (long i = tid; i < n; i += 1024) mx = fmaxf(mx, s[i]);
  mx = wave_max(mx);
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = red[0];
  for (int w = 1; w < 16; ++w) mx = fmaxf(mx, red[w]);
  __syncthreads();
  float sum = 0.f;
  for (long i = tid; i < n; i += 1024) sum += __expf(s[i] - mx);
  sum = wave_sum(sum);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  sum = 0.f;
  for (int w = 0; w < 16; ++w) sum += red[w];
  const float inv = 1.f / sum;
  for (long i = tid; i < n; i += 1024) p[i] = f2bf(__expf(s[i] - mx) * inv);
}

// its backward over the same flattened map: dS = P * (dP - sum(P * dP)), bf16 out
__global__ __launch_bounds__(1024) void softmax_all_bwd_kernel(const uint16_t* __restrict__ P, const float* __restrict__ dP,
                                                               uint16_t* __restrict__ dS, long n) {
  __shared__ float red[32];
  const uint16_t* p = P + blockIdx.x * n;
  const float* g = dP + blockIdx.x * n;
  uint16_t* o = dS + blockIdx.x * n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float dot = 0.f;
  for (long i = tid; i < n; i += 1024) dot += bf2f(p[i]) * g[i];
  dot = wave_sum(dot);
  if (lane == 0) red[wave] = dot;
  __syncthreads();
  dot = 0.f;
  for (int w = 0; w < 16; ++w) dot += red[w];
  for (long i = tid; i < n; i += 1024) o[i] = f2bf(bf2f(p[i]) * (g[i] - dot));
}

}  // namespace

int batched_gemm(const uint16_t* A, const uint16_t* B, void* C, bool out_bf16, int batch, int M, int N, int K, int lda,
                 int ldb, int ldc, long sa, long sb, long sc, bool transA, bool transB, hipStream_t s) {
  if (batch < 1 || M < 1 || N < 1 || K < 1 || batch > 65535) return 1;
  const dim3 grid(cdiv(N, kAtTile), cdiv(M, kAtTile), batch);
  if (out_bf16)
    hipLaunchKernelGGL(batched_gemm_kernel<true>, grid, dim3(256), 0, s, A, B, C, M, N, K, lda, ldb, ldc, sa, sb, sc,
                       transA ? 1 : 0, transB ? 1 : 0);
  else
    hipLaunchKernelGGL(batched_gemm_kernel<false>, grid, dim3(256), 0, s, A, B, C, M, N, K, lda, ldb, ldc, sa, sb, sc,
                       transA ? 1 : 0, transB ? 1 : 0);
  return 0;
}

void softmax_all(const float* S, uint16_t* P, int batch, long n, hipStream_t s) {
  hipLaunchKernelGGL(softmax_all_kernel, dim3(batch), dim3(1024), 0, s, S, P, n);
}

void softmax_all_bwd(const uint16_t* P, const float* dP, uint16_t* dS, int batch, long n, hipStream_t s) {
  hipLaunchKernelGGL(softmax_all_bwd_kernel, dim3(batch), dim3(1024), 0, s, P, dP, dS, n);
}
