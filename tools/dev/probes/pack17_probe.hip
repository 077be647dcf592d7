// Dev probe (round 5): the 17 -> 24 channel padding question measured on two pass types of
// the 17-channel level at the bench size (320 x 352 x 352 pixels):
//   1. a BN(+ReLU) apply pass (bn_act_apply's shape of work): bf16 in -> bf16 out, per-channel scale / shift;
//   2. conv halo staging (the fused kernels' producer role): per 512-pixel tile (16 x 32 + a 1-pixel halo)
//      the input tile into a 24-channel LDS image (what the MFMA loops read), then a token consumer.
// Each for the padded layout ([P][24], 48 B / pixel, 16-B vectors) and a packed layout ([P][17], 34 B / pixel:
// pixel pairs = 68 B = 17 dwords; 16-B vectors that straddle pixels, channel of element e = e % 17).
// hipcc -O3 --offload-arch=gfx950 tools/dev/probes/pack17_probe.hip -o /tmp/pack17 && /tmp/pack17
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ float bf(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t tobf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// ---- 1. BN apply -------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void apply_padded(const uint4* __restrict__ x, uint4* __restrict__ y, long nvec,
                                                    const float* __restrict__ sc, const float* __restrict__ sh) {
  for (long v = blockIdx.x * 256L + threadIdx.x; v < nvec; v += (long)gridDim.x * 256) {
    const int c0 = (int)(v % 3) * 8;   // 3 vectors per pixel
    uint4 a = x[v];
    uint16_t* e = reinterpret_cast<uint16_t*>(&a);
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = c0 + k < 17 ? tobf(fmaxf(fmaf(bf(e[k]), sc[c0 + k], sh[c0 + k]), 0.f)) : 0;
    y[v] = a;
  }
}

__global__ __launch_bounds__(256) void apply_packed(const uint4* __restrict__ x, uint4* __restrict__ y, long nvec,
                                                    const float* __restrict__ sc, const float* __restrict__ sh) {
  for (long v = blockIdx.x * 256L + threadIdx.x; v < nvec; v += (long)gridDim.x * 256) {
    int c = (int)(((unsigned)v * 8u) % 17u);   // channel of the vector's first element (32-bit: < 2^31 elements)
    uint4 a = x[v];
    uint16_t* e = reinterpret_cast<uint16_t*>(&a);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      e[k] = tobf(fmaxf(fmaf(bf(e[k]), sc[c], sh[c]), 0.f));
      c = c == 16 ? 0 : c + 1;
    }
    y[v] = a;
  }
}

// ---- 2. halo staging into a 24-channel LDS image -------------------------------------------------------------
constexpr int TH = 16, TW = 32, HH = TH + 2, HW = TW + 2, PITCH = 24;
__global__ __launch_bounds__(256) void stage_padded(const uint16_t* __restrict__ x, float* __restrict__ out, int N, int H,
                                                    int W, int tiles) {
  __shared__ uint4 tile[HH * HW * 3];
  const int tx_n = (W + TW - 1) / TW, ty_n = (H + TH - 1) / TH;
  float acc = 0.f;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int n = t / (tx_n * ty_n), r = t % (tx_n * ty_n), y0 = (r / tx_n) * TH - 1, x0 = (r % tx_n) * TW - 1;
    for (int e = threadIdx.x; e < HH * HW * 3; e += 256) {
      const int p = e / 3, c8 = e % 3, iy = y0 + p / HW, ix = x0 + p % HW;
      uint4 v = make_uint4(0, 0, 0, 0);
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
        v = *reinterpret_cast<const uint4*>(x + (((long)n * H + iy) * W + ix) * PITCH + 8 * c8);
      tile[e] = v;
    }
    __syncthreads();
    acc += bf(reinterpret_cast<const uint16_t*>(tile)[(threadIdx.x * 7) % (HH * HW * PITCH)]);
    __syncthreads();
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// packed source: each thread copies 16-B vectors of a halo row's contiguous 17-channel run and scatters the 8
// elements (2 B each) into the padded image; rows are pixel-contiguous, so a row is one element range
__global__ __launch_bounds__(256) void stage_packed(const uint16_t* __restrict__ x, float* __restrict__ out, int N, int H,
                                                    int W, int tiles) {
  __shared__ uint16_t tile[HH * HW * PITCH];
  const int tx_n = (W + TW - 1) / TW, ty_n = (H + TH - 1) / TH;
  float acc = 0.f;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int n = t / (tx_n * ty_n), r = t % (tx_n * ty_n), y0 = (r / tx_n) * TH - 1, x0 = (r % tx_n) * TW - 1;
    for (int e = threadIdx.x; e < HH * HW * PITCH / 8; e += 256) reinterpret_cast<uint4*>(tile)[e] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    // per halo row: elements [17 * px0, 17 * px1) of the row's in-image pixels, read in 8-element (16-B) pieces
    // from the enclosing 16-B aligned range
    for (int row = 0; row < HH; ++row) {
      const int iy = y0 + row;
      if ((unsigned)iy >= (unsigned)H) continue;
      const int pa = max(x0, 0), pb = min(x0 + HW, W);
      const long ebeg = (((long)n * H + iy) * W + pa) * 17, eend = (((long)n * H + iy) * W + pb) * 17;
      const long vbeg = ebeg / 8, vend = (eend + 7) / 8;
      for (long v = vbeg + threadIdx.x; v < vend; v += 256) {
        const uint4 a = *reinterpret_cast<const uint4*>(x + 8 * v);
        const uint16_t* ev = reinterpret_cast<const uint16_t*>(&a);
        const int rel0 = (int)(8 * v - ebeg);   // element index within the row's run (32-bit, constant divisor)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int rel = rel0 + k;
          if (rel < 0 || rel >= (int)(eend - ebeg)) continue;
          const int px = (unsigned)rel / 17u, c = rel - px * 17;
          tile[(row * HW + (pa - x0) + px) * PITCH + c] = ev[k];
        }
      }
    }
    __syncthreads();
    acc += bf(tile[(threadIdx.x * 7) % (HH * HW * PITCH)]);
    __syncthreads();
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <typename F>
float time_ms(F f, int reps = 10) {
  f();
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const int N = 320, H = 352, W = 352;
  const long P = (long)N * H * W;
  const long e24 = P * 24, e17 = (P * 17 + 7) / 8 * 8;
  uint16_t *x24, *y24, *x17, *y17;
  float *sc, *sh, *out;
  CK(hipMalloc(&x24, e24 * 2)); CK(hipMalloc(&y24, e24 * 2));
  CK(hipMalloc(&x17, e17 * 2 + 64)); CK(hipMalloc(&y17, e17 * 2 + 64));
  CK(hipMalloc(&sc, 32 * 4)); CK(hipMalloc(&sh, 32 * 4)); CK(hipMalloc(&out, 2048 * 256 * 4));
  CK(hipMemset(x24, 0x3c, e24 * 2)); CK(hipMemset(x17, 0x3c, e17 * 2));
  std::vector<float> h(32, 0.5f);
  CK(hipMemcpy(sc, h.data(), 128, hipMemcpyHostToDevice)); CK(hipMemcpy(sh, h.data(), 128, hipMemcpyHostToDevice));
  const int grid = 256 * 8;
  const float a24 = time_ms([&] { hipLaunchKernelGGL(apply_padded, dim3(grid), dim3(256), 0, 0, (const uint4*)x24, (uint4*)y24, e24 / 8, sc, sh); });
  const float a17 = time_ms([&] { hipLaunchKernelGGL(apply_packed, dim3(grid), dim3(256), 0, 0, (const uint4*)x17, (uint4*)y17, e17 / 8, sc, sh); });
  const int tiles = N * ((H + TH - 1) / TH) * ((W + TW - 1) / TW);
  const float s24 = time_ms([&] { hipLaunchKernelGGL(stage_padded, dim3(grid), dim3(256), 0, 0, x24, out, N, H, W, tiles); });
  const float s17 = time_ms([&] { hipLaunchKernelGGL(stage_packed, dim3(grid), dim3(256), 0, 0, x17, out, N, H, W, tiles); });
  CK(hipDeviceSynchronize());
  const double g24 = e24 * 2 / 1e9, g17 = P * 34 / 1e9;
  printf("{\"pass\": \"bn_apply\", \"padded24_ms\": %.3f, \"packed17_ms\": %.3f, \"padded24_TBps\": %.2f, \"packed17_TBps\": %.2f, \"ratio\": %.3f}\n",
         a24, a17, 2 * g24 / a24, 2 * g17 / a17, a17 / a24);
  printf("{\"pass\": \"halo_staging_512px_tiles\", \"padded24_ms\": %.3f, \"packed17_ms\": %.3f, \"padded24_TBps\": %.2f, \"packed17_TBps\": %.2f, \"ratio\": %.3f}\n",
         s24, s17, g24 * 1.2 / s24, g17 * 1.2 / s17, s17 / s24);
  return 0;
}
