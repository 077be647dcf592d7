// Single-launch optimizers and EMA over flat fp32 arenas (all parameters of a model live in one
// contiguous buffer, so an optimizer step is ONE kernel instead of torch's per-tensor launches).
// Hyper-parameters are read from DEVICE memory so a hipGraph-captured step picks up the OneCycle
// lr / momentum values written before each replay.
//   Adam/AdamW hyper: [lr, beta1, beta2, eps, weight_decay, bias_corr1, bias_corr2, grad_scale]
//   SGD hyper:        [lr, momentum, weight_decay, grad_scale]
//   EMA hyper:        [decay]
//   AMP state (fp16 loss scaling, torch GradScaler semantics; optional):
//                     [scale, growth_tracker, found_inf, applied_steps]
//   With AMP state the optimizers unscale by 1/scale, skip the whole update when the finite check
//   found an inf/NaN (uniform over the grid: every thread reads the same flag), and take Adam's bias
//   corrections from the device step count (skipped steps do not count, as in torch).
// Semantics follow torch.optim.{Adam, AdamW, SGD} (reference utils/optimizer.py:4-21) and
// ModelEmaV2.update (reference utils/model_ema.py:28-40).
#include "common.h"
#include "launchers.h"

namespace {
constexpr int kBlock = 256;

int grid_for(long n) {
  long b = (n / 4 + kBlock - 1) / kBlock;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, const float* __restrict__ hyper, long n, int adamw,
                            const float* __restrict__ amp) {
  const float lr = hyper[0], b1 = hyper[1], b2 = hyper[2], eps = hyper[3], wd = hyper[4];
  float bc1 = hyper[5], bc2 = hyper[6], gs = hyper[7];
  if (amp != nullptr) {
    if (amp[2] != 0.f) return;   // non-finite gradients: step skipped
    gs /= amp[0];
    const float t = amp[3] + 1.f;
    bc1 = 1.f - powf(b1, t);
    bc2 = 1.f - powf(b2, t);
  }
  const float step = lr / bc1, rbc2 = rsqrtf(bc2);
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long)gridDim.x * kBlock) {
    float pi = p[i];
    float gi = g[i] * gs;
    if (!adamw && wd != 0.f) gi += wd * pi;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    if (adamw) pi *= 1.f - lr * wd;
    const float denom = sqrtf(vi) * rbc2 + eps;
    p[i] = pi - step * mi / denom;
  }
}

__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf,
                           const float* __restrict__ hyper, long n, const float* __restrict__ amp) {
  const float lr = hyper[0], mom = hyper[1], wd = hyper[2];
  float gs = hyper[3];
  if (amp != nullptr) {
    if (amp[2] != 0.f) return;
    gs /= amp[0];
  }
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long)gridDim.x * kBlock) {
    const float pi = p[i];
    float gi = g[i] * gs + wd * pi;
    if (mom != 0.f) {
      gi = mom * buf[i] + gi;
      buf[i] = gi;
    }
    p[i] = pi - lr * gi;
  }
}

// Finite check of the (scaled) gradient arena: any inf/NaN sets found_inf.  Every block that finds
// one stores the same 1.0 (benign race, plain vector store).
__global__ void amp_check_kernel(const float* __restrict__ g, long n, float* __restrict__ amp) {
  int bad = 0;
  const long n4 = n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (long)gridDim.x * kBlock) {
    const float4 v = g4[i];
    bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
  }
  for (long i = (n4 << 2) + (long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long)gridDim.x * kBlock)
    bad |= !isfinite(g[i]);
  if (__syncthreads_or(bad) && threadIdx.x == 0) amp[2] = 1.f;
}

// torch._amp_update_scale_: backoff on overflow, growth after `interval` clean steps; re-arms the flag.
__global__ void amp_update_kernel(float* __restrict__ amp, float growth, float backoff, int interval) {
  if (threadIdx.x != 0) return;
  float scale = amp[0], tracker = amp[1];
  if (amp[2] != 0.f) {
    scale *= backoff;
    tracker = 0.f;
  } else {
    amp[3] = amp[3] + 1.f;
    tracker += 1.f;
    if (tracker >= (float)interval) {
      const float grown = scale * growth;
      if (isfinite(grown)) scale = grown;
      tracker = 0.f;
    }
  }
  amp[0] = scale;
  amp[1] = tracker;
  amp[2] = 0.f;
}

__global__ void ema_kernel(float* __restrict__ e, const float* __restrict__ m, const float* __restrict__ hyper, long n) {
  const float d = hyper[0];
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long)gridDim.x * kBlock)
    e[i] = d * e[i] + (1.f - d) * m[i];
}
}  // namespace

void adam_step(float* p, const float* g, float* m, float* v, const float* hyper, long n, int adamw,
               const float* amp, hipStream_t s) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, p, g, m, v, hyper, n, adamw, amp);
}

void sgd_step(float* p, const float* g, float* buf, const float* hyper, long n, const float* amp, hipStream_t s) {
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, p, g, buf, hyper, n, amp);
}

void amp_check(const float* g, long n, float* amp, hipStream_t s) {
  hipLaunchKernelGGL(amp_check_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, g, n, amp);
}

void amp_update(float* amp, float growth, float backoff, int interval, hipStream_t s) {
  hipLaunchKernelGGL(amp_update_kernel, dim3(1), dim3(64), 0, s, amp, growth, backoff, interval);
}

void ema_update(float* ema, const float* model, const float* hyper, long n, hipStream_t s) {
  hipLaunchKernelGGL(ema_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, ema, model, hyper, n);
}
