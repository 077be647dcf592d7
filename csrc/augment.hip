// Train-time augmentation on the GPU over an HBM-resident uint8 dataset (reference
// datasets/polyp.py:37-47, albumentations semantics of SURVEY Appendix D as implemented on the host by
// utils/transforms.SegAugment -- the host draws every random number in the same order, the kernels
// only evaluate).  One batch =
//   aug_geometry   : RandomScale (image bilinear / mask nearest, the uint8 rounding of a resize) ->
//                    PadIfNeeded (centred BORDER_REFLECT_101) -> RandomCrop -> H/V flips, gathered
//                    per OUTPUT pixel straight from the variable-size source image (no intermediate
//                    scaled/padded copies);
//   aug_gray_mean  : per-sample mean of the gray image (ColorJitter contrast needs it at its position
//                    in the random op order; sliced fp64 partials + an in-order final sum);
//   aug_color      : one ColorJitter stage (brightness / contrast / saturation / hue per sample);
//   aug_finalize   : round (when jittered) + Normalize(mean, std) -> fp32 NCHW model input.
// Work buffer: fp32 [B][H*W][3] (RGB 0..255).  iparams (int32, kAugIParams per sample):
//   0 image index, 1 nh, 2 nw (scaled size), 3 pad top, 4 pad left, 5 crop y0, 6 crop x0, 7 hflip,
//   8 vflip, 9 jittered, 10..13 op code per stage (0 none, 1 brightness, 2 contrast, 3 saturation, 4 hue)
// fparams (fp32, 4 per sample): op value per stage.
#include "common.h"
#include "launchers.h"

namespace {
constexpr int kBlock = 256;

int grid_for(long n) {
  long b = (n + kBlock - 1) / kBlock;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (int)b;
}

DEVI int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * (n - 1) - i;
  return i;
}

__global__ __launch_bounds__(kBlock) void aug_geometry_kernel(const uint8_t* __restrict__ images,
                                                              const uint8_t* __restrict__ masks,
                                                              const int64_t* __restrict__ meta,
                                                              const int* __restrict__ ip, float* __restrict__ work,
                                                              int64_t* __restrict__ mask_out, int B, int CH, int CW) {
  const long total = (long)B * CH * CW;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int b = (int)(i / ((long)CH * CW));
    const int pix = (int)(i - (long)b * CH * CW);
    const int oy = pix / CW, ox = pix - oy * CW;
    const int* q = ip + b * kAugIParams;
    const int img = q[0], nh = q[1], nw = q[2];
    const int64_t off = meta[4 * img], moff = meta[4 * img + 3];
    const int h = (int)meta[4 * img + 1], w = (int)meta[4 * img + 2];
    // flips act last in the reference pipeline: output (oy, ox) reads crop pixel (cy, cx)
    const int cy = q[8] ? CH - 1 - oy : oy;
    const int cx = q[7] ? CW - 1 - ox : ox;
    // crop -> padded canvas -> scaled image (reflect-101 padding)
    const int sy = reflect101(cy + q[5] - q[3], nh);
    const int sx = reflect101(cx + q[6] - q[4], nw);
    float rgb[3];
    uint8_t m;
    if (nh == h && nw == w) {
      const uint8_t* p = images + off + ((long)sy * w + sx) * 3;
      rgb[0] = p[0]; rgb[1] = p[1]; rgb[2] = p[2];
      m = masks[moff + (long)sy * w + sx];
    } else {
      // torch F.interpolate(bilinear, align_corners=False): src = max((dst + 0.5) * in/out - 0.5, 0)
      const float ry = (float)h / (float)nh, rx = (float)w / (float)nw;
      const float fy = fmaxf((sy + 0.5f) * ry - 0.5f, 0.f), fx = fmaxf((sx + 0.5f) * rx - 0.5f, 0.f);
      const int y0 = (int)fy, x0 = (int)fx;
      const int y1 = y0 + (y0 < h - 1), x1 = x0 + (x0 < w - 1);
      const float ly = fy - y0, lx = fx - x0;
      const uint8_t* r0 = images + off + (long)y0 * w * 3;
      const uint8_t* r1 = images + off + (long)y1 * w * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v = (1.f - ly) * ((1.f - lx) * r0[x0 * 3 + c] + lx * r0[x1 * 3 + c]) +
                        ly * ((1.f - lx) * r1[x0 * 3 + c] + lx * r1[x1 * 3 + c]);
        rgb[c] = fminf(fmaxf(rintf(v), 0.f), 255.f);        // resize of a uint8 image rounds
      }
      // nearest: src = min(floor(dst * in/out), in - 1)
      const int my = min((int)floorf(sy * ry), h - 1), mx = min((int)floorf(sx * rx), w - 1);
      m = masks[moff + (long)my * w + mx];
    }
    float* o = work + i * 3;
    o[0] = rgb[0]; o[1] = rgb[1]; o[2] = rgb[2];
    mask_out[i] = m;
  }
}

DEVI float gray(const float* p) { return p[0] * 0.299f + p[1] * 0.587f + p[2] * 0.114f; }

// mean of each sample's gray image in fp64, deterministic: kGraySlices blocks per sample each reduce a
// fixed pixel slice (tree in LDS) to one fp64 partial, then one thread per sample adds its slices in
// order.  (One block per sample left 3/4 of the CUs idle: 155 us per launch at bs64 x 352^2.)
constexpr int kGraySlices = 16;

__global__ __launch_bounds__(kBlock) void aug_gray_partial_kernel(const float* __restrict__ work,
                                                                  double* __restrict__ part, int HW) {
  const int b = blockIdx.y, sl = blockIdx.x;
  const int per = (HW + kGraySlices - 1) / kGraySlices;
  const int i0 = sl * per, i1 = min(HW, i0 + per);
  const float* w = work + (long)b * HW * 3;
  double acc = 0.0;
  for (int i = i0 + threadIdx.x; i < i1; i += kBlock) acc += (double)gray(w + (long)i * 3);
  __shared__ double red[kBlock];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(long)b * kGraySlices + sl] = red[0];
}

__global__ __launch_bounds__(kBlock) void aug_gray_final_kernel(const double* __restrict__ part,
                                                                float* __restrict__ mean, int B, int HW) {
  const int b = blockIdx.x * kBlock + threadIdx.x;
  if (b >= B) return;
  double t = 0.0;
  for (int sl = 0; sl < kGraySlices; ++sl) t += part[(long)b * kGraySlices + sl];
  mean[b] = (float)(t / HW);
}

DEVI float clip255(float v) { return fminf(fmaxf(v, 0.f), 255.f); }
DEVI float mod1(float x) { return x - floorf(x); }

DEVI void adjust_hue(float* px, float shift) {
  const float r = px[0] / 255.f, g = px[1] / 255.f, b = px[2] / 255.f;
  const float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b));
  const float d = mx - mn;
  float h = 0.f;
  if (d > 1e-12f) {
    const float rc = (mx - r) / d, gc = (mx - g) / d, bc = (mx - b) / d;
    h = r == mx ? bc - gc : (g == mx ? 2.f + rc - bc : 4.f + gc - rc);
    h = mod1(h / 6.f);
  }
  const float s = mx > 1e-12f ? d / mx : 0.f;
  const float v = mx;
  h = mod1(h + shift);
  const float fi = floorf(h * 6.f);
  const float f = h * 6.f - fi;
  const float p = v * (1.f - s), q = v * (1.f - s * f), t = v * (1.f - s * (1.f - f));
  int i = ((int)fi) % 6;
  if (i < 0) i += 6;
  float o0, o1, o2;
  switch (i) {
    case 0: o0 = v; o1 = t; o2 = p; break;
    case 1: o0 = q; o1 = v; o2 = p; break;
    case 2: o0 = p; o1 = v; o2 = t; break;
    case 3: o0 = p; o1 = q; o2 = v; break;
    case 4: o0 = t; o1 = p; o2 = v; break;
    default: o0 = v; o1 = p; o2 = q; break;
  }
  px[0] = clip255(o0 * 255.f); px[1] = clip255(o1 * 255.f); px[2] = clip255(o2 * 255.f);
}

__global__ __launch_bounds__(kBlock) void aug_color_kernel(float* __restrict__ work, const int* __restrict__ ip,
                                                           const float* __restrict__ fp, const float* __restrict__ mean,
                                                           int B, int HW, int stage) {
  const long total = (long)B * HW;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int b = (int)(i / HW);
    const int op = ip[b * kAugIParams + 10 + stage];
    if (op == 0) continue;
    const float v = fp[b * 4 + stage];
    float* px = work + i * 3;
    if (op == 1) {
#pragma unroll
      for (int c = 0; c < 3; ++c) px[c] = clip255(px[c] * v);
    } else if (op == 2) {
      const float m = mean[b];
#pragma unroll
      for (int c = 0; c < 3; ++c) px[c] = clip255((px[c] - m) * v + m);
    } else if (op == 3) {
      const float gr = gray(px);
#pragma unroll
      for (int c = 0; c < 3; ++c) px[c] = clip255((px[c] - gr) * v + gr);
    } else {
      adjust_hue(px, v);
    }
  }
}

__global__ __launch_bounds__(kBlock) void aug_finalize_kernel(const float* __restrict__ work,
                                                              const int* __restrict__ ip, float* __restrict__ out,
                                                              int B, int HW, float m0, float m1, float m2, float s0,
                                                              float s1, float s2) {
  const long total = (long)B * HW;
  for (long i = (long)blockIdx.x * kBlock + threadIdx.x; i < total; i += (long)gridDim.x * kBlock) {
    const int b = (int)(i / HW);
    const long p = i - (long)b * HW;
    const bool rnd = ip[b * kAugIParams + 9] != 0;
    const float* px = work + i * 3;
    const float v0 = rnd ? rintf(px[0]) : px[0], v1 = rnd ? rintf(px[1]) : px[1], v2 = rnd ? rintf(px[2]) : px[2];
    float* o = out + (long)b * 3 * HW + p;
    o[0] = (v0 - m0) / s0;
    o[HW] = (v1 - m1) / s1;
    o[2 * (long)HW] = (v2 - m2) / s2;
  }
}
}  // namespace

void aug_geometry(const uint8_t* images, const uint8_t* masks, const int64_t* meta, const int* ip, float* work,
                  int64_t* mask_out, int B, int CH, int CW, hipStream_t s) {
  hipLaunchKernelGGL(aug_geometry_kernel, dim3(grid_for((long)B * CH * CW)), dim3(kBlock), 0, s, images, masks, meta,
                     ip, work, mask_out, B, CH, CW);
}

int aug_gray_scratch_doubles(int B) { return B * kGraySlices; }

void aug_gray_mean(const float* work, float* mean, double* part, int B, int HW, hipStream_t s) {
  hipLaunchKernelGGL(aug_gray_partial_kernel, dim3(kGraySlices, B), dim3(kBlock), 0, s, work, part, HW);
  hipLaunchKernelGGL(aug_gray_final_kernel, dim3((B + kBlock - 1) / kBlock), dim3(kBlock), 0, s, part, mean, B, HW);
}

void aug_color(float* work, const int* ip, const float* fp, const float* mean, int B, int HW, int stage,
               hipStream_t s) {
  hipLaunchKernelGGL(aug_color_kernel, dim3(grid_for((long)B * HW)), dim3(kBlock), 0, s, work, ip, fp, mean, B, HW,
                     stage);
}

void aug_finalize(const float* work, const int* ip, float* out, int B, int HW, const float* mean3, const float* std3,
                  hipStream_t s) {
  hipLaunchKernelGGL(aug_finalize_kernel, dim3(grid_for((long)B * HW)), dim3(kBlock), 0, s, work, ip, out, B, HW,
                     mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2]);
}
