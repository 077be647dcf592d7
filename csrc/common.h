// Shared device helpers for the MI355X (gfx950 / CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//   * Feature maps are NHWC bf16 with the channel dim padded to a multiple of 8 ("Cp"), so one
//     16-byte vector = 8 channels of one pixel and every vector access is 16-B aligned.  Padded
//     channels always hold +0.0 (producers write zeros there), so consumers may read them freely.
//   * bf16 is carried as raw uint16_t bits on the device side; math is fp32.
//   * Wave size is 64 (CDNA).  Block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

#define DEVI __device__ __forceinline__

DEVI float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// fp32 -> bf16, round-to-nearest-even, NaN preserved: the compiler emits v_cvt_pk_bf16_f32.
DEVI uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
DEVI uint32_t pack2(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

DEVI void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

DEVI uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

DEVI bf16x8_t as_bf16x8(const uint4& v) {
  union { uint4 u; bf16x8_t b; } c; c.u = v; return c.b;
}

DEVI f32x4_t mfma16x16x32(const uint4& a, const uint4& b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a), as_bf16x8(b), c, 0, 0, 0);
}

DEVI void load8f(const float* p, float* d) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

// Deferred BatchNorm(+ReLU) applied by a CONSUMER while it loads 8 channels [c, c+8) of an input
// ("BN prologue"): z = act(scale*y + shift) with scale = coef[c..], shift = coef[ld + c..] (the BN's
// [4][Cp] stats rows 0 and 1; ld = Cp).  Rounded to bf16 exactly like a materialised z, so consumers
// see bit-identical inputs.  Padded channels carry scale = shift = 0 -> 0.  Callers apply it only to
// in-image pixels (zero padding of a conv stays 0 in z space).
DEVI uint4 xform8(const uint4& v, const float* coef, int ld, int c, bool relu) {
  float f[8], s[8], h[8];
  unpack8(v, f);
  load8f(coef + c, s);
  load8f(coef + ld + c, h);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float o = fmaf(f[e], s[e], h[e]);
    f[e] = relu ? fmaxf(o, 0.f) : o;
  }
  return pack8(f);
}

// the same with the channel coefficients already in registers
DEVI uint4 affine8(const uint4& v, const float* s, const float* h, bool relu) {
  float f[8];
  unpack8(v, f);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float o = fmaf(f[e], s[e], h[e]);
    f[e] = relu ? fmaxf(o, 0.f) : o;
  }
  return pack8(f);
}

// BatchNorm(+ReLU) backward apply on 8 channels: dy = k1 * dzr + k2 * y + k3 with dzr = dz where
// scale*y + shift > 0 (or everywhere: shift = +inf for a BN without ReLU), else 0.  ONE definition for
// bn_act_bwd_apply and the conv staging prologues, so the deferred and the materialised dy are
// bit-identical.  t = [5][ld] table (scale, shift, k1, k2, k3) at the 8 channels.
DEVI float bwd1(float d, float v, float sc, float sh, float k1, float k2, float k3) {
  const float gr = fmaf(v, sc, sh) > 0.f ? d : 0.f;
  return fmaf(k1, gr, fmaf(k2, v, k3));
}

DEVI uint4 bwd8(const uint4& dz, const uint4& yv, const float* t, int ld) {
  float d[8], v[8];
  unpack8(dz, d);
  unpack8(yv, v);
#pragma unroll
  for (int e = 0; e < 8; ++e) d[e] = bwd1(d[e], v[e], t[e], t[ld + e], t[2 * ld + e], t[3 * ld + e], t[4 * ld + e]);
  return pack8(d);
}

DEVI float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over the 16 lanes of a DPP row (lanes 16r..16r+15): four v_add_f32_dpp row_ror, every lane
// of the row ends with the total.  The MFMA 16x16 D layout keeps one output column per lane & 15.
DEVI float row16_sum(float x) {
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x128, 0xf, 0xf, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x124, 0xf, 0xf, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x122, 0xf, 0xf, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x121, 0xf, 0xf, false));
  return x;
}

// n / d for 0 <= n < 2^22 via a host-precomputed fp32 reciprocal (one multiply + one fix-up) instead
// of the ~30-instruction integer division sequence; exact in that range.
DEVI int fdiv(int n, int d, float inv) {
  int q = (int)((float)n * inv);
  const int r = n - __mul24(q, d);
  q += (r >= d) - (r < 0);
  return q;
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
