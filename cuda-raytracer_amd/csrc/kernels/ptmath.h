// Device-side fp32 math of the path tracer (gfx950).
//
// Every function here has a fixed operation order.  The translation unit is
// compiled with -ffp-contract=off and IEEE division / square root (hipcc's
// default correctly-rounded fp32 div/sqrt), so results are bit-reproducible and
// equal to any restatement that follows the same order (oracle/ptoracle.c).
// FMA is used only where it is written explicitly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pt {

struct f3 {
  float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 mulv(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
// dot and cross products are FMA chains (nvcc's default contraction of the
// reference's cuda_util.h expressions); the oracle spells them the same way
__device__ __forceinline__ float dot(f3 a, f3 b) { return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
  return mk(__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
            __builtin_fmaf(a.x, b.y, -(a.y * b.x)));
}
__device__ __forceinline__ float length(f3 a) { return sqrtf(dot(a, a)); }
// v * (1 / |v|)
__device__ __forceinline__ f3 normalize(f3 a) {
  float inv = 1.0f / sqrtf(dot(a, a));
  return a * inv;
}

// ---- division by a run-time constant -------------------------------------------
// floor(n / d) = (n * m) >> s for every n < 2^30 (m, s from udiv_make): with
// s = 30 + ceil(log2 d) and m = ceil(2^s / d), e = m d - 2^s < d, so n e < 2^s.
struct udiv {
  uint32_t m, s;
};
__host__ __device__ inline udiv udiv_make(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint32_t s = 30 + l;
  return udiv{(uint32_t)(((1ull << s) + d - 1) / d), s};
}
__device__ __forceinline__ uint32_t udiv_q(uint32_t n, udiv d) {
  return (uint32_t)(((unsigned long long)n * d.m) >> d.s);
}

// ---- Philox4x32-10 (Salmon et al., SC'11) ------------------------------------
struct u4 {
  uint32_t x, y, z, w;
};
// M64: each 32x32 -> 64-bit product as one v_mad_u64_u32 instead of
// v_mul_hi_u32 + v_mul_lo_u32 (same bits; faster, but 4 more VGPRs live)
template <bool M64 = false>
__device__ __forceinline__ u4 philox(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    if constexpr (M64) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
      hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
      hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    } else {
      hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
      hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    }
    c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
// uniform in [0,1): top 24 bits, exact in fp32.  PT_U01_LDEXP: the scaling by
// 2^-24 as v_ldexp_f32 (the same value: an integer below 2^24 scaled by a
// power of two), so no VGPR holds the 2^-24 constant for packed multiplies
#ifndef PT_U01_LDEXP
#define PT_U01_LDEXP 1
#endif
__device__ __forceinline__ float u01(uint32_t v) {
  if (PT_U01_LDEXP) return __builtin_ldexpf((float)(v >> 8), -24);
  return (float)(v >> 8) * (1.0f / 16777216.0f);
}

// Random numbers of one path vertex.  counter = (pixel, sample, 2*vertex+call, 'PT')
template <bool M64 = false>
__device__ __forceinline__ u4 rng(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t vertex,
                                  uint32_t call) {
  return philox<M64>(u4{pixel, sample, vertex * 2u + call, 0x50540000u}, seed, 0x2545F491u);
}

// The second NEE sample of a vertex under the reference schedule: its own
// stream (last counter word 'PT'+1), so it never aliases another vertex's.
template <bool M64 = false>
__device__ __forceinline__ u4 rng_nee2(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t vertex) {
  return philox<M64>(u4{pixel, sample, vertex * 2u, 0x50540001u}, seed, 0x2545F491u);
}

// sin and cos of 2*pi*u for u in [0,1): quadrant reduction on u (exact), then
// Taylor polynomials on [0, pi/2).  Max abs error < 2e-7.
__device__ __forceinline__ void sincos2pi(float u, float* s, float* c) {
  float x4 = u * 4.0f;
  float q = floorf(x4);
  float f = x4 - q;
  float th = f * 1.57079637f;
  float t2 = th * th;
  float sp = -2.50521084e-08f;
  sp = sp * t2 + 2.75573192e-06f;
  sp = sp * t2 + -1.98412698e-04f;
  sp = sp * t2 + 8.33333333e-03f;
  sp = sp * t2 + -1.66666667e-01f;
  sp = sp * t2 + 1.0f;
  float sn = sp * th;
  float cp = 2.08767570e-09f;
  cp = cp * t2 + -2.75573192e-07f;
  cp = cp * t2 + 2.48015873e-05f;
  cp = cp * t2 + -1.38888889e-03f;
  cp = cp * t2 + 4.16666667e-02f;
  cp = cp * t2 + -0.5f;
  cp = cp * t2 + 1.0f;
  int iq = ((int)q) & 3;
  float rs = sn, rc = cp;
  if (iq == 1) {
    rs = cp;
    rc = -sn;
  } else if (iq == 2) {
    rs = -sn;
    rc = -cp;
  } else if (iq == 3) {
    rs = -cp;
    rc = sn;
  }
  *s = rs;
  *c = rc;
}

}  // namespace pt
