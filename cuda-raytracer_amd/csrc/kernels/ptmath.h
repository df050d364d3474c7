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

// ---- correctly rounded sqrt / reciprocal in a bounded range ----------------------
// The compiler's IEEE sqrtf is 16 instructions -- v_sqrt_f32
// (within one ulp), the choice among s - ulp, s, s + ulp by the signs of two
// fma residuals, plus a 2^32 pre-scaling of inputs below 2^-96 (where
// v_sqrt_f32 loses accuracy) and a special-case select.  sqrt_rn keeps the
// residual choice only: the same bits for x = 0, +inf, NaN and every x >=
// 2^-96.  It is used only where the argument is provably 0 or >= 2^-96 (a
// squared length of a near-unit vector, 1 - z^2 of a 24-bit uniform), or
// where a tiny argument's result is discarded (a light sample closer than
// 1e-2); the oracle takes IEEE sqrtf everywhere.  (Round 4: CBempty +3.5 %
// with sqrt_rn / rcp_rn against sqrtf and 1.0f / b.)
__device__ __forceinline__ float sqrt_rn(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
  const float r = rm <= 0.0f ? sm : s;
  return rp > 0.0f ? sp : r;
}
// 1 / b for a normal b in [2^-100, 2^100] (a length): the IEEE quotient's
// reciprocal-and-correction sequence without its range scaling and fixup
// (trace.hip div_rn, the same 8-instruction form)
__device__ __forceinline__ float rcp_rn(float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float e = __builtin_fmaf(-b, y0, 1.0f);
  const float y1 = __builtin_fmaf(e, y0, y0);
  const float r0 = __builtin_fmaf(-b, y1, 1.0f);
  const float q1 = __builtin_fmaf(r0, y1, y1);
  const float r1 = __builtin_fmaf(-b, q1, 1.0f);
  return __builtin_fmaf(r1, y1, q1);
}
// normalize for |a|^2 in [2^-96, 2^126] (directions, unit-normal blends):
// bit-identical to normalize
__device__ __forceinline__ f3 normalize_u(f3 a) {
  const float inv = rcp_rn(sqrt_rn(dot(a, a)));
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
// The seed-dependent round keys k0 + r 0x9E3779B9 are recomputed (one s_add
// each, an empty asm on k0) at every call instead of being hoisted out of the
// path loop as ten loop-invariant SGPRs, which the register allocator then
// spills to VGPR lanes (a v_readlane per round): CBempty +1 %, CBspheres +6 %.
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
    asm volatile("" : "+s"(k0));
    k1 += 0xBB67AE85u;
  }
  return c;
}
// uniform in [0,1): top 24 bits, exact in fp32, scaled by 2^-24 as
// v_ldexp_f32 (the same value as a multiply: an integer below 2^24 scaled by
// a power of two), so no VGPR holds the 2^-24 constant for packed multiplies
__device__ __forceinline__ float u01(uint32_t v) { return __builtin_ldexpf((float)(v >> 8), -24); }

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
  // Horner steps as FMAs (one instruction each)
  float sp = -2.50521084e-08f;
  sp = __builtin_fmaf(sp, t2, 2.75573192e-06f);
  sp = __builtin_fmaf(sp, t2, -1.98412698e-04f);
  sp = __builtin_fmaf(sp, t2, 8.33333333e-03f);
  sp = __builtin_fmaf(sp, t2, -1.66666667e-01f);
  sp = __builtin_fmaf(sp, t2, 1.0f);
  float sn = sp * th;
  float cp = 2.08767570e-09f;
  cp = __builtin_fmaf(cp, t2, -2.75573192e-07f);
  cp = __builtin_fmaf(cp, t2, 2.48015873e-05f);
  cp = __builtin_fmaf(cp, t2, -1.38888889e-03f);
  cp = __builtin_fmaf(cp, t2, 4.16666667e-02f);
  cp = __builtin_fmaf(cp, t2, -0.5f);
  cp = __builtin_fmaf(cp, t2, 1.0f);
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
