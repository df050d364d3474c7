// Breadth-first 4-wide BVH traversal with dynamic ray scheduling (gfx950).
//
// MI355X-native restatement of the reference hot loop
//   rayIntersectSingle           src/cudaRenderer.cu:846-1297
//   kernelRayIntersectSingle     cu:1304-1310   (root pass)
//   kernelScanCounts             cu:1317-1431   (per-level scan)
//   kernelRayIntersectLevel      cu:1435-1489   (per-level pass)
//   kernelMergeIntersections     cu:515-540     (closest-hit min reduction)
//   sharedMemExclusiveScan       src/exclusiveScan.cu_inl:52-110
//
// What is kept: level-synchronous traversal, one ray queue per BVH node,
// per-workgroup compaction of the rays that hit each child box, one atomic
// slot reservation per workgroup per child, child queue capacity = parent's
// ray count (cu:922, 1384), all triangles of a leaf tested per ray.
//
// What is MI355X-first:
//  * queues carry 4-byte ray ids; each ray lives once in a 32-byte record
//    (o, d, and its closest-hit word) instead of 128-byte CuRay copies per
//    queue entry;
//  * compaction = wave64 ballot + mbcnt, cross-wave offsets through LDS
//    (replaces the warp-32 Hillis-Steele scan, exclusiveScan.cu_inl:31-48);
//  * an item is 1024 rays (256 threads x 4), so one atomic reserves up to 1024
//    slots; queues and counters are split into 8 lanes (one per XCD under the
//    observed round-robin dispatch) so top-level nodes see 8x less atomic
//    contention; a ray's lane is fixed by its root item;
//  * the closest hit is ONE 64-bit atomicMin on the record's {fp32 bits of t,
//    prim index} word per ray and leaf: order independent, ties go to the
//    lowest sorted prim index, no 16-slot candidate buffer and no merge kernel;
//    its t doubles as the ray's tmax, so every later box test culls against
//    the closest hit found so far;
//  * per-level work ranges are computed on the device (no D2H per level,
//    cu:2237); the level kernel is a grid-stride loop over items;
//  * node and primitive records are wave-uniform and read with scalar loads.
#include "trace.h"

namespace pt {

// ---- primitive records and tests ------------------------------------------------
//
// Device primitive records (built by pt_load_scene from the pt_api.h pt_prim
// format).  Default arithmetic: PREC = 4 float4 per primitive --
//   triangle: rows U, V, W of its Baldwin-Weber transform (Baldwin & Weber,
//     JCGT 5(3) 2016): the affine map taking world space to the triangle's
//     barycentric frame (v0 -> 0, v1 -> (1,0,0), v2 -> (0,1,0), the plane to
//     w = 0), computed in double from the fp32 vertices, stored as fp32 rows
//     {a, b, c, d} (value = a x + b y + c z + d), then {meta, 0, 0, 0};
//   sphere: {centre, 0}, {radius, radius^2, 0, 0}, 0, {meta, 0, 0, 0}.
// The ray's plane hit is t = -W(o) / W(d) and it hits the triangle iff
// u = U(o) + t U(d) >= 0, v = V(o) + t V(d) >= 0 and u + v <= 1 -- the
// reference's plane hit + inside test (intersectRayTriangle, cu:217-270) in
// 6 multiply-adds fewer per test than its per-ray edge cross products, and
// no vertex data.  PT_FLAG_REF_ARITH (REFA): 6 float4 per primitive, the
// reference's literal operands (ref_prim_records) and test (tri_test).
// Dot products and FMA chains: dot(a, b) = fma(a.z, b.z, fma(a.y, b.y,
// a.x * b.x)) (what nvcc makes of the reference's expressions under its
// default --fmad=true); the oracle (ptoracle.c) spells every one with fmaf.
// Tests return t >= 0 or -1 on a miss; t = -0 is returned as +0 so that the
// {t bits, id} key orders correctly.
__device__ __forceinline__ float fdot(float ax, float ay, float az, float bx, float by, float bz) {
  return __builtin_fmaf(az, bz, __builtin_fmaf(ay, by, ax * bx));
}
template <bool REFA>
constexpr int prim_stride() {
  return REFA ? 6 : 4;
}
struct Prim {
  float4 q0, q1, q2, q3, q4, q5;  // (q4, q5: REFA records only)
};
// a primitive's record in SGPRs, one scalar round trip (the empty use pins
// every load above the sphere/triangle branch; the compiler would otherwise
// wait on the meta word before issuing the rest)
template <bool REFA>
__device__ __forceinline__ Prim load_prim(const CPTR(f4v) P) {
  Prim r;
  r.q0 = f4(P[0]);
  r.q1 = f4(P[1]);
  r.q2 = f4(P[2]);
  r.q3 = f4(P[3]);
  if constexpr (REFA) {
    r.q4 = f4(P[4]);
    r.q5 = f4(P[5]);
    asm volatile("" ::"s"(r.q0.w), "s"(r.q1.x), "s"(r.q2.x), "s"(r.q3.x), "s"(r.q4.x), "s"(r.q5.x));
  } else {
    r.q4 = r.q5 = make_float4(0.f, 0.f, 0.f, 0.f);
    asm volatile("" ::"s"(r.q0.x), "s"(r.q1.x), "s"(r.q2.x), "s"(r.q3.x));
  }
  return r;
}
// two consecutive records (default arithmetic) in one scalar round trip
__device__ __forceinline__ void load_prim_pair(const CPTR(f4v) P, Prim& a, Prim& b) {
  a.q0 = f4(P[0]);
  a.q1 = f4(P[1]);
  a.q2 = f4(P[2]);
  a.q3 = f4(P[3]);
  b.q0 = f4(P[4]);
  b.q1 = f4(P[5]);
  b.q2 = f4(P[6]);
  b.q3 = f4(P[7]);
  a.q4 = a.q5 = b.q4 = b.q5 = make_float4(0.f, 0.f, 0.f, 0.f);
  asm volatile("" ::"s"(a.q0.x), "s"(a.q1.x), "s"(a.q2.x), "s"(a.q3.x), "s"(b.q0.x), "s"(b.q1.x), "s"(b.q2.x),
               "s"(b.q3.x));
}
template <bool REFA>
__device__ __forceinline__ bool prim_sphere(const Prim& q) {
  return !REFA && (__float_as_uint(q.q3.x) >> 28) == PT_PRIM_SPHERE;
}
// Baldwin-Weber triangle test (default arithmetic): one branch after the
// plane hit (a wave skips the inside test when no lane has t in [tlo, tbest]),
// the inside test predicated.  A ray parallel to the plane has t = +-inf or
// NaN and misses.
// t = num / den of the Baldwin-Weber test: the compiler's IEEE
// division sequence (reciprocal, one refinement, quotient, two residual
// corrections) without its range scaling (v_div_scale x 2) and special-case
// fixup (v_div_fixup): 8 instead of 11 instructions and the same bits wherever
// the scaling is the identity -- both operands and the quotient in the normal
// range, away from the extremes.  Outside it (|den| denormal or zero, an
// overflowing quotient: a ray parallel to the plane) the result is NaN, an
// infinity or a huge t, and the test misses as it does for the IEEE quotient
// (|u| or |v| huge, or unordered).  The residuals r0, r1 are ~2^-24 |num|:
// for |num| below ~2^-101 they are subnormal and the quotient may differ
// from IEEE's by one ulp -- a t below ~2^-96 at a unit ray (an origin on the
// plane to 29 decimal places).  The oracle divides with IEEE `/`; the GPU
// parity tests check the two agree, tests/test_gpu_regress.py checks the
// division itself down to |num| = 2^-100 bit for bit and to 2^-126 within
// one ulp.  (Round 3: CBempty +1.5-3 %, the wavefront scenes +1.2-1.5 %.)
__device__ __forceinline__ float div_rn(float a, float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float e = __builtin_fmaf(-b, y0, 1.0f);
  const float y1 = __builtin_fmaf(e, y0, y0);
  const float q0 = a * y1;
  const float r0 = __builtin_fmaf(-b, q0, a);
  const float q1 = __builtin_fmaf(r0, y1, q0);
  const float r1 = __builtin_fmaf(-b, q1, a);
  return __builtin_fmaf(r1, y1, q1);
}
// pt_check_division: div_rn over host-given pairs
// pt_check_fast_math: every fp32 bit pattern x in [lo, hi) through sqrt_rn
// (which = 0) or rcp_rn (which = 1) against the compiler's IEEE sqrtf / 1 / x;
// out[0] += mismatches, out[1] = min mismatching pattern (zeroed / 0xFFFFFFFF by
// the host)
__global__ __launch_bounds__(TPB) void k_check_fast_math(int which, uint32_t lo, uint32_t hi, unsigned int* out) {
  uint32_t bad = 0, first = 0xFFFFFFFFu;
  for (uint64_t b = (uint64_t)lo + (uint64_t)blockIdx.x * TPB + threadIdx.x; b < hi; b += (uint64_t)gridDim.x * TPB) {
    const float x = __uint_as_float((uint32_t)b);
    const float f = which == 0 ? sqrt_rn(x) : rcp_rn(x);
    const float r = which == 0 ? sqrtf(x) : 1.0f / x;
    if (__float_as_uint(f) != __float_as_uint(r)) {
      ++bad;
      first = min(first, (uint32_t)b);
    }
  }
  if (bad) {
    atomicAdd(out, bad);
    atomicMin(out + 1, first);
  }
}

__global__ __launch_bounds__(TPB) void k_check_division(const float* __restrict__ a, const float* __restrict__ b,
                                                        float* __restrict__ q, uint32_t n) {
  const uint32_t i = blockIdx.x * TPB + threadIdx.x;
  if (i < n) q[i] = div_rn(a[i], b[i]);
}
__device__ __forceinline__ float bw_plane(const f3 o, const float4 W) {
  return __builtin_fmaf(W.z, o.z, __builtin_fmaf(W.y, o.y, __builtin_fmaf(W.x, o.x, W.w)));
}
// STRICT: a hit needs t < tbest (the caller's best so far, no hit yet at
// tbest = +inf, which no hit reaches): then every hit returned is a new best
// u and v from the hit point, the oracle's form (round 4: 9 FMAs for both
// instead of 14 for U(o) + t U.d and V(o) + t V.d; CBempty +5.4 %)
// ZFIX: a hit at t = -0 is returned as +0 (the {prim, t} keys order t by its
// bits); false where t only feeds comparisons and the hit point
template <bool STRICT = false, bool ZFIX = true>
__device__ __forceinline__ float bw_test(const f3 o, const f3 d, const float4 U, const float4 V, const float4 W,
                                         float tbest, float tlo = 0.0f) {
  const float t = div_rn(-bw_plane(o, W), fdot(W.x, W.y, W.z, d.x, d.y, d.z));
  if (!(t >= tlo) | (STRICT ? !(t < tbest) : (t > tbest))) return -1.0f;
  // barycentrics of the plane hit P = o + t d: U(P), V(P)
  const f3 P = mk(__builtin_fmaf(t, d.x, o.x), __builtin_fmaf(t, d.y, o.y), __builtin_fmaf(t, d.z, o.z));
  const float u = bw_plane(P, U), v = bw_plane(P, V);
  // (unordered compares: a NaN u or v -- a ray parallel to the plane, t =
  // +-inf -- is a miss)
  const bool miss = !(u >= 0.0f) | !(v >= 0.0f) | !(u + v <= 1.0f);
  return miss ? -1.0f : (ZFIX ? t + 0.0f : t);  // (t + 0 maps -0 to +0)
}
// PT_FLAG_REF_ARITH (REFA): the literal edge test of cu:251-267,
// dot(N, cross(e_k, P - v_k)) < 0, on the reference-arithmetic primitive
// records (pt_ctx::d_prims_ref): the edge-normal slots hold the edges
// e0 = v1 - v0, e1 = v2 - v1, e2 = v0 - v2 and q3 / q1.w hold
// N = cross(v1 - v0, v2 - v0) and dot(N, v0) in this file's FMA-chain
// arithmetic (cu:223-237).  The parallel test |N.d| < 1e-6 is a double
// comparison in the reference (1e-6 is a double literal): for an fp32 x,
// x < 1e-6 holds exactly when x <= 1e-6f.
__device__ __forceinline__ float edge_ref(const float4 N, float ex, float ey, float ez, const f3 P, const float4 v) {
  const f3 C = cross(mk(ex, ey, ez), mk(P.x - v.x, P.y - v.y, P.z - v.z));
  return fdot(N.x, N.y, N.z, C.x, C.y, C.z);
}
// The reference's literal test (REFA records): plane hit, then the three edge
// tests dot(N, cross(e_k, P - v_k)) < 0 (cu:223-267).
template <bool STRICT = false>
__device__ __forceinline__ float tri_test_ref(const f3 o, const f3 d, const float4 q0, const float4 q1,
                                              const float4 q2, const float4 q3, const float4 q4, const float4 q5,
                                              const float tbest, const float tlo = 0.0f) {
  float ndd = fdot(q3.x, q3.y, q3.z, d.x, d.y, d.z);
  if (fabsf(ndd) <= 1e-6f) return -1.0f;
  float t = (q1.w - fdot(q3.x, q3.y, q3.z, o.x, o.y, o.z)) / ndd;
  // t > tbest cannot win (ties need t == tbest): skip the edge tests; hits
  // before the ray's t_min (tlo >= 0, pt_intersect) do not count
  if (t < tlo || (STRICT ? !(t < tbest) : (t > tbest))) return -1.0f;
  f3 P = mk(__builtin_fmaf(t, d.x, o.x), __builtin_fmaf(t, d.y, o.y), __builtin_fmaf(t, d.z, o.z));
  if (edge_ref(q3, q2.w, q3.w, q4.w, P, q0) < 0.0f) return -1.0f;
  if (edge_ref(q3, q4.x, q4.y, q4.z, P, q1) < 0.0f) return -1.0f;
  if (edge_ref(q3, q5.x, q5.y, q5.z, P, q2) < 0.0f) return -1.0f;
  return t == 0.0f ? 0.0f : t;
}
// A triangle's closest-hit test in the record's arithmetic.
// The U and V rows of a Baldwin-Weber record.  The record holds them
// interleaved, {Ux, Vx, Uy, Vy}{Uz, Vz, Uw, Vw}{W} (bw_prim_records), so the
// packed u / v evaluation (v_pk_fma_f32 with an SGPR pair operand) reads each
// (U_k, V_k) pair straight from the record's SGPRs instead of copying them
// into place (6 s_mov per primitive; round 4, +1-2 % on the single-leaf scenes)
__device__ __forceinline__ void bw_uv(const Prim& q, float4& U, float4& V) {
  U = make_float4(q.q0.x, q.q0.z, q.q1.x, q.q1.z);
  V = make_float4(q.q0.y, q.q0.w, q.q1.y, q.q1.w);
}
template <bool REFA, bool STRICT = false, bool ZFIX = true>
__device__ __forceinline__ float tri_test(const f3 o, const f3 d, const Prim& q, float tbest, float tlo = 0.0f) {
  if constexpr (REFA) {
    return tri_test_ref<STRICT>(o, d, q.q0, q.q1, q.q2, q.q3, q.q4, q.q5, tbest, tlo);
  } else {
    float4 U, V;
    bw_uv(q, U, V);
    return bw_test<STRICT, ZFIX>(o, d, U, V, q.q2, tbest, tlo);
  }
}
// Closest-hit update form of the strict Baldwin-Weber test (default
// arithmetic, tlo = 0): where tri_test<false, true>(o, d, q, bt) would return
// t >= 0, bt = t and bp = idx (a -0 t is kept: for callers whose t only feeds
// compares and the hit point)
__device__ __forceinline__ void bw_closest_update(const f3 o, const f3 d, const Prim& q, int idx, float& bt, int& bp) {
  float4 U, V;
  bw_uv(q, U, V);
  const float4 W = q.q2;
  const float t = div_rn(-bw_plane(o, W), fdot(W.x, W.y, W.z, d.x, d.y, d.z));
  if (!(t >= 0.0f) | !(t < bt)) return;
  const f3 P = mk(__builtin_fmaf(t, d.x, o.x), __builtin_fmaf(t, d.y, o.y), __builtin_fmaf(t, d.z, o.z));
  const float u = bw_plane(P, U), v = bw_plane(P, V);
  const bool take = (u >= 0.0f) & (v >= 0.0f) & (u + v <= 1.0f);
  bt = take ? t : bt;
  bp = take ? idx : bp;
}
// Occlusion form of the Baldwin-Weber test (default arithmetic): true iff
// tri_test(o, d, q, tmax) would return a t in [0, tmax], from the pre-test's
// num and ndd (the same expressions bw_test evaluates, so the same bits)
__device__ __forceinline__ bool bw_occludes(const f3 o, const f3 d, const Prim& q, float num, float ndd, float tmax) {
  float4 U, V;
  bw_uv(q, U, V);
  const float t = div_rn(num, ndd);
  if (!(t >= 0.0f) | (t > tmax)) return false;
  const f3 P = mk(__builtin_fmaf(t, d.x, o.x), __builtin_fmaf(t, d.y, o.y), __builtin_fmaf(t, d.z, o.z));
  const float u = bw_plane(P, U), v = bw_plane(P, V);
  return (u >= 0.0f) & (v >= 0.0f) & (u + v <= 1.0f);
}
// The plane hit as t = num / ndd, for the division-free pre-test.
template <bool REFA>
__device__ __forceinline__ void plane_nd(const f3 o, const f3 d, const Prim& q, float& ndd, float& num) {
  if constexpr (REFA) {
    ndd = fdot(q.q3.x, q.q3.y, q.q3.z, d.x, d.y, d.z);
    num = q.q1.w - fdot(q.q3.x, q.q3.y, q.q3.z, o.x, o.y, o.z);
  } else {
    ndd = fdot(q.q2.x, q.q2.y, q.q2.z, d.x, d.y, d.z);
    num = -bw_plane(o, q.q2);
  }
}

// Division-free early rejection: true only when the plane hit of tri_test is
// certainly outside [0, tmax] (its rounded t = num / ndd is < 0 or > tmax) or
// |ndd| < 1e-6.  Lanes for which it is false run the exact test; a wave whose
// lanes all reject skips the division and the edge tests.
//  * signs differ, 2^-60 < |num|, |ndd| < 2^60: |q| > 2^-120, so t < 0;
//  * same signs, tmax >= 2^-60: x = RN(RN(tmax |ndd|) (1 + 2^-20)) exceeds
//    tmax |ndd| (1 + 2^-21), so |num| > x gives q > tmax (1 + 2^-21), which
//    rounds above tmax (tmax = inf never rejects).
// (FLAT: the test rejects |ndd| <= 1e-6 as parallel, REFA; the Baldwin-Weber
// test has no such rejection)
template <bool FLAT = true>
__device__ __forceinline__ bool tri_outside(float ndd, float num, float tmax) {
  const float an = fabsf(num), ad = fabsf(ndd);
  const bool flat = FLAT && ad <= 1e-6f;
  const bool behind = ((num < 0.0f) != (ndd < 0.0f)) & (an > 0x1p-60f) & (ad < 0x1p60f);
  const bool beyond = ((num < 0.0f) == (ndd < 0.0f)) & (tmax >= 0x1p-60f) & (an > (tmax * ad) * (1.0f + 0x1p-20f));
  return flat | behind | beyond;
}

// Two independent triangle tests at once on packed fp32 (v_pk_fma_f32 /
// v_pk_add_f32): element i is exactly tri_test(o[i], d[i], q..., tbest[i])
// (same operations in the same order, so the same bits), written without
// branches so both halves share every instruction.  Used for two rays against
// one triangle (leaf loops).
typedef float f2v __attribute__((ext_vector_type(2)));
struct f3x2 {
  f2v x, y, z;
};
__device__ __forceinline__ f2v sp(float a) { return f2v{a, a}; }
__device__ __forceinline__ f3x2 sp3(float a, float b, float c) { return f3x2{sp(a), sp(b), sp(c)}; }
__device__ __forceinline__ f3x2 pair3(f3 a, f3 b) { return f3x2{f2v{a.x, b.x}, f2v{a.y, b.y}, f2v{a.z, b.z}}; }
__device__ __forceinline__ f2v fma2(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2v fdot2(const f3x2& a, const f3x2& b) {
  return fma2(a.z, b.z, fma2(a.y, b.y, a.x * b.x));
}

// dot(N, cross(e, P - v)) on two lanes (REFA: edge_ref, element for element)
__device__ __forceinline__ f2v edge_ref2(const f3x2& N, const f3x2& P, const f3x2& v, const f3x2& e) {
  const f3x2 w{P.x - v.x, P.y - v.y, P.z - v.z};
  const f3x2 C{fma2(e.y, w.z, -(e.z * w.y)), fma2(e.z, w.x, -(e.x * w.z)), fma2(e.x, w.y, -(e.y * w.x))};
  return fdot2(N, C);
}

// REFA: N normal, pd plane offset, v0..v2 vertices, e0..e2 edges (the
// reference's operands, tri_test_ref); element i is tri_test_ref of ray i
template <bool STRICT = false>
__device__ __forceinline__ f2v tri_test2_ref(const f3x2& o, const f3x2& d, const f3x2& N, f2v pd, const f3x2& v0,
                                             const f3x2& v1, const f3x2& v2, const f3x2& m0, const f3x2& m1,
                                             const f3x2& m2, f2v tbest, f2v tlo = f2v{0.0f, 0.0f}) {
  const f2v ndd = fdot2(N, d);
  const f2v t = (pd - fdot2(N, o)) / ndd;
  const f3x2 P{fma2(t, d.x, o.x), fma2(t, d.y, o.y), fma2(t, d.z, o.z)};
  const f2v s0 = edge_ref2(N, P, v0, m0);
  const f2v s1 = edge_ref2(N, P, v1, m1);
  const f2v s2 = edge_ref2(N, P, v2, m2);
  // t + 0 maps -0 to +0 and leaves every other value unchanged (strict fp:
  // the add is not folded away)
  const f2v tz = t + sp(0.0f);
  f2v r;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    // non-short-circuit: every comparison is one v_cmp, combined on the SALU
    const bool flat = fabsf(ndd[i]) <= 1e-6f;
    const bool beyond = STRICT ? !(t[i] < tbest[i]) : (t[i] > tbest[i]);
    const bool miss = flat | (t[i] < tlo[i]) | beyond | (s0[i] < 0.0f) | (s1[i] < 0.0f) | (s2[i] < 0.0f);
    r[i] = miss ? -1.0f : tz[i];
  }
  return r;
}
// Baldwin-Weber on two rays (element i is bw_test of ray i, branch-free)
__device__ __forceinline__ f2v bw_plane2(const f3x2& o, const float4 R) {
  return fma2(sp(R.z), o.z, fma2(sp(R.y), o.y, fma2(sp(R.x), o.x, sp(R.w))));
}
template <bool STRICT = false>
__device__ __forceinline__ f2v bw_test2(const f3x2& o, const f3x2& d, const float4 U, const float4 V, const float4 W,
                                        f2v tbest, f2v tlo) {
  const f2v nm = -bw_plane2(o, W), dn = fdot2(sp3(W.x, W.y, W.z), d);
  const f2v t = f2v{div_rn(nm[0], dn[0]), div_rn(nm[1], dn[1])};
  const f3x2 P{fma2(t, d.x, o.x), fma2(t, d.y, o.y), fma2(t, d.z, o.z)};
  const f2v u = bw_plane2(P, U), v = bw_plane2(P, V);
  const f2v uv = u + v;
  const f2v tz = t + sp(0.0f);
  f2v r;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const bool beyond = STRICT ? !(t[i] < tbest[i]) : (t[i] > tbest[i]);
    const bool miss = !(t[i] >= tlo[i]) | beyond | !(u[i] >= 0.0f) | !(v[i] >= 0.0f) | !(uv[i] <= 1.0f);
    r[i] = miss ? -1.0f : tz[i];
  }
  return r;
}
// The strict two-ray test with the hit update inside (default arithmetic):
// where tri_test2<false, true> would return t >= 0 for ray i, bt_i = t (-0 as
// +0: the keys order t by its bits) and bp_i = idx (round 4: the level
// kernels' two-ray leaf test +1.1-1.5 % on the wavefront scenes)
__device__ __forceinline__ void bw_update2(const f3x2& o, const f3x2& d, const Prim& q, f2v tlo, int idx, float& bt0,
                                           float& bt1, int& bp0, int& bp1) {
  float4 U, V;
  bw_uv(q, U, V);
  const float4 W = q.q2;
  const f2v nm = -bw_plane2(o, W), dn = fdot2(sp3(W.x, W.y, W.z), d);
  const f2v t = f2v{div_rn(nm[0], dn[0]), div_rn(nm[1], dn[1])};
  const f3x2 P{fma2(t, d.x, o.x), fma2(t, d.y, o.y), fma2(t, d.z, o.z)};
  const f2v u = bw_plane2(P, U), v = bw_plane2(P, V);
  const f2v uv = u + v;
  const f2v tz = t + sp(0.0f);
  const bool take0 = (t[0] >= tlo[0]) & (t[0] < bt0) & (u[0] >= 0.0f) & (v[0] >= 0.0f) & (uv[0] <= 1.0f);
  const bool take1 = (t[1] >= tlo[1]) & (t[1] < bt1) & (u[1] >= 0.0f) & (v[1] >= 0.0f) & (uv[1] <= 1.0f);
  bt0 = take0 ? tz[0] : bt0;
  bp0 = take0 ? idx : bp0;
  bt1 = take1 ? tz[1] : bt1;
  bp1 = take1 ? idx : bp1;
}
// Two rays (pair j, j + 1) against triangle q in the record's arithmetic.
template <bool REFA, bool STRICT = false>
__device__ __forceinline__ f2v tri_test2(const f3x2& o, const f3x2& d, const Prim& q, f2v tbest, f2v tlo) {
  if constexpr (REFA) {
    const float4 q0 = q.q0, q1 = q.q1, q2 = q.q2, q3 = q.q3, q4 = q.q4, q5 = q.q5;
    return tri_test2_ref<STRICT>(o, d, sp3(q3.x, q3.y, q3.z), sp(q1.w), sp3(q0.x, q0.y, q0.z), sp3(q1.x, q1.y, q1.z),
                         sp3(q2.x, q2.y, q2.z), sp3(q2.w, q3.w, q4.w), sp3(q4.x, q4.y, q4.z),
                         sp3(q5.x, q5.y, q5.z), tbest, tlo);
  } else {
    float4 U, V;
    bw_uv(q, U, V);
    return bw_test2<STRICT>(o, d, U, V, q.q2, tbest, tlo);
  }
}

// Closest-hit update of a leaf loop: take t when it is a hit (t >= 0) that
// beats {bt, bp} -- nearer, or as near as the incoming key while this leaf has
// no hit yet (its primitives are tested in increasing index order, so the
// first of equal hits is the lowest).  A lane without a ray has bt < 0 and
// takes nothing.  (As two selects instead of the branch: leaf levels -3 to
// -7 %, CBempty -0.5 %.)
__device__ __forceinline__ void take_hit(float t, int k, float& bt, int& bp) {
  if (t >= 0.0f && (t < bt || (t == bt && bp < 0))) {
    bt = t;
    bp = k;
  }
}

// The strict leaf loops of the level kernels: the running best starts one
// ulp above the ray's tmax (the key's t from the leaves already visited) and
// the triangle tests admit only t below it, so "t <= tmax, and a first hit at
// t == tmax counts" becomes "t < best", every hit the test returns is a new
// best, and the update is a compare and two selects.  The same hits as
// take_hit: equal t within a leaf keeps the lower index (tested first), a
// hit at the incoming tmax still reaches the key's atomicMin (round 4: levels
// +1 %).
__device__ __forceinline__ float next_up(float x) {  // (x >= 0, or negative for an empty lane: unchanged)
  return x >= 0.0f && x < __builtin_inff() ? __uint_as_float(__float_as_uint(x) + 1u) : x;
}
__device__ __forceinline__ void take_strict(float t, int k, float& bt, int& bp) {
  const bool take = (t >= 0.0f) & (t < bt);
  bt = take ? t : bt;
  bp = take ? k : bp;
}

// Ray-sphere (the reference has none: spheres are reinterpret_cast to
// triangles at cu:1760).  Nearest root with t >= tlo (the ray's t_min, >= 0);
// d must be unit length.
__device__ __forceinline__ float sphere_test(const f3 o, const f3 d, const float4 q0, const float4 q1,
                                             const float tlo = 0.0f) {
  f3 oc = mk(o.x - q0.x, o.y - q0.y, o.z - q0.z);
  float b = fdot(oc.x, oc.y, oc.z, d.x, d.y, d.z);
  float cc = fdot(oc.x, oc.y, oc.z, oc.x, oc.y, oc.z) - q1.y;
  float disc = __builtin_fmaf(b, b, -cc);
  if (disc < 0.0f) return -1.0f;
  float sq = sqrtf(disc);
  float t0 = -b - sq;
  float t1 = -b + sq;
  float t = (t0 >= tlo) ? t0 : t1;
  if (t < tlo) return -1.0f;
  return t == 0.0f ? 0.0f : t;
}

// Slab test against one child box.  Conservative replacement of intersectBBox
// (cu:154-207): a box is entered iff its slab interval meets [0, tmax].  Only
// decides which queues a ray enters, never the reported hit.
__device__ __forceinline__ bool box_hit(float bx0, float bx1, float by0, float by1, float bz0, float bz1,
                                        const f3 oi, const f3 inv, float tmax) {
  float tx0 = __builtin_fmaf(bx0, inv.x, -oi.x), tx1 = __builtin_fmaf(bx1, inv.x, -oi.x);
  float ty0 = __builtin_fmaf(by0, inv.y, -oi.y), ty1 = __builtin_fmaf(by1, inv.y, -oi.y);
  float tz0 = __builtin_fmaf(bz0, inv.z, -oi.z), tz1 = __builtin_fmaf(bz1, inv.z, -oi.z);
  float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
  float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
  return tn <= tf;
}

// one axis's two slab distances b * inv - oi, as two v_fma_f32 (in one
// v_pk_fma_f32 instead -- packed fp32 FMAs issue at twice the rate of
// v_fma_f32 on gfx950, 130 against 74 TFLOP/s on independent chains,
// scripts/cal/pk_rate.hip -- the cluster masks of k_path_leaf measured slower:
// CBempty 103,800 -> 100,800 Mrays/s, CBspheres 64,850 -> 62,700, round 5; a
// cluster pair's two triangles on packed fp32 likewise lost: their records
// and the ray's broadcast pairs spilled at 64 VGPRs)
__device__ __forceinline__ f2v slab2(float b0, float b1, float inv, float oi) {
  return f2v{__builtin_fmaf(b0, inv, -oi), __builtin_fmaf(b1, inv, -oi)};
}
// The same test for a ray without a far limit (tmax = +inf: its min is the
// identity here, directions come through safe_dir, so no slab value is NaN)
__device__ __forceinline__ bool box_hit_open(float bx0, float bx1, float by0, float by1, float bz0, float bz1,
                                             const f3 oi, const f3 inv) {
  const f2v tx = slab2(bx0, bx1, inv.x, oi.x), ty = slab2(by0, by1, inv.y, oi.y), tz = slab2(bz0, bz1, inv.z, oi.z);
  float tn = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fmaxf(fminf(tz.x, tz.y), 0.0f));
  float tf = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
  return tn <= tf;
}
// ... and with a far limit as a second compare (tmax not NaN: a shadow
// segment), which keeps tmax out of the per-box min (the compiler re-emits
// its NaN canonicalisation inside the box loop otherwise)
__device__ __forceinline__ bool box_hit_seg(float bx0, float bx1, float by0, float by1, float bz0, float bz1,
                                            const f3 oi, const f3 inv, float tmax) {
  const f2v tx = slab2(bx0, bx1, inv.x, oi.x), ty = slab2(by0, by1, inv.y, oi.y), tz = slab2(bz0, bz1, inv.z, oi.z);
  float tn = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fmaxf(fminf(tz.x, tz.y), 0.0f));
  float tf = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
  return (tn <= tf) & (tn <= tmax);
}
// bit c of a mask from a per-lane condition: v_cndmask + v_lshl_or
__device__ __forceinline__ uint32_t mask_bit(uint32_t m, bool h, int c) { return ((uint32_t)h << c) | m; }

__device__ __forceinline__ float safe_dir(float x) {
  return fabsf(x) < 1e-20f ? copysignf(1e-20f, x) : x;
}

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ---- queue entries ---------------------------------------------------------------
// The root pass pushes 4-byte ray ids (its targets' queues are sized for the
// worst case, every ray in every target).  Below that, queues hold 32-byte ray
// entries {o, d.x}{d.y, d.z, id, tmax}: a level reads its rays as contiguous
// entries (full lines) instead of gathering 32-byte records through ids
// (a 64-128 B memory request each), and pushes copies to the children.  The
// closest-hit key stays in the ray record (atomicMin through id); an entry's
// tmax is the ray's tmax when it was pushed (conservative: it only shrinks).
__device__ __forceinline__ void push_ray(const TraceArgs& A, bool entry, uint32_t e, uint32_t id, const f3 o,
                                         const f3 d, float tmax) {
  PT_CHECK(entry || e < A.dbg_qids, "push id", e, A.dbg_qids);
  PT_CHECK(id < A.dbg_nslots, "push id value", id, A.dbg_nslots);
  if (entry) {
    A.qe[QESTRIDE * (size_t)e] = make_float4(o.x, o.y, o.z, d.x);
    A.qe[QESTRIDE * (size_t)e + 1] = make_float4(d.y, d.z, __uint_as_float(id), tmax);
  } else {
    A.q[e] = id;
  }
}
// Ray e of a level queue: an id (gather from the ray record) or an entry.
__device__ __forceinline__ void load_ray(const TraceArgs& A, bool ids, uint32_t e, uint32_t& id, f3& o, f3& d,
                                         float& tmax) {
  if (ids) {
    id = A.q[e];
    const float4 a = A.ray[RSTRIDE * id], b = A.ray[RSTRIDE * id + 1];
    o = mk(a.x, a.y, a.z);
    d = mk(a.w, b.x, b.y);
    tmax = b.w;
  } else {
    const float4 a = A.qe[QESTRIDE * (size_t)e], b = A.qe[QESTRIDE * (size_t)e + 1];
    o = mk(a.x, a.y, a.z);
    d = mk(a.w, b.x, b.y);
    id = __float_as_uint(b.z);
    tmax = b.w;
  }
}

// ---- push targets ------------------------------------------------------------
// A node's 4 children (level passes), or the root table's targets (root pass).
struct ChildTargets {
  const CPTR(pt_node) nd;
  __device__ __forceinline__ int count() const { return 4; }
  __device__ __forceinline__ void box(const TraceArgs&, int c, float (&b)[6]) const {
    b[0] = nd->bmin_x[c];
    b[1] = nd->bmax_x[c];
    b[2] = nd->bmin_y[c];
    b[3] = nd->bmax_y[c];
    b[4] = nd->bmin_z[c];
    b[5] = nd->bmax_z[c];
  }
  __device__ __forceinline__ int node(const TraceArgs&, int c) const { return nd->child[c]; }
};
struct TableTargets {
  const RootTable& T;
  __device__ __forceinline__ int count() const { return T.nt; }
  __device__ __forceinline__ void box(const TraceArgs&, int c, float (&b)[6]) const {
#pragma unroll
    for (int i = 0; i < 6; ++i) b[i] = T.tb[i][c];
  }
  __device__ __forceinline__ int node(const TraceArgs&, int c) const { return T.tnode[c]; }
};

#ifndef PT_SHADE_TIMING
#define PT_SHADE_TIMING 0
#endif
#if PT_SHADE_TIMING
// diagnostic: thread 0's s_memtime after the root pass's stages (barriers
// without a memory fence added in this build only, so stores in flight do not
// count): inline leaves and record writes issued, target counts, reservations,
// pushes
static __shared__ unsigned long long g_rp_t[6];
#define RP_STAMP(k)              \
  __builtin_amdgcn_s_barrier();  \
  if (threadIdx.x == 0) g_rp_t[k] = __builtin_amdgcn_s_memtime()
__device__ __forceinline__ void g_rp_t_set(int k) { g_rp_t[k] = __builtin_amdgcn_s_memtime(); }
#else
#define RP_STAMP(k)
__device__ __forceinline__ void g_rp_t_set(int) {}
#endif

// Block-wide push of R rays per thread into the queues of up to NC targets in
// queue lane `lane`: slab tests, wave64 ballot compaction, one atomic slot
// reservation per target for the whole workgroup, cross-wave offsets through
// LDS (sh: NC * 8 u32).  Every thread of the workgroup must call it (two
// barriers); rays with valid[j] false push nothing, ray groups j >= nj
// (uniform) are skipped.
template <int R, int NC, class Tg>
__device__ __forceinline__ void push_children(const TraceArgs& A, const Tg& tg, int lane, const uint32_t (&id)[R],
                                              const f3 (&o)[R], const f3 (&d)[R], const float (&tmax)[R],
                                              const bool (&valid)[R], int nj, uint32_t* sh, bool entry) {
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int nt = tg.count();
  uint32_t bits[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    bits[j] = 0;
    if (j >= nj) continue;
    // |d| components below 1e-20 are clamped so 1/d stays finite: the FMA slab
    // form t = b*inv - o*inv would turn an axis-parallel ray (inv = inf) lying
    // inside a slab into inf - inf = NaN and wrongly miss the box
    f3 inv = mk(__builtin_amdgcn_rcpf(safe_dir(d[j].x)), __builtin_amdgcn_rcpf(safe_dir(d[j].y)),
                __builtin_amdgcn_rcpf(safe_dir(d[j].z)));
    f3 oi = mk(o[j].x * inv.x, o[j].y * inv.y, o[j].z * inv.z);
    uint32_t b = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (c >= nt) break;
      float bx[6];
      tg.box(A, c, bx);
      bool h = box_hit(bx[0], bx[1], bx[2], bx[3], bx[4], bx[5], oi, inv, tmax[j]);
      b |= (valid[j] && h) ? (1u << c) : 0u;
    }
    bits[j] = b;
  }
  // per-wave counts per target -> LDS sh[c*4 + wave]; bases -> sh[NC*4 + c*4 + wave]
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c >= nt) break;
    uint32_t wc = 0;
#pragma unroll
    for (int j = 0; j < R; ++j) wc += (uint32_t)__popcll(__ballot((bits[j] >> c) & 1u));
    if ((tid & 63) == 0) sh[c * 4 + wave] = wc;
  }
  __syncthreads();
  if (threadIdx.x == 0 && PT_SHADE_TIMING) g_rp_t_set(2);
  if (tid < nt) {
    const int c = tid;
    const int child = tg.node(A, c);
    uint32_t w0 = sh[c * 4 + 0], w1 = sh[c * 4 + 1], w2 = sh[c * 4 + 2], w3 = sh[c * 4 + 3];
    uint32_t tot = w0 + w1 + w2 + w3;
    uint32_t b = 0;
    // the queue's absolute offset is read here, in the round trip of the
    // reservation, and folded into the bases (not after the barrier below)
    if (child >= 0 && tot) b = atomicAdd(A.cnt + cnt_idx(child, lane), tot) + A.qoff[(size_t)child * NLANE + lane];
    sh[NC * 4 + c * 4 + 0] = b;
    sh[NC * 4 + c * 4 + 1] = b + w0;
    sh[NC * 4 + c * 4 + 2] = b + w0 + w1;
    sh[NC * 4 + c * 4 + 3] = b + w0 + w1 + w2;
  }
  __syncthreads();
  if (threadIdx.x == 0 && PT_SHADE_TIMING) g_rp_t_set(3);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c >= nt) break;
    const int child = tg.node(A, c);
    if (child < 0) continue;
    uint32_t off = sh[NC * 4 + c * 4 + wave];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const bool h = (bits[j] >> c) & 1u;
      const unsigned long long m = __ballot(h);
      if (h) push_ray(A, entry, off + mbcnt64(m), id[j], o[j], d[j], tmax[j]);
      off += (uint32_t)__popcll(m);
    }
  }
}

// Root pass of R rays per thread (every thread of the workgroup calls it):
//  1. the inline leaves of the root table, when the ray enters their box:
//     closest hit with the leaf rules of process_item (ties to the lowest
//     primitive) -- it becomes the ray's initial key {prim, t} and its tmax;
//  2. the record {o, d.x}{d.y, d.z, prim, t} of every valid ray is written
//     here (the callers write the empty r1 of invalid slots);
//  3. a shadow ray (anyhit) occluded by an inline leaf is done: not queued;
//     the others are pushed into the targets' queues with the tightened tmax.
// (The hit update as selects measured slower: CBbunny -2.4 %, dragon proxy
// -0.6 %, round 4; a division-free pre-test for extension rays too: CBbunny
// shade +3.7 ms, round 4.)
// Candidate clusters: an extension ray (closest hit) tests the inline leaves'
// primitive clusters (RootTable::nc: host-built, guard-banded boxes as
// conservative as the BVH's) only where it enters the cluster's box, each lane
// its own candidates (the member records staged in LDS by the caller: lrec,
// linfo = RootTable::cmem (REFA: cmem_ref), cinfo; CL callers only).  The hit taken is
// the lowest (t, primitive) over the primitives tested, which is the same over
// any set that holds every primitive the ray hits: the leaf loop's result.
// Shadow rays likewise (box tests over their segment, the pre-test on the
// candidates, done at the first hit; RootTable::nc_shadow = 0 gives them the
// leaf loop).  CBbunny's 18 inline primitives form 7 clusters (a wall's two
// triangles, the light's two, the 6 bunny triangles that share a leaf with the
// walls): the inline-leaf phase of a shade workgroup-pass 24,900 -> 11,150
// cycles (extension rays 13,900 -> 6,300; PT_SHADE_TIMING), CBbunny 122 ->
// 114.7 ms per frame, dragon proxy +0.5 %; uncached vector loads of the
// records instead of LDS lost 2,000 cycles in that phase (the dependent
// round trips per candidate).  Shadow rays pick their candidates by the slab
// test too: the segment-box overlap k_path_leaf uses (shade.hip
// leaf_occluded_aabb) measured CBbunny 112.35 -> 113.2 ms per frame, the
// dragon proxy unchanged (the root pass computes the slab test's reciprocals
// for its target boxes anyway).
template <int R, bool REFA = false, bool TMIN = false, bool CL = false>
__device__ __forceinline__ void root_pass(const TraceArgs& A, const RootTable& T, int lane, const uint32_t (&id)[R],
                                          const f3 (&o)[R], const f3 (&d)[R], const float (&tmax)[R],
                                          const bool (&valid)[R], const bool (&anyhit)[R], uint32_t* sh,
                                          const float4* lrec = nullptr, const uint32_t* linfo = nullptr) {
  float tm[R];
  bool pv[R];
  RP_STAMP(0);
#pragma unroll
  for (int j = 0; j < R; ++j) {
    float bt = tmax[j];
    int bp = -1;
    // hits before the ray's t_min do not count (pt_intersect; 0 otherwise)
    const float tlo = (TMIN && valid[j]) ? A.tmin[id[j]] : 0.0f;
    // the closest-hit rule: ties go to the lowest primitive across the inline
    // leaves too (their primitive ranges are not in increasing order)
    auto test = [&](const Prim& q, int gi) {
      float tt;
      if (prim_sphere<REFA>(q)) {
        tt = sphere_test(o[j], d[j], q.q0, q.q1, tlo);
      } else if (anyhit[j]) {
        // shadow rays: division-free pre-test (they mostly point away from
        // the walls or end before them, see tri_outside)
        float ndd, num;
        plane_nd<REFA>(o[j], d[j], q, ndd, num);
        tt = -1.0f;
        if (!tri_outside<REFA>(ndd, num, bt)) tt = tri_test<REFA>(o[j], d[j], q, bt, tlo);
      } else {
        tt = tri_test<REFA>(o[j], d[j], q, bt, tlo);
      }
      if (tt >= 0.0f && (tt < bt || (tt == bt && (bp < 0 || gi < bp)))) {
        bt = tt;
        bp = gi;
      }
    };
    if (T.ni > 0) {
      const f3 inv = mk(__builtin_amdgcn_rcpf(safe_dir(d[j].x)), __builtin_amdgcn_rcpf(safe_dir(d[j].y)),
                        __builtin_amdgcn_rcpf(safe_dir(d[j].z)));
      const f3 oi = mk(o[j].x * inv.x, o[j].y * inv.y, o[j].z * inv.z);
      if (CL && (anyhit[j] ? T.nc_shadow : T.nc) > 0) {
        if (valid[j]) {
          const CPTR(f4v) B = (const CPTR(f4v))T.cbox;
          uint32_t cm = 0u;
          for (int c = 0; c < T.nc; ++c) {
            const float4 b0 = f4(B[2 * c]), b1 = f4(B[2 * c + 1]);
            cm |= box_hit(b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, oi, inv, bt) ? (1u << c) : 0u;
          }
          // (a shadow ray is done at its first hit)
          while (cm && !(anyhit[j] && bp >= 0)) {
            const int c = __builtin_ctz(cm);
            cm &= cm - 1u;
            const uint32_t fc = linfo[c];
            const int m0 = (int)(fc & 0xFFFFu), m1 = m0 + (int)(fc >> 16);
            for (int m = m0; m < m1; ++m) {
              Prim q;
              constexpr int PS = prim_stride<REFA>();
              q.q0 = lrec[PS * m];
              q.q1 = lrec[PS * m + 1];
              q.q2 = lrec[PS * m + 2];
              q.q3 = lrec[PS * m + 3];
              if constexpr (REFA) {
                q.q4 = lrec[PS * m + 4];
                q.q5 = lrec[PS * m + 5];
              }
              test(q, (int)linfo[ROOT_CL_MAX + m]);
            }
          }
        }
      } else {
        for (int i = 0; i < T.ni; ++i) {
          // the leaf's primitive range in the round trip of its box (the
          // compiler would read it behind the box test: two more round trips)
          const int pstart = T.istart[i], pcount = T.icount[i];
          const float b0 = T.ib[0][i], b1 = T.ib[1][i], b2 = T.ib[2][i], b3 = T.ib[3][i], b4 = T.ib[4][i],
                      b5 = T.ib[5][i];
          asm volatile("" ::"s"(pstart), "s"(pcount));
          if (!valid[j] || !box_hit(b0, b1, b2, b3, b4, b5, oi, inv, bt)) continue;
          constexpr int PS = prim_stride<REFA>();
          const CPTR(f4v) P = (const CPTR(f4v))(A.prims + (size_t)pstart * PS);
          int kk = 0;
          if constexpr (!REFA) {
            // two records per scalar round trip (round 4: +0.8 % on CBbunny)
            for (; kk + 1 < pcount; kk += 2, P += 2 * PS) {
              Prim qa, qb;
              load_prim_pair(P, qa, qb);
              test(qa, pstart + kk);
              test(qb, pstart + kk + 1);
            }
          }
          for (; kk < pcount; ++kk, P += PS) test(load_prim<REFA>(P), pstart + kk);
        }
      }
    }
    if (valid[j]) {  // the whole 32-B record at once (one full half line per ray)
      PT_CHECK(id[j] < A.dbg_nslots, "root_pass record", id[j], A.dbg_nslots);
      A.ray[RSTRIDE * id[j]] = make_float4(o[j].x, o[j].y, o[j].z, d[j].x);
      A.ray[RSTRIDE * id[j] + 1] =
          make_float4(d[j].y, d[j].z, __uint_as_float(bp >= 0 ? (uint32_t)bp : PT_PRIM_NONE), bt);
    }
    tm[j] = bt;
    pv[j] = valid[j] && !(anyhit[j] && bp >= 0);
    if (j == 0) {
      RP_STAMP(4);
    }
  }
  RP_STAMP(1);
  push_children<R, MAX_ROOT_TARGETS>(A, TableTargets{T}, lane, id, o, d, tm, pv, R, sh, false);
  RP_STAMP(5);
}

// LEAF: the node is known to be a leaf (the leaf-only level kernel): the
// interior code is not compiled in (fewer registers, more waves)
template <bool IMPLICIT, bool REFA = false, bool LEAF = false, bool TMIN = false>
__device__ __forceinline__ uint32_t process_item(const TraceArgs& A, int node, uint32_t base, int n, int lane,
                                             uint32_t* sh, bool ids = true, bool out_ids = true) {
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  // node and primitive records are wave-uniform: read them through the
  // constant address space so they land in SGPRs via s_load
  const CPTR(pt_node) nd = (const CPTR(pt_node))(A.nodes + node);

  uint32_t id[RPT];
  f3 o[RPT], d[RPT];
  float tmax[RPT];
  bool valid[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int i = j * TPB + tid;
    valid[j] = i < n;
    id[j] = 0;
    tmax[j] = -1.0f;
    o[j] = mk(0.f, 0.f, 0.f);
    d[j] = mk(0.f, 0.f, 1.f);
    if (valid[j]) {
      if (IMPLICIT) {
        id[j] = base + (uint32_t)i;
        const float4 b = A.ray[RSTRIDE * id[j] + 1];
        tmax[j] = b.w;
        valid[j] = b.w >= 0.0f;
        if (valid[j]) {
          const float4 a = A.ray[RSTRIDE * id[j]];
          o[j] = mk(a.x, a.y, a.z);
          d[j] = mk(a.w, b.x, b.y);
        }
      } else {
        load_ray(A, ids, base + (uint32_t)i, id[j], o[j], d[j], tmax[j]);
      }
    }
  }

  uint32_t nvalid = 0;
  float tlo[RPT];  // the rays' t_min (pt_intersect; TMIN only)
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    nvalid += valid[j] ? 1u : 0u;
    tlo[j] = (TMIN && valid[j]) ? A.tmin[id[j]] : 0.0f;
  }

  const int nj = (n + TPB - 1) / TPB;  // ray groups with at least one valid thread (uniform)
  const int pcount = nd->prim_count;
  if (LEAF || pcount > 0) {
    // ---------------- leaf: all primitives against every ray -----------------
    const int pstart = nd->prim_start;
    float bt[RPT];
    int bp[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      bt[j] = next_up(tmax[j]);
      bp[j] = -1;
    }
    constexpr int PS = prim_stride<REFA>();
    const CPTR(f4v) P = (const CPTR(f4v))(A.prims + (size_t)pstart * PS);
    for (int k = 0; k < pcount; ++k, P += PS) {
      const Prim q = load_prim<REFA>(P);
      if (prim_sphere<REFA>(q)) {
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
          if (j >= nj) break;
          take_strict(sphere_test(o[j], d[j], q.q0, q.q1, tlo[j]), pstart + k, bt[j], bp[j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < RPT; j += 2) {
          if (j >= nj) break;
          if constexpr (!REFA) {
            // (the update inside the test, no -1 sentinel)
            bw_update2(pair3(o[j], o[j + 1]), pair3(d[j], d[j + 1]), q, f2v{tlo[j], tlo[j + 1]}, pstart + k, bt[j],
                       bt[j + 1], bp[j], bp[j + 1]);
            continue;
          }
          const f2v t2 = tri_test2<REFA, true>(pair3(o[j], o[j + 1]), pair3(d[j], d[j + 1]), q, f2v{bt[j], bt[j + 1]},
                                               f2v{tlo[j], tlo[j + 1]});
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            take_strict(t2[i], pstart + k, bt[j + i], bp[j + i]);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      // the record's {prim, t} word: later box tests of this ray read the
      // tightened t as their tmax (a shadow ray: occluded, done)
#ifdef PT_DBG_BOUNDS
      if (valid[j] && bp[j] >= 0 && id[j] >= A.dbg_nslots)
        printf("PT_DBG_BOUNDS report_hit %u vs %u\n", id[j], A.dbg_nslots);
      else
#endif
      if (valid[j] && bp[j] >= 0) report_hit(A.ray, A.shadow_base, id[j], bt[j], (uint32_t)bp[j]);
    }
    return nvalid;
  }

  // ---------------- interior: NC child boxes, compaction, push ----------------
  if constexpr (!LEAF) push_children<RPT, 4>(A, ChildTargets{nd}, lane, id, o, d, tmax, valid, nj, sh, !out_ids);
  return nvalid;
}

// ---- root pass (level 0) of pt_intersect: implicit queue = slots [r0, r1) ------------
// Single-leaf trees: the root leaf's primitives against every ray (process_item).
// Otherwise root_pass: inline leaves, then the root table's targets.
template <bool REFA, bool TMIN = false>
__global__ __launch_bounds__(TPB) void k_trace_root(TraceArgs A, RootTable T, uint32_t r0, uint32_t r1,
                                                    unsigned long long* __restrict__ rcount) {
  __shared__ uint32_t sh[MAX_ROOT_TARGETS * 8 + 4];
  const uint32_t item = blockIdx.x;
  const uint32_t first = r0 + item * TILE;
  const int n = (int)min((uint32_t)TILE, r1 - first);
  const int lane = item & (NLANE - 1);
  uint32_t v = 0;
  if (((const CPTR(pt_node))A.nodes)->prim_count > 0) {
    v = process_item<true, REFA, false, TMIN>(A, 0, first, n, lane, sh);
  } else {
    uint32_t id[RPT];
    f3 o[RPT], d[RPT];
    float tmax[RPT];
    bool valid[RPT], anyhit[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int i = j * TPB + (int)threadIdx.x;
      id[j] = first + (uint32_t)i;
      o[j] = mk(0.f, 0.f, 0.f);
      d[j] = mk(0.f, 0.f, 1.f);
      tmax[j] = -1.0f;
      valid[j] = false;
      anyhit[j] = false;
      if (i < n) {
        const float4 b = A.ray[RSTRIDE * id[j] + 1];
        if (b.w >= 0.0f) {
          const float4 a = A.ray[RSTRIDE * id[j]];
          o[j] = mk(a.x, a.y, a.z);
          d[j] = mk(a.w, b.x, b.y);
          tmax[j] = b.w;
          valid[j] = true;
          v++;
        }
      }
    }
    root_pass<RPT, REFA, TMIN>(A, T, lane, id, o, d, tmax, valid, anyhit, sh);
  }
  // valid-ray count (R of the roofline formula): one fire-and-forget atomic per
  // workgroup into this lane's counter line
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[MAX_ROOT_TARGETS * 8 + (threadIdx.x >> 6)] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = sh[MAX_ROOT_TARGETS * 8] + sh[MAX_ROOT_TARGETS * 8 + 1] + sh[MAX_ROOT_TARGETS * 8 + 2] +
                       sh[MAX_ROOT_TARGETS * 8 + 3];
    if (t) atomicAdd(rcount + (size_t)(item & (RCOUNT_SLOTS - 1)) * 16, (unsigned long long)t);
  }
}

// ---- one wave-sized item: up to WTILE rays of one node's queue lane ---------------
// Levels >= 1 are processed at wave granularity: no LDS, no workgroup barrier,
// one returning atomic per wave per child.  Deep levels hold many nodes with a
// few hundred rays each, where 1024-ray workgroup items would run mostly empty.
// Two-level push (real levels of the two-level traversal): the wave's rays
// that enter child c of the node go straight to c's queue when c is a leaf,
// else to the queues of c's children that they enter (c itself is never
// queued: one ray gather, one queue round trip and one scan instead of two per
// pair of BVH levels).  Target t = 4c + g (g = 0 for a leaf child); lane t
// holds its node, count and slot base, so the up to 16 slot reservations take
// one atomic round trip.  A grandchild's box is tested only for rays that
// entered its parent's box.  Ray ids only (the queues hold ids).
__device__ __forceinline__ float f4c(const float4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
__device__ __forceinline__ void push_two_level(const TraceArgs& A, int node, const CPTR(pt_node) nd, int lane,
                                               const uint32_t (&id)[RPTW], const f3 (&inv)[RPTW],
                                               const f3 (&oi)[RPTW], const float (&tmax)[RPTW],
                                               const bool (&valid)[RPTW], int nj) {
  const uint32_t lid = lane_id();
  // the targets (node data only): lane t = 4c + g holds the node of target
  // t -- leaf child c (g = 0) or child g of interior child c -- or -1
  int tnode = -1;
  bool tleaf = false;
  if (lid < 16) {
    const int ch = A.nodes[node].child[lid >> 2];
    if (ch >= 0) {
      tleaf = A.nodes[ch].prim_count > 0;
      tnode = tleaf ? ((lid & 3) == 0 ? ch : -1) : A.nodes[ch].child[lid & 3];
    }
  }
  const uint32_t tmask = (uint32_t)__ballot(tnode >= 0);           // (uniform)
  const uint32_t lmask = (uint32_t)__ballot(tnode >= 0 && tleaf);  // targets that are leaf children
  uint32_t bits[RPTW];
#pragma unroll
  for (int j = 0; j < RPTW; ++j) bits[j] = 0;
  // (not unrolled: one child node's records in SGPRs at a time)
#pragma unroll 1
  for (int c = 0; c < 4; ++c) {
    const uint32_t cm = (tmask >> (4 * c)) & 0xFu;
    if (!cm) continue;
    // the child's box in SGPRs once (the compiler re-issued the six scalar
    // loads inside every ray's branch, one round trip each)
    const float cb0 = nd->bmin_x[c], cb1 = nd->bmax_x[c], cb2 = nd->bmin_y[c], cb3 = nd->bmax_y[c],
                cb4 = nd->bmin_z[c], cb5 = nd->bmax_z[c];
    asm volatile("" ::"s"(cb0), "s"(cb1), "s"(cb2), "s"(cb3), "s"(cb4), "s"(cb5));
    uint32_t hc = 0;  // rays j that enter child c (bit j)
#pragma unroll
    for (int j = 0; j < RPTW; ++j) {
      if (j >= nj) break;
      const bool h = valid[j] && box_hit(cb0, cb1, cb2, cb3, cb4, cb5, oi[j], inv[j], tmax[j]);
      hc |= h ? (1u << j) : 0u;
    }
    if (!__any(hc != 0)) continue;
    if ((lmask >> (4 * c)) & 1u) {
#pragma unroll
      for (int j = 0; j < RPTW; ++j) bits[j] |= ((hc >> j) & 1u) << (4 * c);
      continue;
    }
    // the four grandchild boxes (SoA rows of the child node) in one round trip
    const CPTR(f4v) cn = (const CPTR(f4v))(A.nodes + nd->child[c]);
    const float4 gx0 = f4(cn[0]), gx1 = f4(cn[1]), gy0 = f4(cn[2]), gy1 = f4(cn[3]), gz0 = f4(cn[4]),
                 gz1 = f4(cn[5]);
    asm volatile("" ::"s"(gx0.x), "s"(gx1.x), "s"(gy0.x), "s"(gy1.x), "s"(gz0.x), "s"(gz1.x));
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (!((cm >> g) & 1u)) continue;
      const float b0 = f4c(gx0, g), b1 = f4c(gx1, g), b2 = f4c(gy0, g), b3 = f4c(gy1, g), b4 = f4c(gz0, g),
                  b5 = f4c(gz1, g);
#pragma unroll
      for (int j = 0; j < RPTW; ++j) {
        if (j >= nj) break;
        const bool h = ((hc >> j) & 1u) && box_hit(b0, b1, b2, b3, b4, b5, oi[j], inv[j], tmax[j]);
        bits[j] |= h ? (1u << (4 * c + g)) : 0u;
      }
    }
  }
  // lane t: rays pushed to target t
  uint32_t tot = 0;
  for (uint32_t m = tmask; m; m &= m - 1) {
    const uint32_t t = (uint32_t)__builtin_ctz(m);
    uint32_t cntt = 0;
#pragma unroll
    for (int j = 0; j < RPTW; ++j) cntt += (uint32_t)__popcll(__ballot((bits[j] >> t) & 1u));
    tot = lid == t ? cntt : tot;
  }
#ifdef PT_DBG_SEQ_TARGETS
  for (uint32_t m = tmask; m; m &= m - 1) {
    const uint32_t t = (uint32_t)__builtin_ctz(m);
    const int tn = __builtin_amdgcn_readlane(tnode, t);
    const uint32_t tt = __builtin_amdgcn_readlane(tot, t);
    if (tt == 0) continue;
    uint32_t bb = 0;
    if (lid == 0) bb = atomicAdd(A.cnt + cnt_idx(tn, lane), tt) + A.qoff[(size_t)tn * NLANE + lane];
    uint32_t off = __builtin_amdgcn_readfirstlane(bb);
#else
  // every target's slot reservation and queue offset in one round trip
  uint32_t b = 0;
  if (tnode >= 0 && tot) b = atomicAdd(A.cnt + cnt_idx(tnode, lane), tot) + A.qoff[(size_t)tnode * NLANE + lane];
  for (uint32_t m = tmask; m; m &= m - 1) {
    const uint32_t t = (uint32_t)__builtin_ctz(m);
    uint32_t off = __builtin_amdgcn_readlane(b, t);
#endif
#pragma unroll
    for (int j = 0; j < RPTW; ++j) {
      const bool h = (bits[j] >> t) & 1u;
      const unsigned long long mm = __ballot(h);
#ifdef PT_DBG_BOUNDS
      if (h && off + mbcnt64(mm) >= A.dbg_qids)
        printf("PT_DBG_BOUNDS two-level push %u vs %llu node %d target %u\n", off + mbcnt64(mm),
               (unsigned long long)A.dbg_qids, node, t);
      else
#endif
      if (h) A.q[off + mbcnt64(mm)] = id[j];
      off += (uint32_t)__popcll(mm);
    }
  }
}

#ifndef PT_DBG_LINES
#define PT_DBG_LINES 0
#endif
#if PT_DBG_LINES
// diagnostic build only: how many distinct memory lines a wave item's ray
// record gathers touch, for records of 32 B (4 per 128-B line, as built), 16 B
// (8 per line) and 8 B (16 per line): g_dbg_lines[4 kind + {rays, lines32,
// lines16, lines8}], kind 0 interior, 1 leaf items
static __device__ unsigned long long g_dbg_lines[8];
template <int R>
__device__ __forceinline__ void dbg_count_lines(const uint32_t (&id)[R], const bool (&valid)[R], bool leaf) {
  const uint32_t lid = lane_id();
  uint32_t nl[3] = {0, 0, 0}, nv = 0;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    bool dup[3] = {false, false, false};
    for (int jj = 0; jj <= j; ++jj) {
      for (int k = 0; k < 64; ++k) {
        const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)id[jj], k);
        const bool ov = __builtin_amdgcn_readlane((int)valid[jj], k) != 0;
        const bool before = jj < j || (uint32_t)k < lid;
        if (!ov || !before) continue;
        dup[0] |= (o >> 2) == (id[j] >> 2);
        dup[1] |= (o >> 3) == (id[j] >> 3);
        dup[2] |= (o >> 4) == (id[j] >> 4);
      }
    }
    nv += (uint32_t)__popcll(__ballot(valid[j]));
#pragma unroll
    for (int g = 0; g < 3; ++g) nl[g] += (uint32_t)__popcll(__ballot(valid[j] && !dup[g]));
  }
  if (lid == 0) {
    unsigned long long* c = g_dbg_lines + (leaf ? 4 : 0);
    atomicAdd(c, (unsigned long long)nv);
    for (int g = 0; g < 3; ++g) atomicAdd(c + 1 + g, (unsigned long long)nl[g]);
  }
}
#endif

template <bool REFA = false, bool LEAF = false, bool TMIN = false>
__device__ __forceinline__ void process_wave(const TraceArgs& A, int node, uint32_t base, int n, int lane, bool ids,
                                             bool out_ids, bool two_level) {
  const uint32_t lid = lane_id();
  const CPTR(pt_node) nd = (const CPTR(pt_node))(A.nodes + node);
#ifdef PT_DBG_BOUNDS
  if (ids && (uint64_t)base + (uint64_t)n > A.dbg_qids) {
    if (lid == 0)
      printf("PT_DBG_BOUNDS process_wave queue read node %d lane %d base %u n %d vs %llu ids\n", node, lane, base, n,
             (unsigned long long)A.dbg_qids);
    return;
  }
#endif
  uint32_t id[RPTW];
  f3 o[RPTW], d[RPTW];
  float tmax[RPTW];
  bool valid[RPTW];
#pragma unroll
  for (int j = 0; j < RPTW; ++j) {
    const int i = j * 64 + (int)lid;
    valid[j] = i < n;
    id[j] = 0u;
    o[j] = mk(0.f, 0.f, 0.f);
    d[j] = mk(1.f, 0.f, 0.f);
    tmax[j] = -1.0f;
#ifdef PT_DBG_BOUNDS
    if (valid[j] && ids) {
      const uint32_t qi = A.q[base + (uint32_t)i];
      if (qi >= A.dbg_nslots) {
        printf("PT_DBG_BOUNDS process_wave ray id %u vs %u (node %d lane %d base %u i %d n %d)\n", qi, A.dbg_nslots,
               node, lane, base, i, n);
        valid[j] = false;
      }
    }
#endif
    if (valid[j]) load_ray(A, ids, base + (uint32_t)i, id[j], o[j], d[j], tmax[j]);
  }
  const int nj = (n + 63) >> 6;  // ray groups with at least one valid lane (uniform)
#if PT_DBG_LINES
  if (ids) dbg_count_lines<RPTW>(id, valid, nd->prim_count > 0);
#endif
  float tlo[RPTW];  // the rays' t_min (pt_intersect; TMIN only)
#pragma unroll
  for (int j = 0; j < RPTW; ++j) tlo[j] = (TMIN && valid[j]) ? A.tmin[id[j]] : 0.0f;
  const int pcount = nd->prim_count;
  if (LEAF || pcount > 0) {
    const int pstart = nd->prim_start;
    float bt[RPTW];
    int bp[RPTW];
#pragma unroll
    for (int j = 0; j < RPTW; ++j) {
      bt[j] = next_up(tmax[j]);
      bp[j] = -1;
    }
    constexpr int PS = prim_stride<REFA>();
    const CPTR(f4v) P = (const CPTR(f4v))(A.prims + (size_t)pstart * PS);
    // one primitive's tests against the wave's rays (its record in SGPRs,
    // loaded in one scalar round trip)
    auto leaf_test = [&](const Prim& q, int k) {
      if (prim_sphere<REFA>(q)) {
#pragma unroll
        for (int j = 0; j < RPTW; ++j) {
          if (j >= nj) break;
          take_strict(sphere_test(o[j], d[j], q.q0, q.q1, tlo[j]), pstart + k, bt[j], bp[j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < RPTW; j += 2) {
          if (j >= nj) break;
          if constexpr (!REFA) {
            // (the update inside the test, no -1 sentinel)
            bw_update2(pair3(o[j], o[j + 1]), pair3(d[j], d[j + 1]), q, f2v{tlo[j], tlo[j + 1]}, pstart + k, bt[j],
                       bt[j + 1], bp[j], bp[j + 1]);
            continue;
          }
          const f2v t2 = tri_test2<REFA, true>(pair3(o[j], o[j + 1]), pair3(d[j], d[j + 1]), q, f2v{bt[j], bt[j + 1]},
                                               f2v{tlo[j], tlo[j + 1]});
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            take_strict(t2[i], pstart + k, bt[j + i], bp[j + i]);
          }
        }
      }
    };
    int k0 = 0;
    if constexpr (!REFA) {
      // two records per scalar round trip (one wait per pair)
      for (; k0 + 1 < pcount; k0 += 2, P += 2 * PS) {
        Prim qa, qb;
        load_prim_pair(P, qa, qb);
        leaf_test(qa, k0);
        leaf_test(qb, k0 + 1);
      }
    }
    for (int k = k0; k < pcount; ++k, P += PS) leaf_test(load_prim<REFA>(P), k);
#pragma unroll
    for (int j = 0; j < RPTW; ++j) {
#ifdef PT_DBG_BOUNDS
      if (valid[j] && bp[j] >= 0 && id[j] >= A.dbg_nslots)
        printf("PT_DBG_BOUNDS report_hit %u vs %u\n", id[j], A.dbg_nslots);
      else
#endif
      if (valid[j] && bp[j] >= 0) report_hit(A.ray, A.shadow_base, id[j], bt[j], (uint32_t)bp[j]);
    }
    return;
  }
  if constexpr (LEAF) return;
  if (two_level) {
    f3 inv[RPTW], oi[RPTW];
#pragma unroll
    for (int j = 0; j < RPTW; ++j) {
      inv[j] = mk(__builtin_amdgcn_rcpf(safe_dir(d[j].x)), __builtin_amdgcn_rcpf(safe_dir(d[j].y)),
                  __builtin_amdgcn_rcpf(safe_dir(d[j].z)));
      oi[j] = mk(o[j].x * inv[j].x, o[j].y * inv[j].y, o[j].z * inv[j].z);
    }
    push_two_level(A, node, nd, lane, id, inv, oi, tmax, valid, nj);
    return;
  }
  uint32_t bits[RPTW];
#pragma unroll
  for (int j = 0; j < RPTW; ++j) {
    bits[j] = 0;
    if (j >= nj) continue;
    f3 inv = mk(__builtin_amdgcn_rcpf(safe_dir(d[j].x)), __builtin_amdgcn_rcpf(safe_dir(d[j].y)),
                __builtin_amdgcn_rcpf(safe_dir(d[j].z)));
    f3 oi = mk(o[j].x * inv.x, o[j].y * inv.y, o[j].z * inv.z);
    uint32_t b = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      bool h = box_hit(nd->bmin_x[c], nd->bmax_x[c], nd->bmin_y[c], nd->bmax_y[c], nd->bmin_z[c],
                       nd->bmax_z[c], oi, inv, tmax[j]);
      b |= (valid[j] && h) ? (1u << c) : 0u;
    }
    bits[j] = b;
  }
  // per-child totals, then the (up to) four slot reservations at once, one per
  // lane 0..3: a single atomic round trip per item instead of four in a row
  uint32_t tot[4], qo[4];
  int child[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    child[c] = nd->child[c];
    tot[c] = 0;
#pragma unroll
    for (int j = 0; j < RPTW; ++j) tot[c] += (uint32_t)__popcll(__ballot((bits[j] >> c) & 1u));
    qo[c] = (child[c] >= 0 && tot[c]) ? A.qoff[(size_t)child[c] * NLANE + lane] : 0u;
  }
  uint32_t b = 0;
  const int lc = (int)lid;
  const int mych = lc == 0 ? child[0] : lc == 1 ? child[1] : lc == 2 ? child[2] : child[3];
  const uint32_t myt = lc == 0 ? tot[0] : lc == 1 ? tot[1] : lc == 2 ? tot[2] : tot[3];
  if (lc < 4 && mych >= 0 && myt) b = atomicAdd(A.cnt + cnt_idx(mych, lane), myt);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (child[c] < 0 || tot[c] == 0) continue;
    uint32_t off = __builtin_amdgcn_readlane(b, c) + qo[c];
#pragma unroll
    for (int j = 0; j < RPTW; ++j) {
      const bool h = (bits[j] >> c) & 1u;
      const unsigned long long m = __ballot(h);
      if (h) push_ray(A, !out_ids, off + mbcnt64(m), id[j], o[j], d[j], tmax[j]);
      off += (uint32_t)__popcll(m);
    }
  }
}

// ---- per-level pass: every wave walks the items of its block's lane ----------------
// Lane s's items are processed by blocks b with b % 8 == s (same XCD under the
// observed round-robin placement: a speed hint only).
// 5 waves per SIMD (<= 96 VGPRs): the two-level push needs 91 without spills
// (at 6 waves, 80 VGPRs, it spilled 19; round 1's one-level push: 6 waves
// +2-3 % over 4, 7 waves spilled and lost 4 %)
constexpr int LEVEL_WAVES = 5;
// LEAF: a level whose queued nodes are all leaves (the levels between two
// real levels hold only the leaf rays of the real level above them): the
// leaf-only code needs fewer registers and runs LEAF_WAVES waves per SIMD
// (8, round 3: 64 VGPRs, 4 spilled, against 68 at 7 waves: the leaf levels'
// share of the dragon proxy's levels ~1 % faster; round 5: 7 waves -0.3-0.5 %)
constexpr int LEAF_WAVES = 8;
// TMIN: the rays carry a t_min (pt_intersect with t_min > 0 somewhere in the
// batch): hits before it do not count (TraceArgs::tmin)
template <bool REFA, bool LEAF, bool BLOCK = true, bool TMIN = false>
__device__ __forceinline__ void trace_level_body(const TraceArgs& A, const LevelArgs& L);
template <bool REFA, bool TMIN = false>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(LEVEL_WAVES, 8))) void k_trace_level(TraceArgs A,
                                                                                                           LevelArgs L) {
  trace_level_body<REFA, false, true, TMIN>(A, L);
}
// The real levels of the two-level traversal always run wave items (their
// push exists for wave items only): without the workgroup-item code the
// kernel needs 22 SGPR spills instead of 51, and runs 6 waves per SIMD (80
// VGPRs, 5 spilled): dragon proxy level 6 30.1 -> 28.4 ms, frame +0.9 %
// (at 5 waves it measured the same as k_trace_level); round 3: 7 waves (72
// VGPRs, 6 spilled) with the leaf kernel at 8: levels -1.5 to -3 % on the
// dragon proxy trees and bunny.dae (round 5: 6 waves -0.3-0.5 %)
constexpr int REAL_WAVES = 7;
template <bool REFA, bool TMIN = false>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(REAL_WAVES, 8))) void k_trace_real(TraceArgs A,
                                                                                                         LevelArgs L) {
  trace_level_body<REFA, false, false, TMIN>(A, L);
}
template <bool REFA, bool TMIN = false>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(LEAF_WAVES, 8))) void k_trace_leaves(
    TraceArgs A, LevelArgs L) {
  trace_level_body<REFA, true, true, TMIN>(A, L);
}
template <bool REFA, bool LEAF, bool BLOCK, bool TMIN>
__device__ __forceinline__ void trace_level_body(const TraceArgs& A, const LevelArgs& L) {
  const int lane = blockIdx.x & (NLANE - 1);
  const uint32_t lid = lane_id();
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t* __restrict__ ep = L.iprefix + (size_t)lane * (L.maxln + 1);
  const uint32_t M = ep[L.nl];  // items of this lane
  if (BLOCK && *L.mode == MODE_BLOCK) {
    // few nodes with many rays: 1024-ray items, one atomic per workgroup per child
    __shared__ uint32_t sh[64];
    __shared__ int s_node;
    __shared__ uint32_t s_base;
    __shared__ int s_n;
    for (uint32_t m = blockIdx.x / NLANE; m < M; m += gridDim.x / NLANE) {
      if (wave == 0) {
        int lo = 0, hi = L.nl;
        while (hi - lo > 1) {
          const int step = (hi - lo + 63) >> 6;
          const int idx = lo + (int)lid * step;
          const bool le = idx < hi && ep[idx] <= m;
          const unsigned long long msk = __ballot(le);
          lo = lo + (63 - __clzll(msk)) * step;
          hi = min(lo + step, hi);
        }
        if (lid == 0) {
          const int node = L.first + lo;
          const uint32_t i = m - ep[lo];
          const uint32_t c = L.icnt[(size_t)lane * (L.maxln + 1) + lo];
          s_node = node;
          s_base = A.qoff[(size_t)node * NLANE + lane] + i * TILE;
          s_n = (int)min((uint32_t)TILE, c - i * TILE);
        }
      }
      __syncthreads();
      const int node = __builtin_amdgcn_readfirstlane(s_node);
      const uint32_t base = __builtin_amdgcn_readfirstlane(s_base);
      const int n = __builtin_amdgcn_readfirstlane(s_n);
      __syncthreads();
      process_item<false, REFA, LEAF, TMIN>(A, node, base, n, lane, sh, L.ids != 0, L.out_ids != 0);
      __syncthreads();
    }
    return;
  }
  // many nodes with few rays each: every wave walks its own 256-ray items
  const uint32_t stride = (gridDim.x / NLANE) * (TPB / 64);
  for (uint32_t m = (blockIdx.x / NLANE) * (TPB / 64) + wave; m < M; m += stride) {
    // 64-ary search for the node k with ep[k] <= m < ep[k+1]
    int lo = 0, hi = L.nl;
    while (hi - lo > 1) {
      const int step = (hi - lo + 63) >> 6;
      const int idx = lo + (int)lid * step;
      const bool le = idx < hi && ep[idx] <= m;
      const unsigned long long msk = __ballot(le);
      lo = lo + (63 - __clzll(msk)) * step;
      hi = min(lo + step, hi);
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    const int node = L.first + lo;
    const uint32_t i = m - ep[lo];
    const uint32_t c = L.icnt[(size_t)lane * (L.maxln + 1) + lo];
    const uint32_t base = A.qoff[(size_t)node * NLANE + lane] + i * WTILE;
    const int n = (int)min((uint32_t)WTILE, c - i * WTILE);
    process_wave<REFA, LEAF, TMIN>(A, node, __builtin_amdgcn_readfirstlane(base), __builtin_amdgcn_readfirstlane(n), lane,
                       L.ids != 0, L.out_ids != 0, L.two_level != 0);
  }
}

// ---- depth-first subtree traversal below the DFS cut level -----------------------
// The rays of the cut level's (node, lane) queues are gathered once and each
// lane walks its ray through the node's whole subtree: nearest child first,
// the others on a per-lane LDS stack; node and primitive records through
// vector loads (a subtree's records stay L2-resident while its queue is
// processed).  Same closest-hit rules as the level kernels (min of the {t,
// prim} key, ties to the lowest primitive; a shadow ray stops at its first
// occluder), so the result does not depend on the traversal order.
constexpr int DFS_STACK = 32;  // per-lane stack entries (the host checks 3 x subtree depth fits)
__device__ __forceinline__ bool box_hit_t(float bx0, float bx1, float by0, float by1, float bz0, float bz1,
                                          const f3 oi, const f3 inv, float tmax, float& tn) {
  float tx0 = __builtin_fmaf(bx0, inv.x, -oi.x), tx1 = __builtin_fmaf(bx1, inv.x, -oi.x);
  float ty0 = __builtin_fmaf(by0, inv.y, -oi.y), ty1 = __builtin_fmaf(by1, inv.y, -oi.y);
  float tz0 = __builtin_fmaf(bz0, inv.z, -oi.z), tz1 = __builtin_fmaf(bz1, inv.z, -oi.z);
  tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
  float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
  return tn <= tf;
}
template <bool REFA, bool TMIN>
__device__ __forceinline__ void dfs_ray(const TraceArgs& A, int root, uint32_t id, const f3 o, const f3 d,
                                        float tmax, int* __restrict__ stk) {
  const float tlo = TMIN ? A.tmin[id] : 0.0f;
  const bool anyhit = id >= A.shadow_base;
  const f3 inv = mk(__builtin_amdgcn_rcpf(safe_dir(d.x)), __builtin_amdgcn_rcpf(safe_dir(d.y)),
                    __builtin_amdgcn_rcpf(safe_dir(d.z)));
  const f3 oi = mk(o.x * inv.x, o.y * inv.y, o.z * inv.z);
  float bt = tmax;
  int bp = -1;
  int sp = 0;
  int node = root;
  constexpr int PS = prim_stride<REFA>();
  while (true) {
    if (node < 0) {
      if (sp == 0) break;
      --sp;
      node = stk[sp * TPB];
    }
    const float4* nv = reinterpret_cast<const float4*>(A.nodes + node);
    const int4 lk = reinterpret_cast<const int4*>(nv)[6];  // child[4]
    const int4 pr = reinterpret_cast<const int4*>(nv)[7];  // prim_start, prim_count, ...
    if (pr.y > 0) {
      const float4* P = A.prims + (size_t)pr.x * PS;
      bool stop = false;
      for (int k = 0; k < pr.y; ++k, P += PS) {
        Prim q;
        q.q0 = P[0];
        q.q1 = P[1];
        q.q2 = P[2];
        q.q3 = P[3];
        if constexpr (REFA) {
          q.q4 = P[4];
          q.q5 = P[5];
        }
        const float t = prim_sphere<REFA>(q) ? sphere_test(o, d, q.q0, q.q1, tlo) : tri_test<REFA>(o, d, q, bt, tlo);
        const int pi = pr.x + k;
        if (t >= 0.0f && t <= bt && (t < bt || bp < 0 || pi < bp)) {
          bt = t;
          bp = pi;
          if (anyhit) {
            stop = true;
            break;
          }
        }
      }
      node = -1;
      if (stop) break;
      continue;
    }
    const float4 bx0 = nv[0], bx1 = nv[1], by0 = nv[2], by1 = nv[3], bz0 = nv[4], bz1 = nv[5];
    node = -1;
    float best = 0.0f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int ch = c == 0 ? lk.x : c == 1 ? lk.y : c == 2 ? lk.z : lk.w;
      float tn;
      const bool h = ch >= 0 && box_hit_t(f4c(bx0, c), f4c(bx1, c), f4c(by0, c), f4c(by1, c), f4c(bz0, c),
                                          f4c(bz1, c), oi, inv, bt, tn);
      if (h) {
        if (node < 0) {
          node = ch;
          best = tn;
        } else {
          const bool nearer = tn < best;
          stk[sp * TPB] = nearer ? node : ch;
          ++sp;
          node = nearer ? ch : node;
          best = nearer ? tn : best;
        }
      }
    }
  }
  if (bp >= 0) report_hit(A.ray, A.shadow_base, id, bt, (uint32_t)bp);
}
// The DFS cut level: wave items of 256 rays (the scan runs it in wave mode),
// each lane's rays one after another through dfs_ray.
template <bool REFA, bool TMIN = false>
__global__ __launch_bounds__(TPB) void k_trace_dfs(TraceArgs A, LevelArgs L) {
  __shared__ int stk[DFS_STACK * TPB];
  const int lane = blockIdx.x & (NLANE - 1);
  const uint32_t lid = lane_id();
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t* __restrict__ ep = L.iprefix + (size_t)lane * (L.maxln + 1);
  const uint32_t M = ep[L.nl];
  const uint32_t stride = (gridDim.x / NLANE) * (TPB / 64);
  for (uint32_t m = (blockIdx.x / NLANE) * (TPB / 64) + wave; m < M; m += stride) {
    int lo = 0, hi = L.nl;
    while (hi - lo > 1) {
      const int step = (hi - lo + 63) >> 6;
      const int idx = lo + (int)lid * step;
      const bool le = idx < hi && ep[idx] <= m;
      const unsigned long long msk = __ballot(le);
      lo = lo + (63 - __clzll(msk)) * step;
      hi = min(lo + step, hi);
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    const int node = L.first + lo;
    const uint32_t i = m - ep[lo];
    const uint32_t c = L.icnt[(size_t)lane * (L.maxln + 1) + lo];
    const uint32_t base = __builtin_amdgcn_readfirstlane(A.qoff[(size_t)node * NLANE + lane] + i * WTILE);
    const int n = __builtin_amdgcn_readfirstlane((int)min((uint32_t)WTILE, c - i * WTILE));
    for (int j = 0; j < RPTW; ++j) {
      const int r = j * 64 + (int)lid;
      if (r >= n) break;
      uint32_t id;
      f3 o, d;
      float tmax;
      load_ray(A, L.ids != 0, base + (uint32_t)r, id, o, d, tmax);
      if (tmax >= 0.0f) dfs_ray<REFA, TMIN>(A, node, id, o, d, tmax, stk + threadIdx.x);
    }
  }
}

// ---- per-level scan: work ranges and child queue allocation ---------------------
// One workgroup of 1024 threads.  For every (node, lane) of level l it
//  1. snapshots the node's ray count into a dense per-level array (read by
//     k_trace_level) and re-zeroes the atomic counter for the next pass;
//  2. picks the level's item shape (workgroup or wave items);
//  3. turns counts into items (exclusive prefix per lane) and allocates each
//     child's queue lane with capacity = the parent's count in that lane (the
//     reference's wOffset + i*rayCount, cu:922 and cu:1384, without the
//     single-warp scan and the D2H of maxBlocks, cu:2237).
// Each thread owns SCAN_NPT consecutive nodes of a chunk of 1024 * SCAN_NPT:
// their counter loads are issued together, and a level that fits one chunk
// (all but the widest) keeps its counts in registers between the passes.
constexpr int SCAN_NPT = 2;
// A node's child ids and prim_count in two 16-B loads (pt_node: child[4] at
// byte 96, {prim_start, prim_count, level, ref_id} at 112).
__device__ __forceinline__ void load_links(const TraceArgs& A, int node, int4& ch, int& pc) {
  const int4* q = reinterpret_cast<const int4*>(&A.nodes[node].child[0]);
  ch = q[0];
  pc = q[1].y;
}
__device__ __forceinline__ int i4(const int4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
// Queue targets of an interior node: t = 4c + g (the numbering of
// push_two_level) -- one level: child c (g = 0); two-level: the leaf child c
// (g = 0) or child g of the interior child c.  The node's links c4, its
// children's g4 / gpc (prim_count); -1 if none.
__device__ __forceinline__ int scan_target(const int4& c4, const int4 (&g4)[4], const int (&gpc)[4], int t,
                                           bool two_level) {
  const int ch = i4(c4, t >> 2);
  const bool direct = !two_level || gpc[t >> 2] > 0;
  return ch < 0 ? -1 : direct ? ((t & 3) == 0 ? ch : -1) : i4(g4[t >> 2], t & 3);
}
__device__ __forceinline__ void load_targets(const TraceArgs& A, int node, int4& c4, int4 (&g4)[4], int (&gpc)[4]) {
  int pc;
  load_links(A, node, c4, pc);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    g4[c] = make_int4(-1, -1, -1, -1);
    gpc[c] = 1;
    if (i4(c4, c) >= 0) load_links(A, i4(c4, c), g4[c], gpc[c]);
  }
}
__global__ __launch_bounds__(1024) void k_scan_level(TraceArgs A, LevelArgs L, uint32_t lanecap,
                                                     uint32_t out_parity_base, unsigned long long* stats,
                                                     int level, uint32_t* err) {
  static_assert((TILE & (TILE - 1)) == 0 && (WTILE & (WTILE - 1)) == 0, "item sizes are powers of two");
  constexpr int CH = 1024 * SCAN_NPT;
  __shared__ uint32_t wsum[16][16];
  __shared__ uint32_t run[16];
  __shared__ uint32_t ctot[16];
  __shared__ unsigned long long red[3][16];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, ln = tid & 63;
  const size_t row = (size_t)L.maxln + 1;
  const bool one = L.nl <= CH;
  if (tid < 16) run[tid] = 0;

  // pass 1: snapshot + zero the counters, totals for the mode decision
  uint32_t cnt[SCAN_NPT][NLANE];
  unsigned long long v = 0, pairs = 0, leafv = 0;
  for (int chunk = 0; chunk < L.nl; chunk += CH) {
    bool leaf[SCAN_NPT];
#pragma unroll
    for (int i = 0; i < SCAN_NPT; ++i) {
      const int k = chunk + tid * SCAN_NPT + i;
      leaf[i] = false;
#pragma unroll
      for (int s = 0; s < NLANE; ++s) cnt[i][s] = 0u;
      if (k < L.nl) {
        const int node = L.first + k;
        leaf[i] = A.nodes[node].prim_count > 0;
#pragma unroll
        for (int s = 0; s < NLANE; ++s) cnt[i][s] = A.cnt[cnt_idx(node, s)];
      }
    }
#pragma unroll
    for (int i = 0; i < SCAN_NPT; ++i) {
      const int k = chunk + tid * SCAN_NPT + i;
      if (k >= L.nl) continue;
      const int node = L.first + k;
#pragma unroll
      for (int s = 0; s < NLANE; ++s) {
        const uint32_t c = cnt[i][s];
        L.icnt_w[s * row + k] = c;
        v += c;
        pairs += c ? 1 : 0;
        if (leaf[i]) leafv += c;
        A.cnt[cnt_idx(node, s)] = 0u;
      }
    }
  }
  v = wave_sum64(v);
  pairs = wave_sum64(pairs);
  leafv = wave_sum64(leafv);
  if (ln == 0) {
    red[0][wave] = v;
    red[1][wave] = pairs;
    red[2][wave] = leafv;
  }
  __syncthreads();
  unsigned long long V = 0, PAIRS = 0, LEAFV = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    V += red[0][w];
    PAIRS += red[1][w];
    LEAFV += red[2][w];
  }
  // workgroup items when the (node, lane) queues are long (few nodes, high
  // atomic contention), wave items otherwise
  // (the two-level push exists for wave items only)
  const bool block_mode =
      !L.two_level && V >= (unsigned long long)BLOCK_MODE_RAYS_PER_PAIR * (PAIRS ? PAIRS : 1ull);
  const uint32_t itile = block_mode ? TILE : WTILE;
  const uint32_t ishift = (uint32_t)__builtin_ctz(itile);

  // pass 2: items and child capacities (16 values per node: items per lane,
  // child capacity per lane), thread-sequential over its nodes, then a block
  // exclusive scan of the thread totals
  for (int chunk = 0; chunk < L.nl; chunk += CH) {
    // queue targets of each node: its children, or (two-level) its leaf
    // children and the children of its interior children; none for the
    // interior nodes of a level that is not real (their children's queues are
    // allocated by the real level above them)
    // (the targets are counted here and listed again where their queues are
    // written: 16 of them per node do not fit this kernel's registers.  The
    // count is written without early exits: an increment in a `continue`
    // branch of this loop was dropped by the compiler -- hipcc, ROCm 7.2 --
    // for the first child, the first two-level build lost rays)
    uint32_t nch[SCAN_NPT];
#pragma unroll
    for (int i = 0; i < SCAN_NPT; ++i) {
      const int k = chunk + tid * SCAN_NPT + i;
      uint32_t n = 0;
      if (L.real && k < L.nl && A.nodes[L.first + k].prim_count == 0) {
        int4 c4, g4[4];
        int gpc[4];
        load_targets(A, L.first + k, c4, g4, gpc);
#pragma unroll
        for (int t = 0; t < 16; ++t) n += scan_target(c4, g4, gpc, t, L.two_level != 0) >= 0 ? 1u : 0u;
      }
      nch[i] = n;
      if (!one) {
#pragma unroll
        for (int s = 0; s < NLANE; ++s) cnt[i][s] = k < L.nl ? L.icnt_w[s * row + k] : 0u;
      }
    }
    // two halves of 8 values each (items per lane, then child capacity per
    // lane): half the registers of one 16-value scan
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t tv[NLANE];
#pragma unroll
      for (int s = 0; s < NLANE; ++s) {
        tv[s] = 0;
#pragma unroll
        for (int i = 0; i < SCAN_NPT; ++i)
          tv[s] += h == 0 ? (cnt[i][s] + itile - 1) >> ishift : cnt[i][s] * nch[i];
      }
      uint32_t ex[NLANE];
#pragma unroll
      for (int s = 0; s < NLANE; ++s) {
        uint32_t x = tv[s];
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const uint32_t y = __shfl_up(x, off, 64);
          if (ln >= off) x += y;
        }
        ex[s] = x - tv[s];
        if (ln == 63) wsum[wave][8 * h + s] = x;
      }
      __syncthreads();
      if (tid < NLANE) {
        uint32_t acc = 0;
        for (int w = 0; w < 16; ++w) {
          const uint32_t t = wsum[w][8 * h + tid];
          wsum[w][8 * h + tid] = acc;
          acc += t;
        }
        ctot[8 * h + tid] = acc;
      }
      __syncthreads();
#pragma unroll
      for (int s = 0; s < NLANE; ++s) ex[s] += run[8 * h + s] + wsum[wave][8 * h + s];
#pragma unroll
      for (int i = 0; i < SCAN_NPT; ++i) {
        const int k = chunk + tid * SCAN_NPT + i;
        if (k < L.nl) {
          if (h == 0) {
#pragma unroll
            for (int s = 0; s < NLANE; ++s) L.iprefix_w[s * row + k] = ex[s];
          } else {
            uint32_t jj = 0;
            auto alloc = [&](int target) {
              PT_CHECK((uint32_t)target < A.dbg_nnodes, "scan qoff", target, A.dbg_nnodes);
#pragma unroll
              for (int s = 0; s < NLANE; ++s)
                A.qoff[(size_t)target * NLANE + s] = out_parity_base + (uint32_t)s * lanecap + ex[s] + jj * cnt[i][s];
              jj++;
            };
            if (nch[i]) {
              // the node's links and its children's, all loaded before the
              // first qoff store (a load issued after a store waits for it:
              // one memory round trip per target otherwise)
              int4 c4, g4[4];
              int gpc[4];
              load_targets(A, L.first + k, c4, g4, gpc);
#pragma unroll
              for (int t = 0; t < 16; ++t) {
                const int tn = scan_target(c4, g4, gpc, t, L.two_level != 0);
                if (tn >= 0) alloc(tn);
              }
            }
          }
        }
#pragma unroll
        for (int s = 0; s < NLANE; ++s) ex[s] += h == 0 ? (cnt[i][s] + itile - 1) >> ishift : cnt[i][s] * nch[i];
      }
    }
    __syncthreads();
    if (tid < 16) run[tid] += ctot[tid];
    __syncthreads();
  }
  if (tid == 0) {
    bool ovf = false;
    unsigned long long items = 0, need = 0;
    for (int s = 0; s < NLANE; ++s) {
      if (run[8 + s] > lanecap) ovf = true;
      items += run[s];
      need = max(need, (unsigned long long)run[8 + s]);
    }
    // sentinels ep[nl] = items per lane; an overflowing level runs no items
    // (the rest of the pass is abandoned and the host reports PT_E_OVERFLOW)
    for (int s = 0; s < NLANE; ++s) L.iprefix_w[s * row + L.nl] = ovf ? 0u : run[s];
    *L.mode_w = block_mode ? MODE_BLOCK : MODE_WAVE;
    if (ovf) atomicOr(err, 1u);
    if (stats) {  // fire-and-forget atomics: no round trip on the critical path
      atomicAdd(stats + STAT_V, V);
      if (level < 16) {
        atomicAdd(stats + STAT_LV0 + level, V);
        atomicAdd(stats + STAT_LEAF0 + level, LEAFV);
        atomicAdd(stats + STAT_ITEMS0 + level, items);
      }
      atomicMax(stats + STAT_PEAKQ, need * NLANE);
    }
  }
}


// ---- multi-workgroup level scan (wide levels) --------------------------------------
// The results of k_scan_level in two launches of G = ceil(nl / SCAN_WG)
// workgroups, one node per thread, for levels too wide for one workgroup to
// scan quickly (a single workgroup walks them in chunks, one memory round trip
// after another):
//  k_scan_count: snapshot + re-zero the node's counters, count its queue
//    targets (kept in aux for the second launch) and reduce the workgroup's
//    partials: items per lane at TILE and at WTILE rays per item (the item
//    shape is not known before the level's totals are), child capacity per
//    lane, V, PAIRS, LEAFV;
//  k_scan_alloc: every workgroup sums the partials of the workgroups before
//    it (its exclusive offset) and of all (the level's totals: item shape,
//    overflow), scans its own nodes and writes their item prefixes and their
//    targets' queue offsets; the last workgroup writes the sentinels, the
//    mode, the overflow flag and the stats.
// aux: SCAN_MAXG rows of AGG_STRIDE u32 partials, then one target count per node.
constexpr int SCAN_WG = 256;
constexpr int AGG_N = 27, AGG_STRIDE = 32, SCAN_MAXG = 256;
enum { AGG_IT = 0, AGG_IW = 8, AGG_CAP = 16, AGG_V = 24, AGG_PAIRS = 25, AGG_LEAFV = 26 };

__global__ __launch_bounds__(SCAN_WG) void k_scan_count(TraceArgs A, LevelArgs L, uint32_t* __restrict__ aux) {
  __shared__ uint32_t red[SCAN_WG / 64][AGG_N];
  const int tid = threadIdx.x, wave = tid >> 6, ln = tid & 63;
  const int k = blockIdx.x * SCAN_WG + tid;
  const size_t row = (size_t)L.maxln + 1;
  uint32_t c[NLANE], nch = 0;
  bool leaf = false;
#pragma unroll
  for (int s = 0; s < NLANE; ++s) c[s] = 0u;
  if (k < L.nl) {
    const int node = L.first + k;
    int4 c4;
    int pc;
    load_links(A, node, c4, pc);
#pragma unroll
    for (int s = 0; s < NLANE; ++s) c[s] = A.cnt[cnt_idx(node, s)];
    leaf = pc > 0;
    if (L.real && !leaf) {
      int4 g4[4];
      int gpc[4];
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        g4[cc] = make_int4(-1, -1, -1, -1);
        gpc[cc] = 1;
        if (i4(c4, cc) >= 0) load_links(A, i4(c4, cc), g4[cc], gpc[cc]);
      }
#pragma unroll
      for (int t = 0; t < 16; ++t) nch += scan_target(c4, g4, gpc, t, L.two_level != 0) >= 0 ? 1u : 0u;
    }
#pragma unroll
    for (int s = 0; s < NLANE; ++s) {
      L.icnt_w[s * row + k] = c[s];
      A.cnt[cnt_idx(node, s)] = 0u;
    }
    aux[SCAN_MAXG * AGG_STRIDE + k] = nch;
  }
  constexpr uint32_t sT = __builtin_ctz(TILE), sW = __builtin_ctz(WTILE);
  uint32_t v = 0, pairs = 0;
#pragma unroll
  for (int s = 0; s < NLANE; ++s) {
    const uint32_t a = wave_sum((c[s] + TILE - 1) >> sT), b = wave_sum((c[s] + WTILE - 1) >> sW),
                   d = wave_sum(c[s] * nch);
    if (ln == 0) {
      red[wave][AGG_IT + s] = a;
      red[wave][AGG_IW + s] = b;
      red[wave][AGG_CAP + s] = d;
    }
    v += c[s];
    pairs += c[s] ? 1u : 0u;
  }
  const uint32_t wv = wave_sum(v), wp = wave_sum(pairs), wl = wave_sum(leaf ? v : 0u);
  if (ln == 0) {
    red[wave][AGG_V] = wv;
    red[wave][AGG_PAIRS] = wp;
    red[wave][AGG_LEAFV] = wl;
  }
  __syncthreads();
  if (tid < AGG_N) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < SCAN_WG / 64; ++w) t += red[w][tid];
    aux[(size_t)blockIdx.x * AGG_STRIDE + tid] = t;
  }
}

__global__ __launch_bounds__(SCAN_WG) void k_scan_alloc(TraceArgs A, LevelArgs L, const uint32_t* __restrict__ aux,
                                                       uint32_t lanecap, uint32_t out_parity_base,
                                                       unsigned long long* stats, int level, uint32_t* err) {
  __shared__ uint32_t s_pre[AGG_N], s_tot[AGG_N];
  __shared__ uint32_t wsum[SCAN_WG / 64][2 * NLANE];
  const int tid = threadIdx.x, wave = tid >> 6, ln = tid & 63;
  const int G = gridDim.x, b = blockIdx.x;
  const size_t row = (size_t)L.maxln + 1;
  // partials of the workgroups before this one, and of all: wave 0, one
  // workgroup row per lane (all of a row's loads in flight together)
  if (wave == 0) {
    uint32_t pre[AGG_N], tot[AGG_N];
#pragma unroll
    for (int i = 0; i < AGG_N; ++i) pre[i] = tot[i] = 0u;
    for (int r0 = 0; r0 < G; r0 += 64) {
      const int r = r0 + ln;
      uint32_t x[AGG_N];
#pragma unroll
      for (int i = 0; i < AGG_N; ++i) x[i] = r < G ? aux[(size_t)r * AGG_STRIDE + i] : 0u;
#pragma unroll
      for (int i = 0; i < AGG_N; ++i) {
        tot[i] += x[i];
        pre[i] += r < b ? x[i] : 0u;
      }
    }
#pragma unroll
    for (int i = 0; i < AGG_N; ++i) {
      const uint32_t a = wave_sum(pre[i]), t = wave_sum(tot[i]);
      if (ln == 0) {
        s_pre[i] = a;
        s_tot[i] = t;
      }
    }
  }
  __syncthreads();
  const bool block_mode =
      !L.two_level && (unsigned long long)s_tot[AGG_V] >=
                          (unsigned long long)BLOCK_MODE_RAYS_PER_PAIR * (s_tot[AGG_PAIRS] ? s_tot[AGG_PAIRS] : 1u);
  const uint32_t itile = block_mode ? TILE : WTILE;
  const uint32_t ishift = (uint32_t)__builtin_ctz(itile);
  const int ia = block_mode ? AGG_IT : AGG_IW;

  const int k = b * SCAN_WG + tid;
  uint32_t c[NLANE], nch = 0;
#pragma unroll
  for (int s = 0; s < NLANE; ++s) c[s] = 0u;
  if (k < L.nl) {
#pragma unroll
    for (int s = 0; s < NLANE; ++s) c[s] = L.icnt[s * row + k];
    nch = aux[SCAN_MAXG * AGG_STRIDE + k];
  }
  // workgroup exclusive scan of 16 values (items, capacity per lane)
  uint32_t ex[2 * NLANE];
#pragma unroll
  for (int j = 0; j < 2 * NLANE; ++j) {
    const uint32_t tv = j < NLANE ? (c[j] + itile - 1) >> ishift : c[j - NLANE] * nch;
    uint32_t x = tv;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off, 64);
      if (ln >= off) x += y;
    }
    ex[j] = x - tv;
    if (ln == 63) wsum[wave][j] = x;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2 * NLANE; ++j) {
    uint32_t w = j < NLANE ? s_pre[ia + j] : s_pre[AGG_CAP + j - NLANE];
    for (int q = 0; q < wave; ++q) w += wsum[q][j];
    ex[j] += w;
  }
  if (k < L.nl) {
#pragma unroll
    for (int s = 0; s < NLANE; ++s) L.iprefix_w[s * row + k] = ex[s];
    if (nch) {
      int4 c4, g4[4];
      int gpc[4];
      load_targets(A, L.first + k, c4, g4, gpc);
      uint32_t jj = 0;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int tn = scan_target(c4, g4, gpc, t, L.two_level != 0);
        if (tn >= 0) {
#pragma unroll
          for (int s = 0; s < NLANE; ++s)
            A.qoff[(size_t)tn * NLANE + s] = out_parity_base + (uint32_t)s * lanecap + ex[NLANE + s] + jj * c[s];
          jj++;
        }
      }
    }
  }
  if (b == G - 1 && tid == 0) {
    bool ovf = false;
    unsigned long long items = 0, need = 0;
    for (int s = 0; s < NLANE; ++s) {
      if (s_tot[AGG_CAP + s] > lanecap) ovf = true;
      items += s_tot[ia + s];
      need = max(need, (unsigned long long)s_tot[AGG_CAP + s]);
    }
    for (int s = 0; s < NLANE; ++s) L.iprefix_w[s * row + L.nl] = ovf ? 0u : s_tot[ia + s];
    *L.mode_w = block_mode ? MODE_BLOCK : MODE_WAVE;
    if (ovf) atomicOr(err, 1u);
    if (stats) {
      atomicAdd(stats + STAT_V, (unsigned long long)s_tot[AGG_V]);
      if (level < 16) {
        atomicAdd(stats + STAT_LV0 + level, (unsigned long long)s_tot[AGG_V]);
        atomicAdd(stats + STAT_LEAF0 + level, (unsigned long long)s_tot[AGG_LEAFV]);
        atomicAdd(stats + STAT_ITEMS0 + level, items);
      }
      atomicMax(stats + STAT_PEAKQ, need * NLANE);
    }
  }
}

}  // namespace pt
