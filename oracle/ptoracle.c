/*
 * ptoracle.c -- CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference's hot-path arithmetic, used ONLY by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker.  The product path (libptcore.so) never links, loads or calls it.
 *
 * It restates, with the parity decisions of SURVEY.md §8(a):
 *   intersectRayTriangle         src/cudaRenderer.cu:217-270   -> pto_tri (the build's
 *                                Baldwin-Weber form) / pto_tri_ref (literal)
 *   kernelMergeIntersections     cu:515-540 (min over candidates) -> pto_closest_brute
 *   rayIntersectSingle leaf loop cu:1144-1169                   -> pto_closest_bvh
 *   kernelPrimaryRays            cu:312-376                     -> camera_ray
 *   leaf hit record              cu:1201-1291                   -> shade_normal
 *   kernelDirectLightRays        cu:380-481                     -> NEE in path_radiance
 *   kernelProcessIntersections   cu:544-664                     -> BSDF in path_radiance
 *   kernelAccumulate / Reconstruct cu:705-742                   -> accumulation order
 *   PathTracer::start_raytracing / worker_thread / raytrace_tile / raytrace_pixel
 *                                src/pathtracer.cpp:183-213, 499-558 -> pto_render
 *                                (32x32 tiles pulled from a shared queue by N threads)
 * The RNG is Philox4x32-10 (Salmon et al. 2011), not curand XORWOW: the
 * reference's streams are not reproducible without the CUDA toolkit
 * (parity unpinned for RNG streams).
 *
 * PT_FLAG_REF_ARITH selects the reference kernels' literal arithmetic
 * (pto_tri_ref, camera_dir_ref, nee_ref and the REF branches of
 * path_radiance): every expression of cu:217-270, 347-354, 416-446, 570-653
 * and 1205-1234 in source order, with the build's single contraction
 * convention (a*b + c is fma(a, b, c), so dot = fma(a.z, b.z, fma(a.y, b.y,
 * a.x*b.x)) and cross = (fma(a.y, b.z, -(a.z*b.y)), ...) -- what nvcc's
 * default --fmad=true makes of cuda_util.h; the exact contraction nvcc chose
 * is unknowable here), double-literal comparisons evaluated exactly, and
 * rsqrtf (an approximate hardware instruction on NVIDIA) as 1/sqrtf.
 *
 * Every float expression keeps the operation order of the HIP kernels and is
 * compiled with -ffp-contract=off, so per-sample radiance is bit-identical.
 */
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/pt_api.h"

typedef struct {
  float x, y, z;
} v3;
static inline v3 mk(float x, float y, float z) {
  v3 r = {x, y, z};
  return r;
}
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 scl(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 mulv(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
/* dot and cross as FMA chains, exactly as ptmath.h */
static inline float dot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 cross(v3 a, v3 b) {
  return mk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline float len3(v3 a) { return sqrtf(dot(a, a)); }
static inline v3 nrm(v3 a) {
  float inv = 1.0f / sqrtf(dot(a, a));
  return scl(a, inv);
}
static inline v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

/* ---- Philox4x32-10 --------------------------------------------------------- */
typedef struct {
  uint32_t v[4];
} u4;
static inline uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
static u4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  u4 o = {{c0, c1, c2, c3}};
  return o;
}
static inline float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }
static inline u4 rng(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t vertex, uint32_t call) {
  return philox(pixel, sample, vertex * 2u + call, 0x50540000u, seed, 0x2545F491u);
}
/* second NEE sample of a vertex under the reference schedule: own stream */
static inline u4 rng_nee2(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t vertex) {
  return philox(pixel, sample, vertex * 2u, 0x50540001u, seed, 0x2545F491u);
}
void pto_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t* out) {
  u4 r = philox(c0, c1, c2, c3, k0, k1);
  memcpy(out, r.v, 16);
}

/* sin/cos of 2*pi*u: quadrant reduction on u, Taylor polynomials on [0, pi/2) */
static void sincos2pi(float u, float* s, float* c) {
  float x4 = u * 4.0f;
  float q = floorf(x4);
  float f = x4 - q;
  float th = f * 1.57079637f;
  float t2 = th * th;
  /* Horner steps as FMAs (ptmath.h sincos2pi) */
  float sp = -2.50521084e-08f;
  sp = fmaf(sp, t2, 2.75573192e-06f);
  sp = fmaf(sp, t2, -1.98412698e-04f);
  sp = fmaf(sp, t2, 8.33333333e-03f);
  sp = fmaf(sp, t2, -1.66666667e-01f);
  sp = fmaf(sp, t2, 1.0f);
  float sn = sp * th;
  float cp = 2.08767570e-09f;
  cp = fmaf(cp, t2, -2.75573192e-07f);
  cp = fmaf(cp, t2, 2.48015873e-05f);
  cp = fmaf(cp, t2, -1.38888889e-03f);
  cp = fmaf(cp, t2, 4.16666667e-02f);
  cp = fmaf(cp, t2, -0.5f);
  cp = fmaf(cp, t2, 1.0f);
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
void pto_sincos2pi(float u, float* s, float* c) { sincos2pi(u, s, c); }

/* ---- primitive tests -------------------------------------------------------- */
/* dot products as FMA chains, exactly as trace.hip:
 * fdot(a, b) = fma(a.z, b.z, fma(a.y, b.y, a.x * b.x)) */
static inline float fdot(float ax, float ay, float az, float bx, float by, float bz) {
  return fmaf(az, bz, fmaf(ay, by, ax * bx));
}
/* The build's triangle test (the default arithmetic; trace.hip bw_test): the
 * reference's plane hit + inside test (intersectRayTriangle, cu:217-270) on
 * the triangle's Baldwin-Weber transform (Baldwin & Weber, JCGT 5(3) 2016).
 * bw_rows restates pt_device.hip's record builder: from the fp32 vertices in
 * double, e1 = B - A, e2 = C - A, n = e1 x e2, k = the axis of n's largest
 * magnitude, and rows U, V, W (value = a x + b y + c z + d) with W the plane
 * scaled by 1 / n_k; each entry one double division rounded to fp32. */
static void bw_rows(const float* q, float out[12]) {
  const double A[3] = {q[0], q[1], q[2]}, B[3] = {q[4], q[5], q[6]}, C[3] = {q[8], q[9], q[10]};
  double e1[3], e2[3], n[3], r[12];
  for (int k = 0; k < 3; ++k) {
    e1[k] = B[k] - A[k];
    e2[k] = C[k] - A[k];
  }
  n[0] = e1[1] * e2[2] - e1[2] * e2[1];
  n[1] = e1[2] * e2[0] - e1[0] * e2[2];
  n[2] = e1[0] * e2[1] - e1[1] * e2[0];
  const double an = n[0] * A[0] + n[1] * A[1] + n[2] * A[2];
  if (fabs(n[0]) > fabs(n[1]) && fabs(n[0]) > fabs(n[2])) {
    const double x = n[0];
    r[0] = 0; r[1] = e2[2] / x; r[2] = -e2[1] / x; r[3] = (C[1] * A[2] - C[2] * A[1]) / x;
    r[4] = 0; r[5] = -e1[2] / x; r[6] = e1[1] / x; r[7] = -(B[1] * A[2] - B[2] * A[1]) / x;
    r[8] = 1; r[9] = n[1] / x; r[10] = n[2] / x; r[11] = -an / x;
  } else if (fabs(n[1]) > fabs(n[2])) {
    const double y = n[1];
    r[0] = -e2[2] / y; r[1] = 0; r[2] = e2[0] / y; r[3] = (C[2] * A[0] - C[0] * A[2]) / y;
    r[4] = e1[2] / y; r[5] = 0; r[6] = -e1[0] / y; r[7] = -(B[2] * A[0] - B[0] * A[2]) / y;
    r[8] = n[0] / y; r[9] = 1; r[10] = n[2] / y; r[11] = -an / y;
  } else {
    const double z = n[2];
    r[0] = e2[1] / z; r[1] = -e2[0] / z; r[2] = 0; r[3] = (C[0] * A[1] - C[1] * A[0]) / z;
    r[4] = -e1[1] / z; r[5] = e1[0] / z; r[6] = 0; r[7] = -(B[0] * A[1] - B[1] * A[0]) / z;
    r[8] = n[0] / z; r[9] = n[1] / z; r[10] = 1; r[11] = -an / z;
  }
  for (int i = 0; i < 12; ++i) out[i] = (float)r[i];
}
/* every triangle's rows (12 floats per primitive; spheres: zeros) */
static float* bw_table(const pt_scene_desc* S) {
  float* t = (float*)calloc((size_t)(S->n_prims > 0 ? S->n_prims : 1) * 12, sizeof(float));
  for (int i = 0; i < S->n_prims; ++i) {
    uint32_t meta;
    memcpy(&meta, &S->prims[i].q[3], 4);
    if ((meta >> 28) != PT_PRIM_SPHERE) bw_rows(S->prims[i].q, t + (size_t)12 * i);
  }
  return t;
}
static inline float bw_plane(const float* R, v3 o) { return fmaf(R[2], o.z, fmaf(R[1], o.y, fmaf(R[0], o.x, R[3]))); }
/* t = -W(o) / W(d); a hit iff t >= tlo and the plane hit P = o + t d (FMAs)
 * has u = U(P) >= 0, v = V(P) >= 0, u + v <= 1 (trace.hip bw_test,
 * PT_BW_POINT) */
static float pto_tri(v3 o, v3 d, const float* M, float tlo) {
  const float t = -bw_plane(M + 8, o) / fdot(M[8], M[9], M[10], d.x, d.y, d.z);
  if (!(t >= tlo)) return -1.0f;
  const v3 P = mk(fmaf(t, d.x, o.x), fmaf(t, d.y, o.y), fmaf(t, d.z, o.z));
  const float u = bw_plane(M, P);
  const float v = bw_plane(M + 4, P);
  /* unordered compares: a NaN u or v (t = +-inf, a ray parallel to the plane) misses */
  if (!(u >= 0.0f) || !(v >= 0.0f) || !(u + v <= 1.0f)) return -1.0f;
  return t + 0.0f; /* (-0 -> +0) */
}
/* intersectRayTriangle, cu:217-270, literally (PT_FLAG_REF_ARITH): N and
 * dot(N, v0) per call, edge k rejected when dot(N, cross(e_k, P - v_k)) < 0,
 * the parallel test |N.d| < 1e-6 against the double literal. */
static float pto_tri_ref(v3 o, v3 d, const float* q) {
  v3 v0 = mk(q[0], q[1], q[2]), v1 = mk(q[4], q[5], q[6]), v2 = mk(q[8], q[9], q[10]);
  v3 v0v1 = sub(v1, v0), v0v2 = sub(v2, v0);
  v3 N = cross(v0v1, v0v2);
  float ndd = dot(N, d);
  if ((double)fabsf(ndd) < 1e-6) return -1.0f;
  float dd = dot(N, v0);
  float t = (dd - dot(N, o)) / ndd;
  if (t < 0.0f) return -1.0f;
  v3 P = mk(fmaf(t, d.x, o.x), fmaf(t, d.y, o.y), fmaf(t, d.z, o.z));
  if (dot(N, cross(sub(v1, v0), sub(P, v0))) < 0.0f) return -1.0f;
  if (dot(N, cross(sub(v2, v1), sub(P, v1))) < 0.0f) return -1.0f;
  if (dot(N, cross(sub(v0, v2), sub(P, v2))) < 0.0f) return -1.0f;
  return t == 0.0f ? 0.0f : t;
}
/* nearest root with t >= tlo (the ray's t_min, >= 0) */
static float pto_sphere(v3 o, v3 d, const float* q, float tlo) {
  v3 oc = mk(o.x - q[0], o.y - q[1], o.z - q[2]);
  float b = fdot(oc.x, oc.y, oc.z, d.x, d.y, d.z);
  float cc = fdot(oc.x, oc.y, oc.z, oc.x, oc.y, oc.z) - q[5];
  float disc = fmaf(b, b, -cc);
  if (disc < 0.0f) return -1.0f;
  float sq = sqrtf(disc);
  float t0 = -b - sq, t1 = -b + sq;
  float t = (t0 >= tlo) ? t0 : t1;
  if (t < tlo) return -1.0f;
  return t == 0.0f ? 0.0f : t;
}
/* t of primitive i's hit with t >= tlo, or -1 (bw: the scene's rows, bw_table) */
static inline float prim_test(const pt_scene_desc* S, const float* bw, int i, v3 o, v3 d, int ref, float tlo) {
  const pt_prim* p = &S->prims[i];
  uint32_t meta;
  memcpy(&meta, &p->q[3], 4);
  if ((meta >> 28) == PT_PRIM_SPHERE) return pto_sphere(o, d, p->q, tlo);
  if (!ref) return pto_tri(o, d, bw + (size_t)12 * i, tlo);
  const float t = pto_tri_ref(o, d, p->q);
  return t >= tlo ? t : -1.0f;
}
/* A ray record: o.xyz, tmax, d.xyz, t_min (BVHAccel's Ray::min_t; pt_api.h
 * pt_intersect).  Valid hits have t in [max(t_min, 0), tmax], both ends
 * inclusive (triangle.cpp:189 rejects t < r.min_t and t > r.max_t). */
static inline float ray_tlo(const float* ray) { return ray[7] > 0.0f ? ray[7] : 0.0f; }
static inline uint64_t key(float t, uint32_t prim) {
  uint32_t b;
  memcpy(&b, &t, 4);
  return ((uint64_t)b << 32) | prim;
}

/* Closest hit by brute force: min over all primitives of (t, index), t <= tmax. */
static uint64_t closest_brute(const pt_scene_desc* S, const float* bw, const float* ray, int ref) {
  v3 o = mk(ray[0], ray[1], ray[2]), d = mk(ray[4], ray[5], ray[6]);
  float tmax = ray[3], tlo = ray_tlo(ray);
  uint64_t best = PT_HIT_NONE;
  for (int i = 0; i < S->n_prims; ++i) {
    float t = prim_test(S, bw, i, o, d, ref, tlo);
    if (t >= 0.0f && t <= tmax) {
      uint64_t k = key(t, (uint32_t)i);
      if (k < best) best = k;
    }
  }
  return best;
}

/* Closest hit through the wide BVH, depth-first with a stack.  The box test is
 * done in double precision on the (outward-rounded) fp32 boxes. */
static int box_hit_d(const pt_node* nd, int c, v3 o, v3 d, double tmax) {
  double t0 = 0.0, t1 = tmax;
  const float* mn[3] = {nd->bmin_x, nd->bmin_y, nd->bmin_z};
  const float* mx[3] = {nd->bmax_x, nd->bmax_y, nd->bmax_z};
  double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
  for (int a = 0; a < 3; ++a) {
    double lo = mn[a][c], hi = mx[a][c];
    if (dd[a] == 0.0) {
      if (oo[a] < lo || oo[a] > hi) return 0;
      continue;
    }
    double inv = 1.0 / dd[a];
    double ta = (lo - oo[a]) * inv, tb = (hi - oo[a]) * inv;
    if (ta > tb) {
      double x = ta;
      ta = tb;
      tb = x;
    }
    if (ta > t0) t0 = ta;
    if (tb < t1) t1 = tb;
    if (t0 > t1) return 0;
  }
  return 1;
}
static uint64_t closest_bvh(const pt_scene_desc* S, const float* bw, const float* ray, int ref) {
  v3 o = mk(ray[0], ray[1], ray[2]), d = mk(ray[4], ray[5], ray[6]);
  float tmax = ray[3], tlo = ray_tlo(ray);
  uint64_t best = PT_HIT_NONE;
  int stack[256];
  int sp = 0;
  stack[sp++] = 0;
  while (sp) {
    const pt_node* nd = &S->nodes[stack[--sp]];
    if (nd->prim_count > 0) {
      for (int k = 0; k < nd->prim_count; ++k) {
        int i = nd->prim_start + k;
        float t = prim_test(S, bw, i, o, d, ref, tlo);
        if (t >= 0.0f && t <= tmax) {
          uint64_t kk = key(t, (uint32_t)i);
          if (kk < best) best = kk;
        }
      }
      continue;
    }
    double lim = tmax;
    if (best != PT_HIT_NONE) {
      uint32_t b = (uint32_t)(best >> 32);
      float bt;
      memcpy(&bt, &b, 4);
      if (bt < lim) lim = bt;
    }
    for (int c = 0; c < 4; ++c)
      if (nd->child[c] >= 0 && sp < 256 && box_hit_d(nd, c, o, d, lim)) stack[sp++] = nd->child[c];
  }
  return best;
}

uint64_t pto_closest_brute(const pt_scene_desc* S, const float* ray) {
  float* bw = bw_table(S);
  const uint64_t h = closest_brute(S, bw, ray, 0);
  free(bw);
  return h;
}
uint64_t pto_closest_bvh(const pt_scene_desc* S, const float* ray) {
  float* bw = bw_table(S);
  const uint64_t h = closest_bvh(S, bw, ray, 0);
  free(bw);
  return h;
}

void pto_intersect_ex(const pt_scene_desc* S, const float* rays, int n, uint64_t* hits, int use_bvh, uint32_t flags) {
  const int ref = (flags & PT_FLAG_REF_ARITH) != 0;
  float* bw = bw_table(S);
  for (int i = 0; i < n; ++i)
    hits[i] = use_bvh ? closest_bvh(S, bw, rays + 8 * i, ref) : closest_brute(S, bw, rays + 8 * i, ref);
  free(bw);
}
void pto_intersect(const pt_scene_desc* S, const float* rays, int n, uint64_t* hits, int use_bvh) {
  pto_intersect_ex(S, rays, n, hits, use_bvh, 0);
}

/* Level-synchronous breadth-first traversal statistics: R rays, V (ray, node)
 * visits, per level, with the same conservative box test as pto_closest_bvh but
 * no culling by the best hit (an upper bound of the GPU's V). */
void pto_bfs_visits(const pt_scene_desc* S, const float* rays, int n, uint64_t* level_visits, int max_levels) {
  for (int l = 0; l < max_levels; ++l) level_visits[l] = 0;
  for (int i = 0; i < n; ++i) {
    const float* r = rays + 8 * i;
    if (r[3] < 0.0f) continue;
    v3 o = mk(r[0], r[1], r[2]), d = mk(r[4], r[5], r[6]);
    int stack[256];
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
      int id = stack[--sp];
      const pt_node* nd = &S->nodes[id];
      if (nd->level < max_levels) level_visits[nd->level]++;
      if (nd->prim_count > 0) continue;
      for (int c = 0; c < 4; ++c)
        if (nd->child[c] >= 0 && sp < 256 && box_hit_d(nd, c, o, d, r[3])) stack[sp++] = nd->child[c];
    }
  }
}

/* ---- path tracing ------------------------------------------------------------ */
typedef struct {
  const pt_scene_desc* S;
  const float* bw; /* bw_table(S) */
  int W, H, spp, max_bounces, sample_offset, use_bvh;
  uint32_t seed, flags;
  int tile, rank, nranks;
  const uint32_t* owned_tiles;
  int n_owned_tiles;
  atomic_int next_tile;
  float* img;
  atomic_ulong rays;
} job_t;

static uint64_t trace(const job_t* J, v3 o, v3 d, float tmax) {
  float r[8] = {o.x, o.y, o.z, tmax, d.x, d.y, d.z, 0.0f};
  const int ref = (J->flags & PT_FLAG_REF_ARITH) != 0;
  return J->use_bvh ? closest_bvh(J->S, J->bw, r, ref) : closest_brute(J->S, J->bw, r, ref);
}

/* Radiance of sample s of pixel g: the per-path state machine of k_shade. */
/* One NEE sample toward the scene light, kernelDirectLightRays cu:380-481.
 * weight < 0: unweighted (default schedule); else the reference schedule's
 * per-sample weight (cu:2515-2533). */
/* sel: the low byte of the sample's first Philox word; with several lights
 * (S->lights, n_lights > 1) it picks light k = floor(sel n / 256), whose
 * contribution is weighted by 256 / cnt_k, the inverse of its probability
 * (shade.hip nee_sample). */
static int nee_sample(const pt_scene_desc* S, uint32_t flags, v3 T, v3 alb, v3 n, v3 pt, float ux, float uy,
                      float weight, v3* C, v3* sw, float* stmax, uint32_t sel) {
  const float INV_PI = 0.318309886183790671f, EPS = 1e-3f;
  const pt_light* Lp = &S->light;
  float lw = 1.0f;
  if (S->n_lights > 1) {
    const uint32_t nl = (uint32_t)S->n_lights, k = ((sel & 0xFFu) * nl) >> 8;
    const uint32_t cnt = (256u * (k + 1u) + nl - 1u) / nl - (256u * k + nl - 1u) / nl;
    lw = 256.0f / (float)cnt;
    Lp = &S->lights[k];
  }
  const pt_light LL = *Lp;
  const pt_light* const L = &LL;
  if (L->type == PT_LIGHT_AREA) {
    float sx = ux - 0.5f, sy = uy - 0.5f;
    v3 pos = ld3(L->position), dx = ld3(L->dim_x), dy = ld3(L->dim_y);
    v3 lpt = mk(fmaf(sy, dy.x, fmaf(sx, dx.x, pos.x)), fmaf(sy, dy.y, fmaf(sx, dx.y, pos.y)),
                fmaf(sy, dy.z, fmaf(sx, dx.z, pos.z)));
    v3 dv = sub(lpt, pt);
    float sq = dot(dv, dv);
    float dist = sqrtf(sq);
    float inv = 1.0f / dist;
    v3 w = mk(dv.x * inv, dv.y * inv, dv.z * inv);
    /* AreaLight::sample_L, light.cpp:81-92: cosTheta = dot(d, direction) of
     * the unnormalised d, pdf = sqDist / (area |cosTheta|), one-sided;
     * PT_FLAG_EXACT_LIGHT_PDF: the normalised cosine (solid-angle pdf) */
    float cu = dot(dv, ld3(L->direction));
    float cosl = cu * inv;
    float cosn = dot(n, w);
    if (dist > 1e-2f && cosl < -1e-2f && cosn > 0.0f) {
      /* cosn / pdf, pdf = sq / (area * -cosTheta), as one division */
      float lc = (flags & PT_FLAG_EXACT_LIGHT_PDF) ? cosl : cu;
      float scale = ((cosn * (L->area * -lc)) / sq) * INV_PI;
      if (weight >= 0.0f) scale = scale * weight;
      if (lw != 1.0f) scale = scale * lw;
      *C = scl(mulv(mulv(T, alb), ld3(L->radiance)), scale);
      *sw = w;
      *stmax = dist - EPS;
      return 1;
    }
  } else if (L->type == PT_LIGHT_POINT) {
    v3 dv = sub(ld3(L->position), pt);
    float sq = dot(dv, dv);
    float dist = sqrtf(sq);
    float inv = 1.0f / dist;
    v3 w = mk(dv.x * inv, dv.y * inv, dv.z * inv);
    float cosn = dot(n, w);
    if (dist > 1e-2f && cosn > 0.0f) {
      float scale = cosn * INV_PI;
      if (weight >= 0.0f) scale = scale * weight;
      if (lw != 1.0f) scale = scale * lw;
      *C = scl(mulv(mulv(T, alb), ld3(L->radiance)), scale);
      *sw = w;
      *stmax = dist - EPS;
      return 1;
    }
  } else if (L->type == PT_LIGHT_DIRECTIONAL) {
    /* DirectionalLight::sample_L, light.cpp:18-24: wi = dirToLight, pdf 1,
     * infinitely far */
    v3 w = ld3(L->direction);
    float cosn = dot(n, w);
    if (cosn > 0.0f) {
      float scale = cosn * INV_PI;
      if (weight >= 0.0f) scale = scale * weight;
      if (lw != 1.0f) scale = scale * lw;
      *C = scl(mulv(mulv(T, alb), ld3(L->radiance)), scale);
      *sw = w;
      *stmax = INFINITY;
      return 1;
    }
  } else if (L->type == PT_LIGHT_HEMISPHERE) {
    /* InfiniteHemisphereLight::sample_L, light.cpp:36-44: a uniform direction
     * of the upper (+y) hemisphere, pdf 1 / (2 pi): cos / pdf * albedo / pi =
     * 2 cos albedo */
    float sn, cs;
    sincos2pi(uy, &sn, &cs);
    float rr = sqrtf(fmaxf(0.0f, fmaf(-ux, ux, 1.0f)));
    v3 w = mk(rr * cs, ux, rr * sn);
    float cosn = dot(n, w);
    if (cosn > 0.0f) {
      float scale = cosn * 2.0f;
      if (weight >= 0.0f) scale = scale * weight;
      if (lw != 1.0f) scale = scale * lw;
      *C = scl(mulv(mulv(T, alb), ld3(L->radiance)), scale);
      *sw = w;
      *stmax = INFINITY;
      return 1;
    }
  }
  return 0;
}

/* PT_FLAG_REF_ARITH NEE: kernelDirectLightRays, cu:416-446, REAL_TIME.  The
 * shadow ray's tmax: the light counts when its closest hit t > maxT - 1e-3 in
 * double (cu:1279), so it is occluded by any t <= D = dist - 1e-3, i.e. by any
 * fp32 t <= D rounded down. */
static float rd_f32(double D) {
  float f = (float)D;
  if ((double)f > D) f = nextafterf(f, -INFINITY);
  return f;
}
static int nee_ref(const pt_scene_desc* S, v3 T, v3 alb, v3 n, v3 pt, float ux, float uy, float weight, v3* C,
                   v3* sw, float* stmax) {
  const float MULT = (float)0.3183; /* BSDF_DIFFUSE_MULTIPLIER, cu:272 */
  const float wgt = weight >= 0.0f ? weight : 1.0f;
  if (S->light.type == PT_LIGHT_AREA) {
    float sx = ux - 0.5f, sy = uy - 0.5f;
    v3 pos = ld3(S->light.position), dx = ld3(S->light.dim_x), dy = ld3(S->light.dim_y);
    /* e.position + sampleX * e.dim_x + sampleY * e.dim_y */
    v3 lpt = mk(fmaf(sy, dy.x, fmaf(sx, dx.x, pos.x)), fmaf(sy, dy.y, fmaf(sx, dx.y, pos.y)),
                fmaf(sy, dy.z, fmaf(sx, dx.z, pos.z)));
    v3 d = sub(lpt, pt);
    float cosTheta = dot(d, ld3(S->light.direction));
    float sqDist = dot(d, d);
    float dist = sqrtf(sqDist);
    v3 w = scl(d, 1.0f / dist); /* d / dist (cuda_util.h: a * (1 / s)) */
    float pdf = sqDist / (S->light.area * fabsf(cosTheta));
    float fpdf = fabsf(dot(n, w)) / pdf;
    if ((double)dist > 1e-2 && (double)fabsf(cosTheta) > 1e-2) {
      *C = scl(scl(mulv(scl(mulv(T, alb), fpdf), ld3(S->light.radiance)), MULT), wgt);
      *sw = w;
      *stmax = rd_f32((double)dist - 1e-3);
      return 1;
    }
    return 0;
  }
  if (S->light.type == PT_LIGHT_POINT) { /* no reference counterpart: fpdf = |n.w| */
    v3 d = sub(ld3(S->light.position), pt);
    float dist = sqrtf(dot(d, d));
    v3 w = scl(d, 1.0f / dist);
    float fpdf = fabsf(dot(n, w));
    if ((double)dist > 1e-2) {
      *C = scl(scl(mulv(scl(mulv(T, alb), fpdf), ld3(S->light.radiance)), MULT), wgt);
      *sw = w;
      *stmax = rd_f32((double)dist - 1e-3);
      return 1;
    }
  }
  return 0;
}

/* Camera ray through sensor point (ssx = row + jitter, ssy = column + jitter)
 * of a W x H frame, kernelPrimaryRays cu:338-354 (direction; the origin is
 * the camera's). */
static v3 camera_dir(const pt_camera* cam, int W, int H, float ssx, float ssy, int refa) {
  float kx = ssy / (float)W - 0.5f;
  float ky = -(ssx / (float)H - 0.5f);
  float kz = 1.0f;
  float len = sqrtf(fmaf(kz, kz, fmaf(ky, ky, kx * kx)));
  kx = kx / len;
  ky = ky / len;
  kz = kz / len;
  v3 Lf = ld3(cam->left), Up = ld3(cam->up), K = ld3(cam->look_at);
  if (refa) { /* cu:347-354: k = k / length(k); dir = k.x left + k.y up + k.z lookAt */
    v3 k = mk(ssy / (float)W - 0.5f, -(ssx / (float)H - 0.5f), 1.0f);
    k = scl(k, 1.0f / len3(k));
    return mk(dot(k, mk(Lf.x, Up.x, K.x)), dot(k, mk(Lf.y, Up.y, K.y)), dot(k, mk(Lf.z, Up.z, K.z)));
  }
  v3 k = mk(kx, ky, kz);
  return nrm(mk(dot(k, mk(Lf.x, Up.x, K.x)), dot(k, mk(Lf.y, Up.y, K.y)), dot(k, mk(Lf.z, Up.z, K.z))));
}
/* The camera ray of sensor point (ssx, ssy) as out[6] = o.xyz, d.xyz. */
void pto_camera_ray(const pt_camera* cam, int W, int H, float ssx, float ssy, uint32_t flags, float* out) {
  v3 d = camera_dir(cam, W, H, ssx, ssy, (flags & PT_FLAG_REF_ARITH) != 0);
  out[0] = cam->origin[0];
  out[1] = cam->origin[1];
  out[2] = cam->origin[2];
  out[3] = d.x;
  out[4] = d.y;
  out[5] = d.z;
}

static v3 path_radiance(const job_t* J, uint32_t g, uint32_t s, uint64_t* nrays) {
  const pt_scene_desc* S = J->S;
  const float EPS = 1e-3f;
  const int ref_sched = (J->flags & PT_FLAG_REF_SCHEDULE) != 0;
  const int max_bounces = ref_sched ? 2 : J->max_bounces;
  uint32_t row = g / (uint32_t)J->W, col = g - row * (uint32_t)J->W;
  u4 u = rng(J->seed, g, s, 0, 0);
  /* camera ray, cu:338-354 */
  float ssx = (float)row + u01(u.v[0]);
  float ssy = (float)col + u01(u.v[1]);
  const int refa = (J->flags & PT_FLAG_REF_ARITH) != 0;
  v3 d = camera_dir(&S->camera, J->W, J->H, ssx, ssy, refa);
  v3 o = ld3(S->camera.origin);
  v3 T = mk(1.0f, 1.0f, 1.0f), L = mk(0.0f, 0.0f, 0.0f);
  int spec = 0;
  for (uint32_t vtx = 1;; ++vtx) {
    uint64_t h = trace(J, o, d, INFINITY);
    (*nrays)++;
    if (h == PT_HIT_NONE) {
      /* reference quirk (i): kernelUpdateSSImage writes 0 for a path whose
       * intersection became invalid (cu:679-698) */
      if (J->flags & PT_FLAG_REF_DROP_ON_MISS) L = mk(0.0f, 0.0f, 0.0f);
      break;
    }
    uint32_t tb = (uint32_t)(h >> 32), prim = (uint32_t)h;
    float t;
    memcpy(&t, &tb, 4);
    /* cu:1205 its.pt = r->o + r->d * t */
    /* hit point and offsets as FMAs in both arithmetics (shade.hip) */
    v3 P = mk(fmaf(d.x, t, o.x), fmaf(d.y, t, o.y), fmaf(d.z, t, o.z));
    const float* q = S->prims[prim].q;
    uint32_t meta;
    memcpy(&meta, &q[3], 4);
    v3 ns;
    if ((meta >> 28) == PT_PRIM_SPHERE) {
      ns = nrm(mk(P.x - q[0], P.y - q[1], P.z - q[2]));
    } else {
      const pt_prim_shading* sh = &S->shading[prim];
      v3 n0 = ld3(sh->n0), n1 = ld3(sh->n1), n2 = ld3(sh->n2);
      /* flat: the three normals identical to the bit (pt_load_scene's test) */
      if (!refa && memcmp(sh->n0, sh->n1, 3 * sizeof(float)) == 0 && memcmp(sh->n1, sh->n2, 3 * sizeof(float)) == 0) {
        /* flat triangle: the barycentric blend is a positive multiple of n0 */
        ns = nrm(n0);
      } else { /* barycentric shading normal, cu:1213-1221 */
        v3 A = mk(q[0], q[1], q[2]), B = mk(q[4], q[5], q[6]), Cv = mk(q[8], q[9], q[10]);
        float total = len3(cross(sub(A, B), sub(B, Cv)));
        float bC = len3(cross(sub(A, P), sub(B, P))) / total;
        float bA = len3(cross(sub(B, P), sub(Cv, P))) / total;
        float bB = len3(cross(sub(Cv, P), sub(A, P))) / total;
        { /* cu:1221 normalize(bA * n0 + bB * n1 + bC * n2), FMA chains in both arithmetics */
          v3 bw = mk(bA, bB, bC);
          ns = nrm(mk(dot(bw, mk(n0.x, n1.x, n2.x)), dot(bw, mk(n0.y, n1.y, n2.y)), dot(bw, mk(n0.z, n1.z, n2.z))));
        }
      }
    }
    int front = dot(ns, d) < 0.0f;
    v3 n = front ? ns : mk(-ns.x, -ns.y, -ns.z);
    /* cu:1224 its.pt += -r->d * 1e-3 */
    v3 pt = mk(fmaf(-d.x, EPS, P.x), fmaf(-d.y, EPS, P.y), fmaf(-d.z, EPS, P.z));
    pt_bsdf Bv = S->bsdfs[meta & 0x0FFFFFFFu];
    const pt_bsdf* Bs = &Bv;
    int emitter = 0;
    if (refa) {
      /* cu:1243 (without REAL_TIME) its.light = radiance * importance + light;
       * an emission BSDF is a diffuse one with albedo = radiance (cu:1705-1711) */
      v3 rad = Bv.type == PT_BSDF_EMISSION ? ld3(Bv.albedo) : mk(0.0f, 0.0f, 0.0f);
      if (!(J->flags & PT_FLAG_NO_EMISSION)) {
        L = mk(fmaf(rad.x, T.x, L.x), fmaf(rad.y, T.y, L.y), fmaf(rad.z, T.z, L.z));
        emitter = rad.x != 0.0f || rad.y != 0.0f || rad.z != 0.0f; /* cu:436 */
      }
      if (Bv.type == PT_BSDF_EMISSION) Bv.type = PT_BSDF_DIFFUSE;
      /* cu:1713-1719: a delta BSDF read through MirrorBSDF -- over a GlassBSDF
       * reflectance = (roughness, reflectance.r, reflectance.g), over a
       * RefractionBSDF (roughness, transmittance.r, transmittance.g)
       * (bsdf.h:138-139 against 180-182 and 206-210) */
      if (Bv.type == PT_BSDF_GLASS || Bv.type == PT_BSDF_REFRACTION) {
        float c1 = Bv.type == PT_BSDF_GLASS ? Bv.albedo[0] : Bv.transmittance[0];
        float c2 = Bv.type == PT_BSDF_GLASS ? Bv.albedo[1] : Bv.transmittance[1];
        Bv.albedo[0] = Bv.roughness;
        Bv.albedo[1] = c1;
        Bv.albedo[2] = c2;
        Bv.type = PT_BSDF_MIRROR;
      }
    }
    if (!refa && Bs->type == PT_BSDF_EMISSION) {
      if (!(J->flags & PT_FLAG_NO_EMISSION) && (vtx == 1 || spec)) L = add(L, mulv(T, ld3(Bs->albedo)));
      break;
    }
    u4 r = rng(J->seed, g, s, vtx, 0);
    v3 dpdu, dpdv;
    if (J->flags & PT_FLAG_REF_GUIDE) { /* reference quirk (ii), cu:572-574 */
      v3 guide = ((double)n.y < 1e-4) ? mk(0.0f, 1.0f, 0.0f) : mk(1.0f, 0.0f, 0.0f);
      dpdu = nrm(cross(guide, n));
      dpdv = nrm(cross(dpdu, n));
    } else if (!refa) {
      /* branchless orthonormal basis (Duff et al., JCGT 6(1), 2017), shade.hip
       * PT_ONB_DUFF */
      float sg = copysignf(1.0f, n.z);
      float a = -(1.0f / (sg + n.z));
      float b = (n.x * n.y) * a;
      float sx = sg * n.x;
      dpdu = mk(fmaf(sx * n.x, a, 1.0f), sg * b, -sx);
      dpdv = mk(b, fmaf(n.y * n.y, a, sg), -n.y);
    } else {
      v3 guide = (fabsf(n.x) < 0.9f) ? mk(1.0f, 0.0f, 0.0f) : mk(0.0f, 1.0f, 0.0f);
      dpdu = nrm(cross(guide, n));
      dpdv = cross(n, dpdu);
    }
    v3 dn, on;
    if (Bs->type == PT_BSDF_DIFFUSE) {
      v3 alb = ld3(Bs->albedo);
      /* NEE: one sample, or 2, 2, 1 at vertices 1, 2, 3 (reference schedule) */
      const int nee = emitter ? 0 : (ref_sched && vtx <= 2u) ? 2 : 1;
      int have_sh[2] = {0, 0};
      v3 C[2] = {{0, 0, 0}, {0, 0, 0}}, sw[2] = {{0, 0, 1}, {0, 0, 1}};
      float stmax[2] = {-1.0f, -1.0f};
      for (int k = 0; k < nee; ++k) {
        float ux = u01(r.v[0]), uy = u01(r.v[1]);
        uint32_t sel = r.v[0];
        if (k == 1) {
          u4 r2 = rng_nee2(J->seed, g, s, vtx);
          ux = u01(r2.v[0]);
          uy = u01(r2.v[1]);
          sel = r2.v[0];
        }
        float weight = ref_sched ? (nee == 2 ? 0.5f : 1.0f) : -1.0f;
        have_sh[k] = refa ? nee_ref(S, T, alb, n, pt, ux, uy, weight, &C[k], &sw[k], &stmax[k])
                          : nee_sample(S, J->flags, T, alb, n, pt, ux, uy, weight, &C[k], &sw[k], &stmax[k], sel);
      }
      float x, y, z, sn, cs;
      sincos2pi(u01(r.v[3]), &sn, &cs);
      if (J->flags & PT_FLAG_COSINE_DIFFUSE) {
        float u2 = u01(r.v[2]);
        float rr = sqrtf(u2);
        x = rr * cs;
        y = rr * sn;
        z = sqrtf(fmaxf(0.0f, 1.0f - u2));
      } else {
        z = fabsf(2.0f * u01(r.v[2]) - 1.0f);
        float rr = sqrtf(fmaxf(0.0f, 1.0f - z * z));
        x = rr * cs;
        y = rr * sn;
      }
      /* cu:631-637, not normalised (the default basis is orthonormal) */
      dn = mk(fmaf(y, dpdv.x, fmaf(x, dpdu.x, n.x * z)), fmaf(y, dpdv.y, fmaf(x, dpdu.y, n.y * z)),
              fmaf(y, dpdv.z, fmaf(x, dpdu.z, n.z * z)));
      if (J->flags & PT_FLAG_COSINE_DIFFUSE) {
        T = mulv(T, alb);
      } else {
        float c = fabsf(dot(dn, n));
        T = mk(((T.x * c) * alb.x) * 2.0f, ((T.y * c) * alb.y) * 2.0f, ((T.z * c) * alb.z) * 2.0f);
      }
      on = mk(fmaf(n.x, EPS, pt.x), fmaf(n.y, EPS, pt.y), fmaf(n.z, EPS, pt.z)); /* cu:593 */
      spec = 0;
      for (int k = 0; k < nee; ++k) {
        if (!have_sh[k]) continue;
        uint64_t hs = trace(J, pt, sw[k], stmax[k]);
        (*nrays)++;
        if (hs == PT_HIT_NONE) L = add(L, C[k]);
      }
    } else if (Bs->type == PT_BSDF_MIRROR) {
      if (refa) {
        /* cu:1234 wi in the local frame; cu:643-650 wo = (-wi.x, -wi.y, wi.z) */
        v3 md = mk(-d.x, -d.y, -d.z);
        v3 wi = nrm(mk(dot(dpdu, md), dot(dpdv, md), dot(n, md)));
        float wx = -wi.x, wy = -wi.y, wz = wi.z;
        dn = mk(fmaf(wy, dpdv.x, fmaf(wx, dpdu.x, n.x * wz)), fmaf(wy, dpdv.y, fmaf(wx, dpdu.y, n.y * wz)),
                fmaf(wy, dpdv.z, fmaf(wx, dpdu.z, n.z * wz)));
        on = mk(fmaf(n.x, EPS, pt.x), fmaf(n.y, EPS, pt.y), fmaf(n.z, EPS, pt.z));
      } else {
        float dd = dot(d, n);
        dn = nrm(sub(d, scl(n, 2.0f * dd)));
        on = mk(fmaf(n.x, EPS, pt.x), fmaf(n.y, EPS, pt.y), fmaf(n.z, EPS, pt.z));
      }
      T = mulv(T, ld3(Bs->albedo));
      spec = 1;
    } else { /* glass, refraction */
      float ior = Bs->ior;
      float eta = front ? (1.0f / ior) : ior;
      float cosi = -dot(d, n);
      float sin2t = (eta * eta) * (1.0f - cosi * cosi);
      int refl = 1;
      float cost = 0.0f;
      if (sin2t < 1.0f) {
        cost = sqrtf(1.0f - sin2t);
        float r0 = (1.0f - ior) / (1.0f + ior);
        r0 = r0 * r0;
        float c = front ? cosi : cost;
        float m = 1.0f - c;
        float F = fmaf(1.0f - r0, ((m * m) * (m * m)) * m, r0);
        refl = u01(r.v[0]) < F; /* the vertex's first word: no NEE at glass */
      }
      if (refl) {
        float dd = dot(d, n);
        dn = nrm(sub(d, scl(n, 2.0f * dd)));
        T = mulv(T, ld3(Bs->albedo));
        on = mk(fmaf(n.x, EPS, pt.x), fmaf(n.y, EPS, pt.y), fmaf(n.z, EPS, pt.z));
      } else {
        dn = nrm(add(scl(d, eta), scl(n, eta * cosi - cost)));
        T = mulv(T, ld3(Bs->transmittance));
        on = mk(fmaf(-n.x, EPS, P.x), fmaf(-n.y, EPS, P.y), fmaf(-n.z, EPS, P.z));
      }
      spec = 1;
    }
    if (!(vtx <= (uint32_t)max_bounces && (T.x > 0.0f || T.y > 0.0f || T.z > 0.0f))) break;
    o = on;
    d = dn;
  }
  return L;
}

static void* worker(void* arg) {
  job_t* J = (job_t*)arg;
  const int T = J->tile;
  const int ntx = (J->W + T - 1) / T;
  uint64_t nrays = 0;
  for (;;) {
    int k = atomic_fetch_add(&J->next_tile, 1);
    if (k >= J->n_owned_tiles) break;
    int t = (int)J->owned_tiles[k];
    int ty = t / ntx, tx = t % ntx;
    for (int r = ty * T; r < (ty + 1) * T && r < J->H; ++r)
      for (int c = tx * T; c < (tx + 1) * T && c < J->W; ++c) {
        uint32_t g = (uint32_t)(r * J->W + c);
        float ax = 0.0f, ay = 0.0f, az = 0.0f;
        for (int s = 0; s < J->spp; ++s) {
          v3 l = path_radiance(J, g, (uint32_t)(J->sample_offset + s), &nrays);
          ax = ax + l.x;
          ay = ay + l.y;
          az = az + l.z;
        }
        float* px = J->img + (size_t)g * 4;
        px[0] = ax;
        px[1] = ay;
        px[2] = az;
        px[3] = 1.0f;
      }
  }
  atomic_fetch_add(&J->rays, nrays);
  return NULL;
}

/* Render spp samples of the pixels owned by (rank, nranks) and write the SUM of
 * their radiance (not divided) into sums[W*H*4]; other pixels are left as is.
 * Returns the number of rays cast. */
uint64_t pto_render(const pt_scene_desc* S, int W, int H, int spp, int max_bounces, uint32_t seed,
                    int sample_offset, uint32_t flags, int tile, int rank, int nranks, int nthreads,
                    int use_bvh, float* sums) {
  if (tile <= 0) tile = 32;
  if (nranks <= 0) nranks = 1;
  if (nthreads <= 0) nthreads = 1;
  int ntx = (W + tile - 1) / tile, nty = (H + tile - 1) / tile;
  uint32_t* owned = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(ntx * nty + 1));
  int no = 0;
  for (int t = 0; t < ntx * nty; ++t)
    if (t % nranks == rank) owned[no++] = (uint32_t)t;
  job_t J;
  J.S = S;
  float* bw = bw_table(S);
  J.bw = bw;
  J.W = W;
  J.H = H;
  J.spp = spp;
  J.max_bounces = max_bounces;
  J.sample_offset = sample_offset;
  J.use_bvh = use_bvh;
  J.seed = seed;
  J.flags = flags;
  J.tile = tile;
  J.rank = rank;
  J.nranks = nranks;
  J.owned_tiles = owned;
  J.n_owned_tiles = no;
  atomic_init(&J.next_tile, 0);
  J.img = sums;
  atomic_init(&J.rays, 0);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, worker, &J);
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  free(th);
  free(owned);
  free(bw);
  return (uint64_t)atomic_load(&J.rays);
}

/* Radiance of one sample (tests of the per-sample state machine). */
void pto_sample(const pt_scene_desc* S, int W, int H, int max_bounces, uint32_t seed, uint32_t flags, uint32_t g,
                uint32_t s, float* out3) {
  job_t J;
  memset(&J, 0, sizeof(J));
  J.S = S;
  float* bw = bw_table(S);
  J.bw = bw;
  J.W = W;
  J.H = H;
  J.max_bounces = max_bounces;
  J.seed = seed;
  J.flags = flags;
  J.use_bvh = 1;
  uint64_t nr = 0;
  v3 l = path_radiance(&J, g, s, &nr);
  free(bw);
  out3[0] = l.x;
  out3[1] = l.y;
  out3[2] = l.z;
}

/* One pixel's estimate as the context reports it (pt_get_image): the fp32 sum
 * of its spp samples in sample order, divided by spp; *rays += rays cast.
 * The per-pixel estimator of the Scotty3D-surface CPU renderer
 * (oracle/scotty_cpu.cpp, PathTracer::raytrace_pixel, pathtracer.cpp:499-508). */
float* pto_bw_table(const pt_scene_desc* S) { return bw_table(S); }
void pto_free(void* p) { free(p); }
/* bw: pto_bw_table(S), built once by the caller (the Scotty3D-surface
 * estimator calls this per pixel) */
void pto_pixel_bw(const pt_scene_desc* S, const float* bw, int W, int H, int spp, int max_bounces, uint32_t seed,
                  uint32_t flags, int sample_offset, uint32_t g, float* out4, uint64_t* rays) {
  job_t J;
  memset(&J, 0, sizeof(J));
  J.S = S;
  J.bw = bw;
  J.W = W;
  J.H = H;
  J.max_bounces = max_bounces;
  J.seed = seed;
  J.flags = flags;
  J.use_bvh = 1;
  uint64_t nr = 0;
  float ax = 0.0f, ay = 0.0f, az = 0.0f;
  for (int s = 0; s < spp; ++s) {
    v3 l = path_radiance(&J, g, (uint32_t)(sample_offset + s), &nr);
    ax = ax + l.x;
    ay = ay + l.y;
    az = az + l.z;
  }
  const float ns = (float)(spp > 0 ? spp : 1);
  out4[0] = ax / ns;
  out4[1] = ay / ns;
  out4[2] = az / ns;
  out4[3] = 1.0f;
  if (rays) *rays += nr;
}
void pto_pixel(const pt_scene_desc* S, int W, int H, int spp, int max_bounces, uint32_t seed, uint32_t flags,
               int sample_offset, uint32_t g, float* out4, uint64_t* rays) {
  float* bw = bw_table(S);
  pto_pixel_bw(S, bw, W, H, spp, max_bounces, seed, flags, sample_offset, g, out4, rays);
  free(bw);
}

/* ---- display filter: kernelMedianFilter, cu:773-842 --------------------------
 * Per channel: remove the maximum of the 3x3 neighbourhood three times (max
 * search from 0.0 with >=, the last index wins, the removed value becomes 0)
 * and keep the fourth; out-of-frame neighbours are 1.0; alpha 1. */
void pto_median(const float* in, float* out, int w, int h) {
  for (int r = 0; r < h; ++r)
    for (int c = 0; c < w; ++c) {
      float v[3][9];
      int k = 0;
      for (int dr = -1; dr <= 1; ++dr)
        for (int dc = -1; dc <= 1; ++dc, ++k) {
          int rr = r + dr, cc = c + dc;
          for (int ch = 0; ch < 3; ++ch)
            v[ch][k] = (rr >= 0 && rr < h && cc >= 0 && cc < w) ? in[((size_t)rr * w + cc) * 4 + ch] : 1.0f;
        }
      float* o = out + ((size_t)r * w + c) * 4;
      for (int ch = 0; ch < 3; ++ch) {
        float res = 0.0f;
        for (int it = 0; it < 4; ++it) {
          int im = 0;
          float m = 0.0f;
          for (int j = 0; j < 9; ++j)
            if (v[ch][j] >= m) {
              m = v[ch][j];
              im = j;
            }
          if (it < 3)
            v[ch][im] = 0.0f;
          else
            res = v[ch][im];
        }
        o[ch] = res;
      }
      o[3] = 1.0f;
    }
}
