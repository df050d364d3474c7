// Wavefront shading kernels: camera rays, per-vertex shade (NEE + BSDF sample),
// progressive accumulation (gfx950).
//
// Restates the reference kernels with the parity decisions of SURVEY §8(a):
//   kernelPrimaryRays            src/cudaRenderer.cu:312-376  -> k_camera
//   kernelDirectLightRays        cu:380-481                   -> NEE part of k_shade
//   kernelProcessIntersections   cu:544-664                   -> BSDF part of k_shade
//   leaf hit construction        cu:1201-1291                 -> hit record in k_shade
//   kernelUpdateSSImage / kernelReconstructImage / kernelAccumulate
//                                cu:666-742                   -> k_accum
// Deviations (all mirrored by oracle/ptoracle.c): per-path radiance
// accumulator (a miss keeps the light gathered so far); orthonormal frame with
// a guide that cannot be parallel to n; counter-based Philox streams instead of
// curand XORWOW; glass, spheres and point lights; parametric bounce count; and
// in the default arithmetic: normalised camera / BSDF directions, a
// one-sided emitter (cosl < -0.01: lights emit along their direction; cu:440
// tests |cosTheta|), NEE only toward the front of the shading normal (cu:429
// takes |n.w|), 1/pi = 0.3183099 (cu:272: 0.3183), the flat-triangle normal
// shortcut.  PT_FLAG_REF_ARITH (template parameter REFA) replaces each of
// these arithmetic choices by the reference's literal expression (see
// shade_vertex, nee_sample, camera_dir).
#include "trace.h"

namespace pt {

constexpr uint32_t F_EXT = 1u;     // extension ray pending in slot p
constexpr uint32_t F_SHADOW = 2u;  // shadow ray pending in slot N + p
constexpr uint32_t F_SPEC = 4u;    // last scattering was specular
constexpr uint32_t F_SHADOW2 = 8u; // second shadow ray pending in slot 2N + p (reference schedule)
__device__ __forceinline__ uint32_t sh_bit(int s) { return s ? F_SHADOW2 : F_SHADOW; }
constexpr float INV_PI = 0.318309886183790671f;
constexpr float REF_DIFFUSE_MULT = 0.3183f;  // BSDF_DIFFUSE_MULTIPLIER, cu:272
constexpr float EPS = 1e-3f;  // reference offsets (cu:593, 1224)
constexpr int SHADE_REC = 5;  // float4 per hit-shading record (ShadeArgs::shade)
constexpr uint32_t SHADE_SMOOTH = 1u << 27;  // shading-record meta bit: a triangle with distinct vertex normals
// The diffuse sampling frame (default arithmetic) is Duff et al.'s
// branchless orthonormal basis with the sampled direction left unnormalised
// (round 4, +4.2 % CBempty; rounds 1-3 used a guide-vector frame and a
// normalised direction).  A flat triangle's shading record holds its
// normalised normal in the first 16 B (host-computed, bit-identical to the
// device's normalize; round 4, +2 % CBempty).
constexpr uint32_t ERR_KERNARG = 2u;  // pt_ctx::d_err bit: k_path_leaf's kernel-argument layout check failed

// slot regions of the tail compaction (ShadeArgs::compact)
constexpr uint32_t CREGIONS = 64;

// A BSDF on the device: pt_bsdf's fields, then the dielectric's 1 / ior and
// Fresnel base reflectance r0 = ((1 - ior) / (1 + ior))^2, both computed on the
// host by IEEE fp32 division (pt_load_scene): the same bits as the kernels'
// correctly rounded division sequences (rcp_rn, div_rn) gave for an index of
// refraction in the normal range, without their ~17 instructions at every
// glass vertex -- a wave with one glass lane ran them all.
struct alignas(16) BsdfRec {
  int32_t type;
  float albedo[3];
  float transmittance[3];
  float ior;
  float roughness;
  float inv_ior;
  float r0;
  float pad;
};
static_assert(sizeof(BsdfRec) == 48, "three 16-B loads per BSDF");

struct ShadeArgs {
  float4* ray;  // ray records (trace.h): ext ray of path p in slot p, shadow ray s in slot (1+s)N + p
  float4* ps0;  // T.xyz, flags | vertex << 8
  float4* ps1;  // L.xyz, path index P (wavefront slots) / pixel (k_path_leaf output)
  float4* ps2;  // pending shadow contribution
  float4* ps3;  // pending contribution of the second shadow ray (PT_FLAG_REF_SCHEDULE)
  const float4* __restrict__ prims;
  // per-primitive hit-shading record, 5 float4 (80 B, two 64-B sectors):
  // {A, meta}{B, n0.x}{C, n0.y}{n0.z, n1}{n2, flat} -- vertices and vertex
  // normals of a triangle (a sphere: {centre, meta}), built by pt_load_scene
  // from pt_prim + pt_prim_shading so a hit gathers 80 B instead of 96
  const float4* __restrict__ shade;
  const BsdfRec* __restrict__ bsdfs;  // (BsdfRec: pt_bsdf + the dielectric's host-computed constants)
  const uint32_t* __restrict__ pix_of;
  pt_light light;
  pt_camera cam;
  const pt_light* lights;  // pt_scene_desc.lights on the device when n_lights > 1
  uint32_t n_lights;
  const float* cbox;  // single-leaf scenes: the leaf's primitive-pair boxes (8 floats each)
  int nclus;
  uint32_t sph_cl;  // the clusters that hold a sphere (bit c: cluster c; spheres are clusters of one)
  uint32_t N, npix, sample_base, seed;
  udiv div_npix, div_width;  // p / npix, pixel / width (N and width * height < 2^30)
  int width, height, max_bounces;
  uint32_t flags;
  TraceArgs A;                   // fused root pass (camera/shade push into the root's target queues)
  RootTable T;                   // its inline leaves and targets
  // path regeneration of the wavefront: the N slots run the M paths of a chunk
  // (P = j * npix + q: sample j of owned pixel q); a slot whose path ends
  // writes res[P] and starts the next unstarted path
  float4* res;        // per-path radiance of the chunk
  uint32_t M;         // paths in the chunk
  // k_path_leaf's path grabs: chunk size, paths per region, regions, the
  // regions' counters (re-read from the kernel-argument segment at each grab)
  uint32_t grab_chunk, grab_region, grab_nreg;
  uint32_t* grab_work;
  // paths are handed out in blocks of POOL_BLOCK consecutive paths (one sample
  // of 256 owned pixels): block c comes from dispenser c % POOLS
  uint4* wstate;      // per workgroup: {next, end} of its current block, live slots after its last pass,
                      // vertices shaded
  uint32_t* pool;     // POOLS dispensers, CSTRIDE apart (block counters)
  int passes;         // vertices per path at most (max_bounces + 2)
  unsigned long long* rcount;    // rays entering the traversal (RCOUNT_SLOTS counters)
  uint32_t kshift;    // record-order key of a path: its hit primitive >> kshift (shade_slot)
  // Tail compaction (pt_render): once every path of the chunk has started and
  // few slots are still live, one shade pass writes the continuing paths'
  // state and new rays densely into a second set of buffers, and the passes
  // after it launch ceil(n / 256) workgroups over slots [0, *nact) of that
  // set.  The output slots come from CREGIONS counters, not one: workgroup b
  // takes them from region b % CREGIONS, whose slots start at the sum of the
  // lower regions' bounds creg[] (each region's live + unstarted paths after
  // the last pass, k_live_sum: an upper bound on what it writes); one counter
  // bumped by every workgroup cost a 73k-workgroup compaction pass 1.3 ms of
  // serialised atomics.  What a region leaves of its bound is a hole of free
  // slots (k_compact_slots).  A shade workgroup's time is
  // mostly a chain of dependent memory round trips, nearly the same for 20
  // live slots as for 256, so without this the tail's passes cost almost as
  // much as full ones.  The slots are read from the *_in buffers (and S.ray)
  // and written to ps0..ps3 and A.ray: the same arrays except in a
  // compaction pass.
  const float4* ps0_in;
  const float4* ps1_in;
  const float4* ps2_in;
  const float4* ps3_in;
  uint32_t* compact;     // compaction pass: the regions' slot counters (CREGIONS, zeroed); else null
  const uint32_t* creg;  // compaction pass: the regions' slot bounds (k_live_sum)
  const uint32_t* nact;  // after a compaction: paths are in slots [0, *nact); else null ([0, N))
  // dense pass (set by the host while the chunk has more than 2 N paths of
  // work left, i.e. nearly every slot is live): k_shade_push issues every
  // slot's loads at entry, in the same memory round trip as its workgroup's
  // wstate word, instead of after the barrier that shares the wstate
  uint32_t dense;
  // diagnostic build only (PT_SHADE_TIMING=1, env PT_SHADE_TIMING): per-phase
  // cycle sums of k_shade_push, 64 x 16 counters; else null
  unsigned long long* tprof;
  // k_path_leaf's first acc_blocks workgroups (0: none) sum the previous
  // launch's per-path results -- acc_npix pixels x acc_spp samples in acc_res
  // -- into acc_dst[acc_slot[q]], k_accum's sums (pipelined frames, pt_render)
  const float4* acc_res;
  float4* acc_dst;
  const uint32_t* acc_slot;
  uint32_t acc_npix, acc_spp, acc_blocks;
};

#ifndef PT_SHADE_TIMING
#define PT_SHADE_TIMING 0
#endif
// k_shade_push phase stamps (PT_SHADE_TIMING): thread 0's s_memtime right
// after the workgroup barriers that close each phase
#if PT_SHADE_TIMING
#define SHADE_STAMP(k) \
  if (tid == 0) t_[k] = __builtin_amdgcn_s_memtime()
#else
#define SHADE_STAMP(k)
#endif

__device__ __forceinline__ f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ f3 xyz(float4 a) { return mk(a.x, a.y, a.z); }

// Camera ray of path p (pixel g = pix_of[p % npix], sample sample_base + p / npix).
// REFA: cu:347-354 literally -- k / length(k) as k * (1 / length(k))
// (cuda_util.h operator/), dir = k.x left + k.y up + k.z lookAt as an FMA chain,
// not normalised.
template <bool KR>
__device__ __forceinline__ pt_camera cam_of(const ShadeArgs& S);
// KR: the camera re-read from the kernel-argument segment (cam_of)
template <bool M64 = false, bool REFA = false, bool KR = false>
__device__ __forceinline__ f3 camera_dir(const ShadeArgs& S, uint32_t p, uint32_t& g) {
  const uint32_t j = udiv_q(p, S.div_npix), q = p - j * S.npix;
  g = S.pix_of[q];
  const uint32_t row = udiv_q(g, S.div_width), col = g - row * (uint32_t)S.width;
  const uint32_t s = S.sample_base + j;
  const u4 u = rng<M64>(S.seed, g, s, 0, 0);
  // cu:338-354: ss = (x + u, y + v); k = ((ss.y/W)-.5, -((ss.x/H)-.5), 1) / |k|
  float ssx = (float)row + u01(u.x);
  float ssy = (float)col + u01(u.y);
  // (div_rn: IEEE's quotient for ssx, ssy = 0 or >= 2^-24 over W, H >= 1)
  float kx = div_rn(ssy, (float)S.width) - 0.5f;
  float ky = -(div_rn(ssx, (float)S.height) - 0.5f);
  float kz = 1.0f;
  const pt_camera cam = cam_of<KR>(S);
  const f3 L = ld3(cam.left), U = ld3(cam.up), K = ld3(cam.look_at);
  if constexpr (REFA) {
    const float inv = 1.0f / length(mk(kx, ky, kz));
    const f3 k = mk(kx, ky, kz) * inv;
    return mk(dot(k, mk(L.x, U.x, K.x)), dot(k, mk(L.y, U.y, K.y)), dot(k, mk(L.z, U.z, K.z)));
  }
  // (sqrt_rn / div_rn / normalize_u give IEEE's bits here: len^2 >= 1, the
  // numerators are 0 or >= 2^-25 in magnitude, |dir| ~ 1)
  float len = sqrt_rn(dot(mk(kx, ky, kz), mk(kx, ky, kz)));
  kx = div_rn(kx, len);
  ky = div_rn(ky, len);
  kz = div_rn(kz, len);
  const f3 k = mk(kx, ky, kz);
  f3 dir = mk(dot(k, mk(L.x, U.x, K.x)), dot(k, mk(L.y, U.y, K.y)), dot(k, mk(L.z, U.z, K.z)));
  return normalize_u(dir);
}

// Path state between vertices (ps0/ps1/ps2 in memory, registers in k_path_leaf).
struct PathState {
  f3 T;            // throughput
  uint32_t flags;  // F_* | vertex << 8
  f3 L;            // radiance gathered so far
  uint32_t g;      // pixel
};
struct RayV {
  f3 o, d;
  float tmax;
};

// One NEE sample toward the scene light (kernelDirectLightRays, cu:380-481)
// from the shading point pt with normal n; (ux, uy) pick the point on an area
// light.  weight < 0: unweighted (the default schedule); otherwise the
// reference schedule's per-sample weight (cu:2515-2533).
// KR: re-read the light from the kernel argument segment at each use (only in
// a kernel whose first argument is the ShadeArgs): its 16 SGPRs are then not
// held, and spilled, across the whole path loop.
// (KR = true only in k_path_leaf, which checks the layout at launch)
template <bool KR>
__device__ __forceinline__ pt_light light_of(const ShadeArgs& S) {
  if (KR) {
    const CPTR(char) kp = (const CPTR(char))__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));  // not loop-invariant for the compiler
    constexpr int NW = sizeof(pt_light) / 4;
    const CPTR(uint32_t) q = (const CPTR(uint32_t))(kp + offsetof(ShadeArgs, light));
    uint32_t w[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) w[i] = q[i];
    pt_light L;
    __builtin_memcpy(&L, w, sizeof(L));
    return L;
  }
  return S.light;
}
// The camera likewise (k_path_leaf: its 12 floats are not held in SGPRs --
// and spilled to VGPR lanes -- across the path loop; the launch check covers
// it too)
template <bool KR>
__device__ __forceinline__ pt_camera cam_of(const ShadeArgs& S) {
  if (KR) {
    const CPTR(char) kp = (const CPTR(char))__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));  // not loop-invariant for the compiler
    constexpr int NW = sizeof(pt_camera) / 4;
    const CPTR(uint32_t) q = (const CPTR(uint32_t))(kp + offsetof(ShadeArgs, cam));
    uint32_t w[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) w[i] = q[i];
    pt_camera c;
    __builtin_memcpy(&c, w, sizeof(c));
    return c;
  }
  return S.cam;
}
// Shadow-ray tmax of the reference (cu:446, 1279): the light counts when the
// closest hit t satisfies t > maxT - 1e-3 in double precision (1e-3 is a
// double literal), i.e. the ray is occluded by any hit t <= D = maxT - 1e-3,
// and for an fp32 t that is t <= D rounded down to fp32.
__device__ __forceinline__ float ref_shadow_tmax(float dist) { return __double2float_rd((double)dist - 1e-3); }

// sel: the low byte of the sample's first Philox word (u01 uses the top 24
// bits), which picks one of several lights (pt_scene_desc.lights): light k =
// floor(sel n / 256) with probability cnt_k / 256, weighted by 256 / cnt_k.
// XL: the extended light model (several lights, directional and hemisphere
// lights; pt_scene_desc.lights) -- its own kernel variants, so the one-light
// kernels keep their registers (the selection and the two light types cost
// k_shade_push its 8th wave when compiled into it)
template <bool KR = false, bool REFA = false, bool XL = false>
__device__ __forceinline__ bool nee_sample(const ShadeArgs& S, const f3 T, const f3 alb, const f3 n, const f3 pt,
                                           float ux, float uy, float weight, f3& C, RayV& r, uint32_t sel = 0u) {
  pt_light L = light_of<KR>(S);
  float lw = 1.0f;
  if (XL && S.n_lights > 1u) {
    const uint32_t nl = S.n_lights, k = ((sel & 0xFFu) * nl) >> 8;
    const uint32_t cnt = (256u * (k + 1u) + nl - 1u) / nl - (256u * k + nl - 1u) / nl;
    lw = 256.0f / (float)cnt;
    L = S.lights[k];
  }
  if (REFA && L.type == PT_LIGHT_AREA) {
    // kernelDirectLightRays, cu:416-446, expression for expression
    const float sx = ux - 0.5f, sy = uy - 0.5f;
    const f3 pos = ld3(L.position), dx = ld3(L.dim_x), dy = ld3(L.dim_y);
    const f3 lpt = mk(__builtin_fmaf(sy, dy.x, __builtin_fmaf(sx, dx.x, pos.x)),
                      __builtin_fmaf(sy, dy.y, __builtin_fmaf(sx, dx.y, pos.y)),
                      __builtin_fmaf(sy, dy.z, __builtin_fmaf(sx, dx.z, pos.z)));
    const f3 dv = lpt - pt;
    const float cosTheta = dot(dv, ld3(L.direction));  // unnormalised d (cu:422)
    const float sq = dot(dv, dv);
    const float dist = sqrtf(sq);
    const f3 w = dv * (1.0f / dist);
    const float pdf = sq / (L.area * fabsf(cosTheta));
    const float fpdf = fabsf(dot(n, w)) / pdf;
    // dist > 1e-2 and |cosTheta| > 1e-2 are double comparisons: for fp32
    // values the same as against 1e-2f (no float lies in (1e-2f, 0.01])
    if (dist > 1e-2f && fabsf(cosTheta) > 1e-2f) {
      C = mulv(mulv(T, alb) * fpdf, ld3(L.radiance)) * REF_DIFFUSE_MULT * (weight >= 0.0f ? weight : 1.0f);
      r.o = pt;
      r.d = w;
      r.tmax = ref_shadow_tmax(dist);
      return true;
    }
    return false;
  }
  if (REFA && L.type == PT_LIGHT_POINT) {
    // (the reference has no point light, cu:1741 reinterpret_casts every light
    // to an AreaLight): the same expression with fpdf = |n.w|
    const f3 dv = ld3(L.position) - pt;
    const float sq = dot(dv, dv);
    const float dist = sqrtf(sq);
    const f3 w = dv * (1.0f / dist);
    const float fpdf = fabsf(dot(n, w));
    if (dist > 1e-2f) {
      C = mulv(mulv(T, alb) * fpdf, ld3(L.radiance)) * REF_DIFFUSE_MULT * (weight >= 0.0f ? weight : 1.0f);
      r.o = pt;
      r.d = w;
      r.tmax = ref_shadow_tmax(dist);
      return true;
    }
    return false;
  }
  if (L.type == PT_LIGHT_AREA) {
    const float sx = ux - 0.5f, sy = uy - 0.5f;
    const f3 pos = ld3(L.position), dx = ld3(L.dim_x), dy = ld3(L.dim_y);
    const f3 lpt = mk(__builtin_fmaf(sy, dy.x, __builtin_fmaf(sx, dx.x, pos.x)),
                      __builtin_fmaf(sy, dy.y, __builtin_fmaf(sx, dx.y, pos.y)),
                      __builtin_fmaf(sy, dy.z, __builtin_fmaf(sx, dx.z, pos.z)));
    const f3 dv = lpt - pt;
    const float sq = dot(dv, dv);
    // (sqrt_rn / rcp_rn: IEEE's bits for sq >= 2^-96; a smaller sq fails
    // dist > 1e-2 either way and its w is never used)
    const float dist = sqrt_rn(sq);
    const float inv = rcp_rn(dist);
    const f3 w = mk(dv.x * inv, dv.y * inv, dv.z * inv);
    // AreaLight::sample_L (light.cpp:81-92): cosTheta = dot(d, direction) of
    // the UNnormalised d, pdf = sqDist / (area |cosTheta|), radiance only when
    // cosTheta < 0 (one-sided); the pdf is the solid-angle pdf times dist.
    // PT_FLAG_EXACT_LIGHT_PDF takes the normalised cosine instead.
    const float cu = dot(dv, ld3(L.direction));
    const float cosl = cu * inv;
    const float cosn = dot(n, w);
    if (dist > 1e-2f && cosl < -1e-2f && cosn > 0.0f) {
      // cosn / pdf with pdf = sq / (area * -cosTheta), as one division
      // (1/pi from an SGPR: as a literal the compiler paired it with another
      // product in a v_pk_mul_f32 and spilled the VGPR pair holding it)
      float inv_pi = INV_PI;
      asm volatile("" : "+s"(inv_pi));
      const float lc = (S.flags & PT_FLAG_EXACT_LIGHT_PDF) ? cosl : cu;
      float scale = ((cosn * (L.area * -lc)) / sq) * inv_pi;
      if (weight >= 0.0f) scale = scale * weight;
      if (XL && lw != 1.0f) scale = scale * lw;
      C = mulv(mulv(T, alb), ld3(L.radiance)) * scale;
      r.o = pt;
      r.d = w;
      r.tmax = dist - EPS;
      return true;
    }
  } else if (L.type == PT_LIGHT_POINT) {
    const f3 dv = ld3(L.position) - pt;
    const float sq = dot(dv, dv);
    const float dist = sqrt_rn(sq);  // (as above)
    const float inv = rcp_rn(dist);
    const f3 w = mk(dv.x * inv, dv.y * inv, dv.z * inv);
    const float cosn = dot(n, w);
    if (dist > 1e-2f && cosn > 0.0f) {
      float scale = cosn * INV_PI;
      if (weight >= 0.0f) scale = scale * weight;
      if (XL && lw != 1.0f) scale = scale * lw;
      C = mulv(mulv(T, alb), ld3(L.radiance)) * scale;
      r.o = pt;
      r.d = w;
      r.tmax = dist - EPS;
      return true;
    }
  } else if (XL && L.type == PT_LIGHT_DIRECTIONAL) {
    // DirectionalLight::sample_L (light.cpp:18-24): wi = dirToLight, pdf 1,
    // distToLight infinite
    const f3 w = ld3(L.direction);
    const float cosn = dot(n, w);
    if (cosn > 0.0f) {
      float scale = cosn * INV_PI;
      if (weight >= 0.0f) scale = scale * weight;
      if (lw != 1.0f) scale = scale * lw;
      C = mulv(mulv(T, alb), ld3(L.radiance)) * scale;
      r.o = pt;
      r.d = w;
      r.tmax = __builtin_inff();
      return true;
    }
  } else if (XL && L.type == PT_LIGHT_HEMISPHERE) {
    // InfiniteHemisphereLight::sample_L (light.cpp:36-44): a uniform
    // direction of the upper (+y) hemisphere (cos theta = ux, phi = 2 pi uy),
    // pdf 1 / (2 pi): cos / pdf * albedo / pi = 2 cos albedo
    float sn, cs;
    sincos2pi(uy, &sn, &cs);
    const float rr = sqrt_rn(fmaxf(0.0f, __builtin_fmaf(-ux, ux, 1.0f)));
    const f3 w = mk(rr * cs, ux, rr * sn);
    const float cosn = dot(n, w);
    if (cosn > 0.0f) {
      float scale = cosn * 2.0f;
      if (weight >= 0.0f) scale = scale * weight;
      if (lw != 1.0f) scale = scale * lw;
      C = mulv(mulv(T, alb), ld3(L.radiance)) * scale;
      r.o = pt;
      r.d = w;
      r.tmax = __builtin_inff();
      return true;
    }
  }
  return false;
}

// One path vertex (restated from cu:380-664, see header): resolves the NSH
// shadow rays of the previous vertex (C[s] added when unoccluded), shades the
// extension hit (prim != PT_PRIM_NONE at distance t along ext), and produces
// the next extension ray and/or shadow rays with their pending contributions.
// NSH = 2 only under PT_FLAG_REF_SCHEDULE (NEE samples 2, 2, 1 per vertex).
// REFA (PT_FLAG_REF_ARITH): the hit record, NEE and BSDF sample are the
// reference's expressions (cu:1205-1234, 416-446, 570-653): P = o + d t and the
// barycentric normal blend as FMA chains with no flat-triangle shortcut, pt +=
// -d 1e-3, an emission BSDF read as a diffuse one whose albedo is its
// radiance (cu:1705-1711 reinterpret_casts it), every hit adding
// radiance * importance unless PT_FLAG_NO_EMISSION (REAL_TIME, cu:1242-1246),
// the unnormalised diffuse direction n z + x dpdu + y dpdv, the mirror
// direction through the local-frame wi (cu:643-650), origins pt + n 1e-3.
// The scene must be triangles with diffuse / mirror / emission BSDFs
// (pt_render refuses spheres and glass under REFA: the reference has neither).
// LDSSH: the new shadow rays and their pending contributions go to this
// thread's column of sh_lds ([NSH][10][TPB]: o, d, tmax, C) as soon as the NEE
// sample has made them, instead of staying in registers through the BSDF
// sample (k_path_leaf: fewer VGPRs live at its peak)
// Occ: no immediate occlusion query (the shadow rays are traced later and
// resolved at the path's next vertex)
struct NoOcc {
  __device__ bool operator()(const RayV&) const { return false; }
};
template <class T>
struct imm_occ {
  static constexpr bool value = true;
};
template <>
struct imm_occ<NoOcc> {
  static constexpr bool value = false;
};
template <int NSH, bool M64 = false, bool KR = false, bool REFA = false, bool LDSSH = false, bool XL = false,
          class Occ = NoOcc, bool EARLY = true>
__device__ __forceinline__ void shade_vertex(const ShadeArgs& S, uint32_t sidx, PathState& st, const f3 o,
                                             const f3 d, uint32_t prim, float t, const bool (&clear)[NSH],
                                             f3 (&C)[NSH], bool& new_ext, RayV& ext, bool (&new_sh)[NSH],
                                             RayV (&shr)[NSH], float* sh_lds = nullptr, const Occ& occ = Occ{}) {
  // IMM (an occlusion query given, k_path_leaf): each NEE shadow ray is
  // tested where it is made and its contribution added at once -- the same
  // sum in the same order as resolving it at the next vertex, where it would
  // be added first -- so nothing is pending: new_sh says which rays were cast
  // (for the ray count), the flags carry no shadow bit
  constexpr bool IMM = imm_occ<Occ>::value;
  const uint32_t flags = st.flags;
  // (LDSSH: the radiance and the throughput live in rows 10 NSH .. 10 NSH + 5
  // of sh_lds -- rows 0 .. 5 under IMM --, re-read where they are used; a
  // memory clobber after each store keeps the compiler from carrying them in
  // registers anyway)
  float* const Lq = LDSSH ? sh_lds + (size_t)(IMM ? 0 : 10 * NSH) * TPB + threadIdx.x : nullptr;
  float* const Tq = LDSSH ? Lq + 3 * TPB : nullptr;
  f3 T = LDSSH ? mk(0.f, 0.f, 0.f) : st.T;
  auto Tv = [&]() { return LDSSH ? mk(Tq[0], Tq[TPB], Tq[2 * TPB]) : T; };
  auto Tset = [&](f3 v) {
    T = v;
    if constexpr (LDSSH) {
      Tq[0] = v.x;
      Tq[TPB] = v.y;
      Tq[2 * TPB] = v.z;
      asm volatile("" ::: "memory");
    }
  };
  f3 L = LDSSH ? mk(Lq[0], Lq[TPB], Lq[2 * TPB]) : st.L;
  const uint32_t g = st.g;
  // 1. resolve the shadow rays of the previous vertex
#pragma unroll
  for (int s = 0; s < NSH; ++s)
    if ((flags & sh_bit(s)) && clear[s]) L = L + C[s];
  // reference quirk (i): a path whose extension ray misses contributes
  // nothing (kernelUpdateSSImage writes 0 for an invalid intersection, cu:679-698)
  if ((S.flags & PT_FLAG_REF_DROP_ON_MISS) && (flags & F_EXT) && prim == PT_PRIM_NONE) L = mk(0.f, 0.f, 0.f);
  if constexpr (LDSSH) {
    Lq[0] = L.x;
    Lq[TPB] = L.y;
    Lq[2 * TPB] = L.z;
    asm volatile("" ::: "memory");
  }
  new_ext = false;
  f3 o_new = mk(0, 0, 0), d_new = mk(0, 0, 1);
#pragma unroll
  for (int s = 0; s < NSH; ++s) {
    new_sh[s] = false;
    C[s] = mk(0, 0, 0);
    shr[s] = RayV{mk(0, 0, 0), mk(0, 0, 1), -1.0f};
  }
  uint32_t spec = flags & F_SPEC;
  const uint32_t vtx = (flags >> 8) & 0xffu;

  // 2. shade the hit of the extension ray
  if (flags & F_EXT) {
    if (prim != PT_PRIM_NONE) {
      // (hit point and the offsets below as FMAs in both arithmetics)
      const f3 P = mk(__builtin_fmaf(d.x, t, o.x), __builtin_fmaf(d.y, t, o.y), __builtin_fmaf(d.z, t, o.z));
      // the record's first 16 B answer spheres ({centre, meta}) and flat
      // triangles ({n0, meta}); the rest is read only for a triangle with
      // distinct vertex normals (or the reference arithmetic's blend)
#ifdef PT_DBG_BOUNDS
      if (prim >= S.A.dbg_nprims) {
        printf("PT_DBG_BOUNDS shade prim %u vs %u (flags %x, t %g, block %d thread %d)\n", prim, S.A.dbg_nprims,
               st.flags, t, (int)blockIdx.x, (int)threadIdx.x);
        prim = 0u;
      }
#endif
      const float4* Q = S.shade + (size_t)prim * SHADE_REC;
      const float4 q0 = Q[0];
      // EARLY: the vertex's Philox words are computed while the shading
      // record's first load is in flight (they depend on the path and vertex
      // only; the shade kernel: +0.1-0.6 % on every workload, round 4)
      u4 u_early{0u, 0u, 0u, 0u};
      if constexpr (EARLY) u_early = rng<M64>(S.seed, g, sidx, vtx, 0);
      const uint32_t meta = __float_as_uint(q0.w) & ~SHADE_SMOOTH;
      f3 ns;
      if ((meta >> 28) == PT_PRIM_SPHERE) {
        ns = normalize(mk(P.x - q0.x, P.y - q0.y, P.z - q0.z));
      } else {
        const bool flat = !(__float_as_uint(q0.w) & SHADE_SMOOTH);
        if (!REFA && flat) {
          // flat triangle (n0 == n1 == n2): the barycentric blend is a
          // positive multiple of n0, so its normalisation is normalize(n0)
          // (computed on the host, pt_load_scene)
          ns = xyz(q0);
        } else {
          const float4 q1 = Q[1], q2 = Q[2], q3 = Q[3], q4 = Q[4];
          const f3 n1 = mk(q1.w, q2.w, q3.w), n2 = xyz(q4);
          // (a flat triangle's first 16 B hold normalize(n0): its raw n0 is n2)
          const f3 n0 = flat ? n2 : xyz(q0);
          // barycentric shading normal (cu:1213-1221)
          const f3 A = xyz(q1), B = xyz(q2), Cv = xyz(q3);
          float total = length(cross(A - B, B - Cv));
          float bC = length(cross(A - P, B - P)) / total;
          float bA = length(cross(B - P, Cv - P)) / total;
          float bB = length(cross(Cv - P, A - P)) / total;
          const f3 bw = mk(bA, bB, bC);
          // (FMA chains in both arithmetics)
          ns = normalize(mk(dot(bw, mk(n0.x, n1.x, n2.x)), dot(bw, mk(n0.y, n1.y, n2.y)),
                            dot(bw, mk(n0.z, n1.z, n2.z))));
        }
      }
      const bool front = dot(ns, d) < 0.0f;
      const f3 n = front ? ns : mk(-ns.x, -ns.y, -ns.z);  // faces the incoming ray (cu:1222)
      // cu:1224 (its.pt += -r->d * 1e-3)
      const f3 pt = mk(__builtin_fmaf(-d.x, EPS, P.x), __builtin_fmaf(-d.y, EPS, P.y), __builtin_fmaf(-d.z, EPS, P.z));
      BsdfRec B = S.bsdfs[meta & 0x0FFFFFFFu];
      bool emitter = false;
      if (REFA) {
        // cu:1243 (without REAL_TIME): its.light = radiance * importance + light
        const f3 rad = B.type == PT_BSDF_EMISSION ? ld3(B.albedo) : mk(0.f, 0.f, 0.f);
        if (!(S.flags & PT_FLAG_NO_EMISSION)) {
          if constexpr (LDSSH) L = mk(Lq[0], Lq[TPB], Lq[2 * TPB]);
          const f3 T0 = Tv();
          L = mk(__builtin_fmaf(rad.x, T0.x, L.x), __builtin_fmaf(rad.y, T0.y, L.y), __builtin_fmaf(rad.z, T0.z, L.z));
          if constexpr (LDSSH) {
            Lq[0] = L.x;
            Lq[TPB] = L.y;
            Lq[2 * TPB] = L.z;
            asm volatile("" ::: "memory");
          }
          emitter = rad.x != 0.0f || rad.y != 0.0f || rad.z != 0.0f;  // cu:436
        }
        if (B.type == PT_BSDF_EMISSION) B.type = PT_BSDF_DIFFUSE;  // albedo = radiance (cu:1705-1711)
        // a delta BSDF is read through a MirrorBSDF reinterpret_cast
        // (cu:1713-1719): over a GlassBSDF its reflectance is (roughness,
        // reflectance.r, reflectance.g), over a RefractionBSDF (roughness,
        // transmittance.r, transmittance.g) (bsdf.h:138-139, 180-182, 206-210)
        if (B.type == PT_BSDF_GLASS || B.type == PT_BSDF_REFRACTION) {
          const float c1 = B.type == PT_BSDF_GLASS ? B.albedo[0] : B.transmittance[0];
          const float c2 = B.type == PT_BSDF_GLASS ? B.albedo[1] : B.transmittance[1];
          B.albedo[0] = B.roughness;
          B.albedo[1] = c1;
          B.albedo[2] = c2;
          B.type = PT_BSDF_MIRROR;
        }
      }
      if (!REFA && B.type == PT_BSDF_EMISSION) {
        if (!(S.flags & PT_FLAG_NO_EMISSION) && (vtx == 1u || spec)) {
          if constexpr (LDSSH) L = mk(Lq[0], Lq[TPB], Lq[2 * TPB]);
          L = L + mulv(Tv(), ld3(B.albedo));
          if constexpr (LDSSH) {
            Lq[0] = L.x;
            Lq[TPB] = L.y;
            Lq[2 * TPB] = L.z;
            asm volatile("" ::: "memory");
          }
        }
      } else {
        const u4 u = EARLY ? u_early : rng<M64>(S.seed, g, sidx, vtx, 0);
        f3 dpdu, dpdv;
        if (S.flags & PT_FLAG_REF_GUIDE) {
          // reference quirk (ii): cu:572-574 (NaN when n is (0,-1,0)); n.y <
          // 1e-4 is a double comparison: n.y <= 1e-4f for an fp32 n.y
          const f3 guide = (n.y <= 1e-4f) ? mk(0.0f, 1.0f, 0.0f) : mk(1.0f, 0.0f, 0.0f);
          dpdu = normalize(cross(guide, n));
          dpdv = normalize(cross(dpdu, n));
        } else if (!REFA) {
          // branchless orthonormal basis (Duff et al., JCGT 6(1), 2017):
          // dpdu x dpdv = n; one reciprocal of sign(n.z) + n.z in [1, 2]
          // instead of a cross product, a normalisation and a second cross
          const float sg = __builtin_copysignf(1.0f, n.z);
          const float a = -rcp_rn(sg + n.z);
          const float b = (n.x * n.y) * a;
          const float sx = sg * n.x;
          dpdu = mk(__builtin_fmaf(sx * n.x, a, 1.0f), sg * b, -sx);
          dpdv = mk(b, __builtin_fmaf(n.y * n.y, a, sg), -n.y);
        } else {  // (REFA without the guide quirk)
          const f3 guide = (fabsf(n.x) < 0.9f) ? mk(1.0f, 0.0f, 0.0f) : mk(0.0f, 1.0f, 0.0f);
          dpdu = normalize_u(cross(guide, n));  // (|cross|^2 >= 0.19)
          dpdv = cross(n, dpdu);
        }
        if (B.type == PT_BSDF_DIFFUSE) {
          const f3 alb = ld3(B.albedo);
          // next-event estimation toward the scene light (cu:380-481); the
          // reference schedule takes 2, 2, 1 samples at vertices 1, 2, 3
          const int nee = emitter ? 0 : (NSH == 2 && vtx <= 2u) ? 2 : 1;
#pragma unroll
          for (int s = 0; s < NSH; ++s) {
            if (s < nee) {
              float ux = u01(u.x), uy = u01(u.y);
              uint32_t selw = u.x;
              if (s == 1) {
                const u4 v = rng_nee2<M64>(S.seed, g, sidx, vtx);
                ux = u01(v.x);
                uy = u01(v.y);
                selw = v.x;
              }
              const float weight = NSH == 2 ? (nee == 2 ? 0.5f : 1.0f) : -1.0f;
              new_sh[s] = nee_sample<KR, REFA, XL>(S, Tv(), alb, n, pt, ux, uy, weight, C[s], shr[s],
                                               selw);
              if constexpr (IMM) {
                if (new_sh[s] && !occ(shr[s])) {
                  if constexpr (LDSSH) L = mk(Lq[0], Lq[TPB], Lq[2 * TPB]);
                  L = L + C[s];
                  if constexpr (LDSSH) {
                    Lq[0] = L.x;
                    Lq[TPB] = L.y;
                    Lq[2 * TPB] = L.z;
                    asm volatile("" ::: "memory");
                  }
                }
              } else if constexpr (LDSSH) {
                float* q = sh_lds + (size_t)s * 10 * TPB + threadIdx.x;
                q[0 * TPB] = shr[s].o.x;
                q[1 * TPB] = shr[s].o.y;
                q[2 * TPB] = shr[s].o.z;
                q[3 * TPB] = shr[s].d.x;
                q[4 * TPB] = shr[s].d.y;
                q[5 * TPB] = shr[s].d.z;
                q[6 * TPB] = shr[s].tmax;
                q[7 * TPB] = C[s].x;
                q[8 * TPB] = C[s].y;
                q[9 * TPB] = C[s].z;
              }
            }
          }
          // BSDF sample
          float x, y, z, sn, cs;
          sincos2pi(u01(u.w), &sn, &cs);
          if (S.flags & PT_FLAG_COSINE_DIFFUSE) {
            const float u2 = u01(u.z);
            // (u2 and 1 - u2 are 0 or >= 2^-24: sqrt_rn is IEEE's sqrt)
            const float r = sqrt_rn(u2);
            x = r * cs;
            y = r * sn;
            z = sqrt_rn(fmaxf(0.0f, 1.0f - u2));
          } else {
            // uniform hemisphere: the reference's folded uniform sphere (cu:619-622)
            z = fabsf(2.0f * u01(u.z) - 1.0f);
            const float r = sqrt_rn(fmaxf(0.0f, 1.0f - z * z));  // (0 or >= 2^-24)
            x = r * cs;
            y = r * sn;
          }
          // cu:631-637: not normalised (the basis is orthonormal: |d_new| = 1 + O(ulp))
          d_new = mk(__builtin_fmaf(y, dpdv.x, __builtin_fmaf(x, dpdu.x, n.x * z)),
                     __builtin_fmaf(y, dpdv.y, __builtin_fmaf(x, dpdu.y, n.y * z)),
                     __builtin_fmaf(y, dpdv.z, __builtin_fmaf(x, dpdu.z, n.z * z)));
          if (S.flags & PT_FLAG_COSINE_DIFFUSE) {
            Tset(mulv(Tv(), alb));
          } else {
            const float c = fabsf(dot(d_new, n));
            const f3 T0 = Tv();
            Tset(mk(((T0.x * c) * alb.x) * 2.0f, ((T0.y * c) * alb.y) * 2.0f, ((T0.z * c) * alb.z) * 2.0f));
          }
          o_new = mk(__builtin_fmaf(n.x, EPS, pt.x), __builtin_fmaf(n.y, EPS, pt.y),
                     __builtin_fmaf(n.z, EPS, pt.z));  // cu:593
          spec = 0;
        } else if (REFA) {  // (a mirror: glass is read as one under REFA, above)
          // cu:1234 wi = normalize(dot(dpdu, -d), dot(dpdv, -d), dot(n, -d));
          // cu:643-650 wo = (-wi.x, -wi.y, wi.z) back to world space
          const f3 md = mk(-d.x, -d.y, -d.z);
          const f3 wi = normalize(mk(dot(dpdu, md), dot(dpdv, md), dot(n, md)));
          const float wx = -wi.x, wy = -wi.y, wz = wi.z;
          d_new = mk(__builtin_fmaf(wy, dpdv.x, __builtin_fmaf(wx, dpdu.x, n.x * wz)),
                     __builtin_fmaf(wy, dpdv.y, __builtin_fmaf(wx, dpdu.y, n.y * wz)),
                     __builtin_fmaf(wy, dpdv.z, __builtin_fmaf(wx, dpdu.z, n.z * wz)));
          o_new = mk(__builtin_fmaf(n.x, EPS, pt.x), __builtin_fmaf(n.y, EPS, pt.y), __builtin_fmaf(n.z, EPS, pt.z));
          Tset(mulv(Tv(), ld3(B.albedo)));
          spec = F_SPEC;
        } else {
          // PT_BSDF_MIRROR, and _GLASS / _REFRACTION (Fresnel-weighted reflect /
          // refract, bsdf.h:167-212) -- one body with the reflected and the
          // refracted direction selected before a single normalisation (a
          // wave's lanes at mirror, reflecting and refracting vertices ran
          // three bodies with a normalisation each)
          const float dn = dot(d, n);
          bool refl = true;
          float eta = 1.0f, cost = 0.0f;
          if (B.type != PT_BSDF_MIRROR) {
            const float ior = B.ior;
            eta = front ? B.inv_ior : ior;
            const float cosi = -dn;
            const float sin2t = (eta * eta) * (1.0f - cosi * cosi);
            if (sin2t < 1.0f) {
              cost = sqrt_rn(1.0f - sin2t);  // (sin2t < 1: 1 - sin2t >= 2^-24)
              const float r0 = B.r0;
              const float c = front ? cosi : cost;
              const float m = 1.0f - c;
              const float F = __builtin_fmaf(1.0f - r0, ((m * m) * (m * m)) * m, r0);
              // u.x: a glass vertex takes no NEE sample, so the vertex's first
              // Philox word is free (no second Philox call in a divergent branch)
              refl = u01(u.x) < F;
            }
          }
          // reflected: d - 2 (d.n) n; refracted (Snell): eta d + (eta cosi - cost) n
          const float kr = 2.0f * dn, kt = eta * -dn - cost;
          const f3 v = refl ? mk(d.x - n.x * kr, d.y - n.y * kr, d.z - n.z * kr)
                            : mk(d.x * eta + n.x * kt, d.y * eta + n.y * kt, d.z * eta + n.z * kt);
          d_new = normalize_u(v);  // (|v| ~ 1)
          Tset(mulv(Tv(), refl ? ld3(B.albedo) : ld3(B.transmittance)));
          const float oe = refl ? EPS : -EPS;
          const f3 ob = refl ? pt : P;
          o_new = mk(__builtin_fmaf(n.x, oe, ob.x), __builtin_fmaf(n.y, oe, ob.y), __builtin_fmaf(n.z, oe, ob.z));
          spec = F_SPEC;
        }
        new_ext = (vtx <= (uint32_t)S.max_bounces) && (T.x > 0.0f || T.y > 0.0f || T.z > 0.0f);
      }
    }
  }

  if constexpr (!LDSSH) {
    st.T = T;
    st.L = L;
  }
  uint32_t fl = spec | (new_ext ? F_EXT : 0u) | ((vtx + 1u) << 8);
#pragma unroll
  for (int s = 0; s < NSH; ++s) fl |= (new_sh[s] && !IMM) ? sh_bit(s) : 0u;
  st.flags = fl;
  ext.o = o_new;
  ext.d = d_new;
  ext.tmax = __builtin_inff();
}

// A finished path's radiance in the chunk's result buffer: 12 B per path
// (the buffer is read once more by k_accum: 16 B per path -> 12 B is a quarter
// of that stream; round 2, k_accum 0.74 -> ~0.5 ms per CBempty frame).
struct res3 {
  float x, y, z;
};
__device__ __forceinline__ void put_res(float4* res, uint32_t P, const f3 L) {
  reinterpret_cast<res3*>(res)[P] = res3{L.x, L.y, L.z};
}
__device__ __forceinline__ f3 get_res(const float4* res, size_t P) {
  const res3 r = reinterpret_cast<const res3*>(res)[P];
  return mk(r.x, r.y, r.z);
}

// Sum each active pixel's samples of this batch into the accumulation buffer
// (slot[q]: its owned slot; culled pixels add exact zeros, so they are not
// touched), in sample order (deterministic; replaces kernelUpdateSSImage +
// kernelReconstructImage + kernelAccumulate, cu:666-742).
__device__ __forceinline__ void accum_pixel(const float4* __restrict__ ps1, float4* accum,
                                            const uint32_t* __restrict__ slot, uint32_t npix, uint32_t spp_b,
                                            uint32_t q) {
  const uint32_t o = slot[q];
  float4 a = accum[o];
  for (uint32_t j = 0; j < spp_b; ++j) {
    const f3 l = get_res(ps1, (size_t)j * npix + q);
    a.x = a.x + l.x;
    a.y = a.y + l.y;
    a.z = a.z + l.z;
  }
  accum[o] = a;
}

// Pixel and sample of path P of the chunk.
__device__ __forceinline__ void path_pixel(const ShadeArgs& S, uint32_t P, uint32_t& g, uint32_t& sidx) {
  const uint32_t j = udiv_q(P, S.div_npix);
  g = S.pix_of[P - j * S.npix];
  sidx = S.sample_base + j;
}

// Philox products as v_mad_u64_u32 in the wavefront shade kernel too (the
// same bits as k_path_leaf's; 62 VGPRs, still 8 waves; CBbunny / dragon proxy
// +1.1 %, round 3)
constexpr bool SHADE_MAD64 = true;
// Slot states returned by shade_slot
constexpr int SLOT_FREE = 0, SLOT_LIVE = 1, SLOT_ENDED = 2;

// Record order: a wave writes its paths' new state and ray
// records back into its own 64 slots in the order of a key -- the primitive
// the path's extension ray hit, in SORT_KEYS equal ranges of the BVH order,
// i.e. roughly the subtree the new rays start in; camera rays, misses and
// free slots last.  Rays of one wave that start in the same subtree (and so
// mostly enter the same queues) then have adjacent 32-B records, so a level
// kernel's gather of consecutive queue entries shares 128-B lines instead of
// fetching one line per ray.  The slots of a path change from pass to pass
// within its wave; results do not depend on it (a permutation of the wave's
// slots, read before any is written).  CBbunny level 2 19.6 -> 15.7 ms,
// frame +3.9 %; dragon proxy +2.0 % (round 2).
// The key is taken after shading and ranked through a per-wave LDS histogram
// (one LDS atomic per lane, a 64-lane scan over the bins) instead of one
// ballot per key (-1.5-2 ms of shade kernel, round 2).  The order of lanes
// with equal keys is the order the LDS serves the atomics in; results do not
// depend on slots.  Measured and dropped: the same order over the whole
// workgroup (two barriers and an LDS scan: levels 1-2 % faster, but the shade
// kernel lost its 8th wave, -2.7 % on CBbunny), 32 key ranges (within noise),
// the octant of the new ray's direction in the key (within noise), the root
// target whose subtree holds the primitive as the key (-1.2 %).
constexpr uint32_t SORT_KEY_BITS = 4, SORT_KEYS = 1u << SORT_KEY_BITS;
constexpr uint32_t HIST_BINS = 256;  // >= SORT_KEYS + 2
__device__ __forceinline__ uint32_t wave_hist_rank(uint32_t key, bool act, uint32_t* bins) {
  const uint32_t ln = lane_id();
#pragma unroll
  for (uint32_t i = 0; i < HIST_BINS / 64; ++i) bins[ln * (HIST_BINS / 64) + i] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const uint32_t r = act ? atomicAdd(bins + key, 1u) : 0u;
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  uint32_t c[HIST_BINS / 64], tot = 0;
#pragma unroll
  for (uint32_t i = 0; i < HIST_BINS / 64; ++i) {
    c[i] = bins[ln * (HIST_BINS / 64) + i];
    tot += c[i];
  }
  uint32_t inc = tot;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t v = __shfl_up(inc, off, 64);
    if ((int)ln >= off) inc += v;
  }
  uint32_t b = inc - tot;
#pragma unroll
  for (uint32_t i = 0; i < HIST_BINS / 64; ++i) {
    bins[ln * (HIST_BINS / 64) + i] = b;
    b += c[i];
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  return act ? bins[key] + r : 0u;
}
// Shade the path in slot p: read its state, hit words and rays, run
// shade_vertex, write the new state and ray records.  Returns the new rays in
// registers.  A path with nothing left to trace (or `passes` vertices done)
// writes its radiance to res[P] and frees the slot.
// q: the slot the path's state and new rays are written to (its place in the
// key order of the wave).  Every thread of the workgroup calls this; act = the
// thread has a slot (p < N).  kc: LDS for the compaction pass's offsets.
// sparse (workgroup-uniform): most of the workgroup's slots are free (the tail
// of a chunk): the flags word is read first and only live slots read the rest
// (a second, dependent round trip instead of ~100 B of loads per free slot)
// Every word a slot may need (shade_slot), loaded in one round trip.
// (plain members, no arrays: the struct must stay in registers)
template <int NSH>
struct SlotLoad {
  float4 s0, s1, r0, r1, h0, c0, h1, c1;
};
template <int NSH>
__device__ __forceinline__ SlotLoad<NSH> load_slot(const ShadeArgs& S, uint32_t p) {
  SlotLoad<NSH> L;
  L.s0 = S.ps0_in[p];
  L.s1 = S.ps1_in[p];
  L.r0 = S.ray[RSTRIDE * p];
  L.r1 = S.ray[RSTRIDE * p + 1];
  L.h0 = S.ray[RSTRIDE * (S.N + p) + 1];
  L.c0 = S.ps2_in[p];
  if (NSH > 1) {
    L.h1 = S.ray[RSTRIDE * (2 * S.N + p) + 1];
    L.c1 = S.ps3_in[p];
  } else {
    L.h1 = L.c1 = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  return L;
}
template <int NSH, bool REFA = false, bool XL = false>
__device__ __forceinline__ int shade_slot(const ShadeArgs& S, uint32_t p, bool act, uint32_t& q, bool& new_ext,
                                          RayV& ext, bool (&new_sh)[NSH], RayV (&shr)[NSH], uint32_t (*kc)[4],
                                          uint32_t* bins, bool sparse, bool use_pre, const SlotLoad<NSH> pre) {
  new_ext = false;
#pragma unroll
  for (int s = 0; s < NSH; ++s) new_sh[s] = false;
  q = p;
  if (!act) p = 0;  // (loads from slot 0, ignored)
  // every word the slot may need is loaded at once (one memory round trip
  // instead of three dependent ones: flags, then records, then the ray and the
  // pending contributions); words the flags do not cover are stale and only
  // pass through selects
  float4 s0, s1, r0, r1, hs[NSH], cs[NSH];
  if (use_pre) {  // (dense pass: loaded at kernel entry)
    s0 = pre.s0;
    s1 = pre.s1;
    r0 = pre.r0;
    r1 = pre.r1;
#pragma unroll
    for (int s = 0; s < NSH; ++s) {
      hs[s] = s ? pre.h1 : pre.h0;
      cs[s] = s ? pre.c1 : pre.c0;
    }
  } else {
    s0 = S.ps0_in[p];
  }
  auto load_rest = [&]() {
    s1 = S.ps1_in[p];
    r0 = S.ray[RSTRIDE * p];
    r1 = S.ray[RSTRIDE * p + 1];
#pragma unroll
    for (int s = 0; s < NSH; ++s) {
      hs[s] = S.ray[RSTRIDE * ((1 + s) * S.N + p) + 1];
      cs[s] = (s ? S.ps3_in : S.ps2_in)[p];
    }
  };
  if (use_pre) {
    asm volatile("" ::"v"(s0.w), "v"(s1.w), "v"(r0.x), "v"(r1.x));
#pragma unroll
    for (int s = 0; s < NSH; ++s) asm volatile("" ::"v"(hs[s].z), "v"(cs[s].x));
  } else if (!sparse) {
    load_rest();
    // (the compiler would sink each load into the branch that uses it, i.e.
    // behind the previous load's wait: pin them all here)
    asm volatile("" ::"v"(s0.w), "v"(s1.w), "v"(r0.x), "v"(r1.x));
#pragma unroll
    for (int s = 0; s < NSH; ++s) asm volatile("" ::"v"(hs[s].z), "v"(cs[s].x));
  } else {
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    s1 = r0 = z;
    r1 = make_float4(0.f, 0.f, __uint_as_float(PT_PRIM_NONE), 0.f);
#pragma unroll
    for (int s = 0; s < NSH; ++s) hs[s] = cs[s] = z;
    if (act && (__float_as_uint(s0.w) & (F_EXT | F_SHADOW | F_SHADOW2))) {
      load_rest();
      asm volatile("" ::"v"(s1.w), "v"(r0.x), "v"(r1.x));
#pragma unroll
      for (int s = 0; s < NSH; ++s) asm volatile("" ::"v"(hs[s].z), "v"(cs[s].x));
    }
  }
  const uint32_t flags = act ? __float_as_uint(s0.w) : 0u;
  const bool live = (flags & (F_EXT | F_SHADOW | F_SHADOW2)) != 0;
  const uint32_t P = __float_as_uint(s1.w);
  PathState st{xyz(s0), flags, xyz(s1), 0u};
  const bool ext_hit = (flags & F_EXT) && __float_as_uint(r1.z) != PT_PRIM_NONE;
  const uint32_t prim = (flags & F_EXT) ? __float_as_uint(r1.z) : PT_PRIM_NONE;
  bool ended = true;
  f3 C[NSH];
  if (live) {
    uint32_t sidx;
    path_pixel(S, P, st.g, sidx);
    bool clear[NSH];
#pragma unroll
    for (int s = 0; s < NSH; ++s) {
      clear[s] = (flags & sh_bit(s)) && __float_as_uint(hs[s].z) == PT_PRIM_NONE;
      C[s] = clear[s] ? xyz(cs[s]) : mk(0, 0, 0);
    }
    const float t = ext_hit ? r1.w : 0.0f;
    const f3 o = ext_hit ? xyz(r0) : mk(0, 0, 0), d = ext_hit ? mk(r0.w, r1.x, r1.y) : mk(0, 0, 1);
    shade_vertex<NSH, SHADE_MAD64, false, REFA, false, XL>(S, sidx, st, o, d, prim, t, clear, C, new_ext, ext, new_sh,
                                                           shr);
    // (vertices done = vtx - 1: the last one resolves shadow rays only)
    ended = !(st.flags & (F_EXT | F_SHADOW | F_SHADOW2)) || ((st.flags >> 8) & 0xffu) - 1u >= (uint32_t)S.passes;
  }
  {  // (every lane of the wave: uniform control flow here)
    // continuing paths first (those whose new ray hit something in key
    // order, then the rest), ended paths and free slots last
    const bool cont = live && !ended;
    uint32_t key = cont ? HIST_BINS - 2 : HIST_BINS - 1;
    if (cont && new_ext && ext_hit) key = min(prim >> S.kshift, SORT_KEYS - 1u);
    const uint32_t r = wave_hist_rank(key, act, bins);
    if (act) q = (q & ~63u) + r;
    if (S.compact) {
      // compaction pass (uniform; every thread of the workgroup is here): the
      // workgroup's continuing paths take consecutive slots of the output
      // buffers from one atomic, wave by wave, each wave's in key order
      // (ranks 0 .. its count - 1)
      const unsigned long long mc = __ballot(act && cont);
      const uint32_t wv = threadIdx.x >> 6;
      if ((threadIdx.x & 63) == 0) kc[0][wv] = (uint32_t)__popcll(mc);
      if (wv == 0) {  // the region's first slot: the bounds of the regions below it
        const uint32_t j = threadIdx.x & 63;
        const uint32_t lo = wave_sum(j < (blockIdx.x & (CREGIONS - 1)) ? S.creg[j] : 0u);
        if (j == 0) kc[1][1] = lo;
      }
      __syncthreads();
      if (threadIdx.x == 0)
        kc[1][0] = kc[1][1] + atomicAdd(S.compact + (blockIdx.x & (CREGIONS - 1)),
                                        kc[0][0] + kc[0][1] + kc[0][2] + kc[0][3]);
      __syncthreads();
      uint32_t base = kc[1][0];
      for (uint32_t w = 0; w < wv; ++w) base += kc[0][w];
      if (act && cont) q = base + r;
    }
    if (!live) return SLOT_FREE;
  }
#ifdef PT_DBG_BOUNDS
  if (q >= S.N || (ended && P >= S.M)) {
    printf("PT_DBG_BOUNDS shade_slot q %u (N %u) P %u (M %u) ended %d compact %d block %d thread %d\n", q, S.N, P,
           S.M, (int)ended, S.compact ? 1 : 0, (int)blockIdx.x, (int)threadIdx.x);
    return SLOT_FREE;
  }
#endif
  if (ended) {
    new_ext = false;
#pragma unroll
    for (int s = 0; s < NSH; ++s) new_sh[s] = false;
    put_res(S.res, P, st.L);
    // (the caller frees the slot -- ps0 flags 0 -- unless it starts a new path)
  } else {
    S.ps0[q] = make_float4(st.T.x, st.T.y, st.T.z, __uint_as_float(st.flags));
    S.ps1[q] = make_float4(st.L.x, st.L.y, st.L.z, __uint_as_float(P));
  }
  // new rays: their records are written by root_pass (with the key of the
  // inline leaves).  A slot without a new ray keeps its stale record: only
  // the path's flags say which records the next shade reads, and nothing
  // else reads a record that was not queued (no 16-B "empty" partial writes)
#pragma unroll
  for (int s = 0; s < NSH; ++s)
    if (new_sh[s]) (s ? S.ps3 : S.ps2)[q] = make_float4(C[s].x, C[s].y, C[s].z, 0.0f);
  return ended ? SLOT_ENDED : SLOT_LIVE;
}

// Start path P in slot p: state and camera ray (kernelPrimaryRays, cu:312-376).
template <bool REFA = false>
__device__ __forceinline__ f3 start_path(const ShadeArgs& S, uint32_t p, uint32_t P) {
  uint32_t g;
  const f3 d = camera_dir<false, REFA>(S, P, g);
  // (the ray record is written by root_pass)
  S.ps0[p] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(F_EXT | (1u << 8)));
  S.ps1[p] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(P));
  return d;
}

// One fire-and-forget atomic per workgroup: rays that enter the traversal.
__device__ __forceinline__ void count_rays(unsigned long long* rcount, uint32_t v, uint32_t* sh4) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh4[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = sh4[0] + sh4[1] + sh4[2] + sh4[3];
    if (t) atomicAdd(rcount + (size_t)(blockIdx.x & (RCOUNT_SLOTS - 1)) * 16, (unsigned long long)t);
  }
}

// ---- path blocks -------------------------------------------------------------
// Block c = paths [POOL_BLOCK c, min(POOL_BLOCK (c + 1), M)); dispenser s hands
// out blocks s, s + POOLS, s + 2 POOLS, ... (its counter v -> block s + POOLS v).
// The first fill gives workgroup b block b; afterwards a workgroup takes one new
// block whenever its current one cannot fill its free slots (one atomic per
// POOL_BLOCK paths, spread over POOLS counters), so every workgroup keeps its
// slots busy until the whole chunk is handed out: no workgroup runs out of
// paths early while others still hold many (a static split of the chunk by
// pixel region leaves a long tail: regions differ in mean path length).
constexpr uint32_t POOL_BLOCK = TPB, POOLS = 64;
__device__ __forceinline__ uint32_t pool_limit(uint32_t nblocks, uint32_t s) {
  return nblocks > s ? (nblocks - s + POOLS - 1) / POOLS : 0u;
}
// Wave 0 of a workgroup: claim one block, trying dispenser (b + k) % POOLS in
// order among those not yet exhausted (all 64 peeked at once, one lane each).
// Returns the block index, or -1 when every dispenser is exhausted (or lost
// the race for its last block).
__device__ __forceinline__ int claim_block(const ShadeArgs& S, uint32_t nblocks) {
  const uint32_t ln = lane_id();
  const uint32_t sd = (blockIdx.x + ln) & (POOLS - 1);
  const bool open =
      __hip_atomic_load(S.pool + (size_t)sd * CSTRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
      pool_limit(nblocks, sd);
  const unsigned long long mo = __ballot(open);
  if (!mo) return -1;
  const uint32_t k = (uint32_t)__builtin_ctzll(mo);
  int c = -1;
  if (ln == k) {
    const uint32_t v = atomicAdd(S.pool + (size_t)sd * CSTRIDE, 1u);
    if (v < pool_limit(nblocks, sd)) c = (int)(sd + POOLS * v);
  }
  return __builtin_amdgcn_readlane(c, k);
}

// Fused root pass: the new rays never take the trip through HBM and back to
// be tested against the root -- the producing kernel tests them against the
// root's targets and pushes their ids into those queues (lane = workgroup & 7).
// First fill: workgroup b runs block b, slot i its path i.
template <int NSH, bool REFA>
__global__ __launch_bounds__(TPB) void k_camera_push(ShadeArgs S) {
  __shared__ uint32_t sh[MAX_ROOT_TARGETS * 8 + 4];
  const uint32_t p = blockIdx.x * TPB + threadIdx.x;
  const uint32_t base = blockIdx.x * POOL_BLOCK, end = min(S.M, base + POOL_BLOCK);
  const uint32_t slots = min((uint32_t)TPB, S.N - blockIdx.x * TPB);  // (the last workgroup may be partial)
  const uint32_t n0 = end > base ? min(slots, end - base) : 0u;
  const bool live = threadIdx.x < n0;
  uint32_t id[1] = {p};
  f3 o[1] = {ld3(S.cam.origin)}, d[1] = {mk(0.f, 0.f, 1.f)};
  float tm[1] = {__builtin_inff()};
  bool valid[1] = {live}, anyhit[1] = {false};
  if (threadIdx.x == 0) S.wstate[blockIdx.x] = make_uint4(base + n0, end, n0, 0u);
  if (p < S.N) {
    // (records are written by root_pass for the rays it receives; a path's
    // flags say which of its records are meaningful)
    if (live)
      d[0] = start_path<REFA>(S, p, base + threadIdx.x);
    else
      S.ps0[p] = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
  }
  root_pass<1, REFA>(S.A, S.T, blockIdx.x & (NLANE - 1), id, o, d, tm, valid, anyhit, sh);
  count_rays(S.rcount, live ? 1u : 0u, sh + MAX_ROOT_TARGETS * 8);
}

// One pass of shading with path regeneration: shade every live slot, then the
// free slots (free before, or their path just ended) start the next paths of
// the workgroup's block (and of a newly claimed block when it runs short), and
// all new rays (extension, shadow, camera) are pushed into the root's target
// queues.  A workgroup with no live slot and nothing left to start returns at
// once (passes queued after the chunk ended).
// at least 7 waves/SIMD (built without SLP vectorisation, pt_shade.hip, it
// needs 64 VGPRs and runs 8; with SLP it needed 74, i.e. 6 waves:
// CBbunny shade 101 -> 105 ms)
constexpr int SHADE_WAVES = 7;
// a workgroup with fewer live slots than this reads its slots sparsely (shade_slot)
constexpr uint32_t SPARSE_LIVE = 128;
template <int NSH, bool REFA, bool XL = false>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(SHADE_WAVES, 8))) void k_shade_push(ShadeArgs S) {
  __shared__ uint32_t sh[MAX_ROOT_TARGETS * 8 + 4];
  __shared__ uint32_t s_free[4], s_live[4], s_busy[4], s_next, s_end, s_shaded, s_nb, s_nbn;
  __shared__ float s_dir[3][TPB];
  __shared__ int s_skip, s_sparse;
  const int tid = threadIdx.x, wave = tid >> 6;
#if PT_SHADE_TIMING
  unsigned long long t_[8];
#endif
  SHADE_STAMP(0);
  const uint32_t nblocks = (S.M + POOL_BLOCK - 1) / POOL_BLOCK;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  SlotLoad<NSH> pre{z4, z4, z4, z4, z4, z4, z4, z4};
  if (S.dense) pre = load_slot<NSH>(S, blockIdx.x * TPB + tid < S.N ? blockIdx.x * TPB + tid : 0u);
  // slots [0, nin) hold paths (after a compaction fewer than N)
  const uint32_t nin = S.nact ? *S.nact : S.N;
  if (tid == 0) {
    const uint4 ws = S.wstate[blockIdx.x];
    s_next = ws.x;
    s_end = ws.y;
    s_shaded = ws.w;
    s_skip = ws.z == 0 && ws.x >= ws.y;  // idle: unless a dispenser is still open (below)
    // (ws.z: the slots live after the last pass's regeneration)
    s_sparse = ws.z < SPARSE_LIVE;
  }
  __syncthreads();
  SHADE_STAMP(1);
  if (s_skip) {  // (uniform: every thread has read it before the barrier below)
    __syncthreads();
    if (wave == 0) {
      const uint32_t sd = lane_id();
      const bool open = __hip_atomic_load(S.pool + (size_t)sd * CSTRIDE, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) < pool_limit(nblocks, sd);
      if (tid == 0) s_skip = 0;
      if (__ballot(open) == 0 && tid == 0) s_skip = 1;
    }
    __syncthreads();
    if (s_skip) return;
  }
  // The root pass's candidate-cluster members into LDS, straight from
  // memory (no VGPRs; in flight across the shading below): 3 wave loads
  // (REFA: the reference-arithmetic records, 6 float4 each: 3 wave loads)
  constexpr int RPS = REFA ? 6 : 4;
  __shared__ float4 s_rcm[RPS * ROOT_CL_MAX];
  __shared__ uint32_t s_rci[2 * ROOT_CL_MAX];
  constexpr int NW = RPS * ROOT_CL_MAX / 64;  // wave loads of 64 records' float4s
  {
    static_assert(RPS * ROOT_CL_MAX % 64 == 0 && 2 * ROOT_CL_MAX == 64 && NW < TPB / 64,
                  "wave-wide LDS loads: the records, then the info words");
    typedef __attribute__((address_space(1))) const void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    if (S.T.nc > 0) {
      const int l = tid & 63;
      const float4* src = REFA ? S.T.cmem_ref : S.T.cmem;
      if (wave < NW)
        __builtin_amdgcn_global_load_lds((gptr_t)(src + wave * 64 + l), (lptr_t)(s_rcm + wave * 64), 16, 0, 0);
      else if (wave == NW)
        __builtin_amdgcn_global_load_lds((gptr_t)(S.T.cinfo + l), (lptr_t)s_rci, 4, 0, 0);
    }
  }
  const uint32_t p = blockIdx.x * TPB + tid;
  bool new_ext = false, new_sh[NSH];
  RayV ext{mk(0, 0, 0), mk(0, 0, 1), -1.0f}, shr[NSH];
#pragma unroll
  for (int s = 0; s < NSH; ++s) {
    new_sh[s] = false;
    shr[s] = RayV{mk(0, 0, 0), mk(0, 0, 1), -1.0f};
  }
  __shared__ uint32_t s_kc[SORT_KEYS + 1][4];
  __shared__ uint32_t s_bins[4 * HIST_BINS];
  uint32_t q = p;  // where this lane's path state and new rays go
  int state = shade_slot<NSH, REFA, XL>(S, p, p < nin, q, new_ext, ext, new_sh, shr, s_kc,
                                    s_bins + wave * HIST_BINS, s_sparse != 0,
                                    S.dense != 0, pre);
  // ---- regeneration: free slots take the next paths in rank order, from the
  // current block and then from a newly claimed one
  const bool fr = p < nin && state != SLOT_LIVE;
  const unsigned long long mf = __ballot(fr), ml = __ballot(p < nin && state == SLOT_LIVE),
                           mb = __ballot(p < nin && state != SLOT_FREE);
  if ((tid & 63) == 0) {
    s_free[wave] = (uint32_t)__popcll(mf);
    s_live[wave] = (uint32_t)__popcll(ml);
    s_busy[wave] = (uint32_t)__popcll(mb);
  }
  __syncthreads();
  SHADE_STAMP(2);
  const uint32_t nf = s_free[0] + s_free[1] + s_free[2] + s_free[3];
  const uint32_t next = s_next, end = s_end;
  const uint32_t avail = end > next ? end - next : 0u;
  // (compaction pass: the block's paths start in the extra round below, not in
  // the free slots, whose positions mean nothing in the compacted layout)
  const uint32_t t1 = S.compact ? 0u : min(nf, avail);
  if (wave == 0) {
    // (nf <= 256 = POOL_BLOCK: one new block always covers the rest)
    int c = -1;
    // (no new paths once the tail is compacted: every block is handed out)
    if (nf > t1 && !S.compact && !S.nact) c = claim_block(S, nblocks);
    if (tid == 0) {
      uint32_t nb = 0, nbn = 0, nnext = next + t1, nend = end;
      if (c >= 0) {
        nb = (uint32_t)c * POOL_BLOCK;
        const uint32_t nbend = min(S.M, nb + POOL_BLOCK);
        nbn = min(nf - t1, nbend - nb);
        nnext = nb + nbn;
        nend = nbend;
      }
      s_nb = nb;
      s_nbn = nbn;
      if (S.compact) nnext = nend;  // (all of them start below)
      S.wstate[blockIdx.x] = make_uint4(nnext, nend, s_live[0] + s_live[1] + s_live[2] + s_live[3] + t1 + nbn,
                                        s_shaded + s_busy[0] + s_busy[1] + s_busy[2] + s_busy[3]);
    }
  }
  __syncthreads();
  SHADE_STAMP(3);
  // camera rays of the paths that start here, computed by the first ns threads
  // of the workgroup (whole waves, not one lane in four of every wave: the
  // camera code then runs in ceil(ns / 64) waves instead of all four), handed
  // to the free slots through LDS in rank order
  const uint32_t ns = min(nf, t1 + s_nbn);
  if ((uint32_t)tid < ns) {
    const uint32_t P = (uint32_t)tid < t1 ? next + (uint32_t)tid : s_nb + (uint32_t)tid - t1;
    uint32_t g;
    const f3 dir = camera_dir<SHADE_MAD64, REFA>(S, P, g);
    s_dir[0][tid] = dir.x;
    s_dir[1][tid] = dir.y;
    s_dir[2][tid] = dir.z;
  }
  // The LDS copies of the cluster records count against vmcnt, and a
  // workgroup barrier waits only for lgkmcnt: each loader wave waits for its
  // copy here, before the barrier that precedes root_pass's reads of s_rcm /
  // s_rci by every wave (a tail workgroup's idle loader wave reaches it within
  // a few hundred cycles of issuing the copy).
  if (S.T.nc > 0 && wave <= NW) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt unchanged
  __syncthreads();
  SHADE_STAMP(4);
  if (fr) {
    uint32_t rank = mbcnt64(mf);
    for (int w = 0; w < wave; ++w) rank += s_free[w];
#ifdef PT_DBG_BOUNDS
    if (q >= S.N) printf("PT_DBG_BOUNDS regen q %u (N %u) block %d thread %d\n", q, S.N, (int)blockIdx.x, (int)threadIdx.x);
#endif
    if (rank < ns) {
      const uint32_t P = rank < t1 ? next + rank : s_nb + rank - t1;
      S.ps0[q] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(F_EXT | (1u << 8)));
      S.ps1[q] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(P));
      ext = RayV{ld3(S.cam.origin), mk(s_dir[0][rank], s_dir[1][rank], s_dir[2][rank]), __builtin_inff()};
      new_ext = true;
    } else if (!S.compact && (state == SLOT_ENDED || q != p)) {
      // the slot stays free (slot q may have held another lane's path until now)
      S.ps0[q] = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
    }
  }
  uint32_t id[1 + NSH];
  f3 o[1 + NSH], d[1 + NSH];
  float tm[1 + NSH];
  bool valid[1 + NSH], anyhit[1 + NSH];
  id[0] = q;
  o[0] = ext.o;
  d[0] = ext.d;
  tm[0] = __builtin_inff();
  valid[0] = new_ext;
  anyhit[0] = false;
  uint32_t n = new_ext ? 1u : 0u;
#pragma unroll
  for (int s = 0; s < NSH; ++s) {
    id[1 + s] = (1 + s) * S.N + q;
    o[1 + s] = shr[s].o;
    d[1 + s] = shr[s].d;
    tm[1 + s] = shr[s].tmax;
    valid[1 + s] = new_sh[s];
    anyhit[1 + s] = true;
    n += new_sh[s] ? 1u : 0u;
  }
  root_pass<1 + NSH, REFA, false, true>(S.A, S.T, blockIdx.x & (NLANE - 1), id, o, d, tm, valid, anyhit, sh, s_rcm,
                                        s_rci);
  count_rays(S.rcount, n, sh + MAX_ROOT_TARGETS * 8);
#if PT_SHADE_TIMING
  __syncthreads();
  SHADE_STAMP(5);
  if (tid == 0 && S.tprof) {
    unsigned long long* tp = S.tprof + (blockIdx.x & 63) * 16;
    for (int k = 1; k <= 5; ++k) atomicAdd(tp + k, t_[k] - t_[k - 1]);
    atomicAdd(tp, 1ull);
    atomicAdd(tp + 6, (unsigned long long)(s_live[0] + s_live[1] + s_live[2] + s_live[3]));
    for (int k = 1; k <= 3; ++k) atomicAdd(tp + 6 + k, g_rp_t[k] - g_rp_t[k - 1]);
    atomicAdd(tp + 10, g_rp_t[5] - g_rp_t[3]);
    atomicAdd(tp + 11, t_[5] - g_rp_t[5]);
    atomicAdd(tp + 12, g_rp_t[4] - g_rp_t[0]);
  }
#endif
  if (S.compact && avail) {
    // compaction pass, extra round (uniform): every unstarted path of the
    // workgroup's block starts here, in consecutive slots of the compacted
    // layout (the dispensers are dry: after this no workgroup holds any)
    if (tid == 0) s_nb = s_kc[1][1] + atomicAdd(S.compact + (blockIdx.x & (CREGIONS - 1)), avail);
    __syncthreads();
    const bool st0 = (uint32_t)tid < avail;
    uint32_t id1[1] = {s_nb + (uint32_t)tid};
    f3 o1[1] = {ld3(S.cam.origin)}, d1[1] = {mk(0.f, 0.f, 1.f)};
    float tm1[1] = {__builtin_inff()};
    bool valid1[1] = {st0}, anyhit1[1] = {false};
    if (st0) {
      const uint32_t P = next + (uint32_t)tid;
      uint32_t g;
      d1[0] = camera_dir<SHADE_MAD64, REFA>(S, P, g);
      S.ps0[id1[0]] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(F_EXT | (1u << 8)));
      S.ps1[id1[0]] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(P));
    }
    root_pass<1, REFA, false, true>(S.A, S.T, blockIdx.x & (NLANE - 1), id1, o1, d1, tm1, valid1, anyhit1, sh, s_rcm,
                                    s_rci);
    count_rays(S.rcount, st0 ? 1u : 0u, sh + MAX_ROOT_TARGETS * 8);
  }
}

// Work left in paths (the host polls it: live[0] = 0 means the chunk is
// done): live slots over all workgroups, the unstarted rest of each
// workgroup's current block, and POOL_BLOCK paths for every block no
// dispenser has handed out yet (the chunk's last block may hold fewer: an
// upper bound); live[1] = the paths of the unclaimed blocks alone (0: the
// dispensers are dry, the tail may be compacted); live[2 + k] = the live
// slots and unstarted paths of the workgroups b with b % CREGIONS = k (the
// compaction regions' bounds); with stats, also the chunk's shaded
// vertices (stats[STAT_SHADED]).  A grid of LIVE_SUM_BLOCKS workgroups, a few
// atomics each into the zeroed live[0 .. 2 + CREGIONS).
constexpr int LIVE_SUM_BLOCKS = 64;
static_assert(LIVE_SUM_BLOCKS * 1024 % CREGIONS == 0 && CREGIONS == 64, "k_live_sum: thread t sums region t % 64");
__global__ __launch_bounds__(1024) void k_live_sum(const uint4* __restrict__ wstate, uint32_t G, const uint32_t* pool,
                                                   uint32_t nblocks, uint32_t* live, unsigned long long* shaded) {
  __shared__ unsigned long long part[3][16];
  __shared__ uint32_t reg[16][CREGIONS];
  unsigned long long v = 0, un = 0, sh = 0;
  uint32_t vr = 0;  // (every b this thread visits has b % CREGIONS = threadIdx.x % CREGIONS)
  for (uint32_t b = blockIdx.x * 1024 + threadIdx.x; b < G; b += gridDim.x * 1024) {
    const uint4 w = wstate[b];
    const uint32_t n = w.z + (w.y > w.x ? w.y - w.x : 0u);
    v += n;
    vr += n;
    sh += w.w;
  }
  reg[threadIdx.x >> 6][threadIdx.x & 63] = vr;
  if (blockIdx.x == 0 && threadIdx.x < POOLS) {
    const uint32_t lim = pool_limit(nblocks, threadIdx.x), c = pool[(size_t)threadIdx.x * CSTRIDE];
    un += c < lim ? (unsigned long long)(lim - c) * POOL_BLOCK : 0ull;
  }
  v = wave_sum64(v + un);
  un = wave_sum64(un);
  sh = wave_sum64(sh);
  if ((threadIdx.x & 63) == 0) {
    part[0][threadIdx.x >> 6] = v;
    part[1][threadIdx.x >> 6] = sh;
    part[2][threadIdx.x >> 6] = un;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0, u = 0, n = 0;
    for (int w = 0; w < 16; ++w) {
      t += part[0][w];
      u += part[1][w];
      n += part[2][w];
    }
    if (t) atomicAdd(live, (uint32_t)min(t, 0xFFFFFFFFull));
    if (n) atomicAdd(live + 1, (uint32_t)min(n, 0xFFFFFFFFull));
    if (shaded && u) atomicAdd(shaded, u);
  }
  if (threadIdx.x < CREGIONS) {
    uint32_t r = 0;
    for (int w = 0; w < 16; ++w) r += reg[w][threadIdx.x];
    if (r) atomicAdd(live + 2 + threadIdx.x, r);
  }
}

// After a compaction pass, first: the old layout's shaded-vertex counts
// added to *shaded (stats; may be null), and the states of its workgroups
// beyond the new layout's Gnew cleared.  One thread per workgroup state.
__global__ __launch_bounds__(TPB) void k_compact_wstate(uint4* wstate, uint32_t Gold, uint32_t Gnew,
                                                        unsigned long long* shaded) {
  const uint32_t b = blockIdx.x * TPB + threadIdx.x;
  unsigned long long w = 0;
  if (b < Gold) w = wstate[b].w;
  if (shaded) {
    w = wave_sum64(w);
    if ((threadIdx.x & 63) == 0 && w) atomicAdd(shaded, w);
  }
  if (b >= Gnew && b < Gold) wstate[b] = make_uint4(0u, 0u, 0u, 0u);
}

// Then, one workgroup per workgroup of the compacted layout: region k holds
// slots [lo_k, lo_k + creg[k]) (lo_k = the sum of the lower bounds), of which
// the pass filled the first cnt[k]; the rest is a hole whose slots are marked
// free (ps0 flags 0: the shade kernel reads nothing else of a free slot), and
// the workgroup's state = nothing to start, its live slots.  Workgroup 0 also
// writes the layout's extent (*nact = the sum of the bounds).
__global__ __launch_bounds__(TPB) void k_compact_slots(float4* ps0, uint4* wstate, const uint32_t* cnt,
                                                       const uint32_t* creg, uint32_t* nact) {
  __shared__ uint32_t s_r[CREGIONS], s_lo[CREGIONS], s_n[TPB / 64];
  if (threadIdx.x < CREGIONS) s_r[threadIdx.x] = creg[threadIdx.x];
  __syncthreads();
  if (threadIdx.x < CREGIONS) {
    uint32_t lo = 0;
    for (uint32_t j = 0; j < threadIdx.x; ++j) lo += s_r[j];
    s_lo[threadIdx.x] = lo;
    if (threadIdx.x == CREGIONS - 1 && blockIdx.x == 0) *nact = lo + s_r[threadIdx.x];
  }
  __syncthreads();
  const uint32_t q = blockIdx.x * TPB + threadIdx.x;
  // the region of q: the last k with lo_k <= q (empty regions share their lo)
  uint32_t k = 0;
#pragma unroll
  for (uint32_t st = CREGIONS / 2; st; st >>= 1) k = s_lo[k + st] <= q ? k + st : k;
  const bool in = q < s_lo[k] + s_r[k];
  const bool live = in && q < s_lo[k] + cnt[k];
  if (in && !live) ps0[q] = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
  const unsigned long long m = __ballot(live);
  if ((threadIdx.x & 63) == 0) s_n[threadIdx.x >> 6] = (uint32_t)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) wstate[blockIdx.x] = make_uint4(0u, 0u, s_n[0] + s_n[1] + s_n[2] + s_n[3], 0u);
}

// ---- scenes whose BVH root is a leaf -----------------------------------------
// With a single-leaf tree every traversal pass is the root pass: each ray tests
// all primitives of the leaf and nothing is queued, so the pass/shade wavefront
// collapses into one kernel that carries each path through all of its vertices
// in registers (no ray records, hit words or path state in HBM).  Closest hits
// use the same primitive tests and tie rule as the leaf code of
// process_item (trace.hip); results are bit-identical to the wavefront path.
// SPH: the leaf may hold spheres (else the sphere branch is not compiled in)
// The closest-hit loop is strict (extension rays, tmax = +inf): the triangle
// test admits only t < the best so far, so a hit is a new best and the update
// is two selects (no exec-mask branches: fewer SALU per primitive; round 4,
// CBempty +3.7 %).  The same hits as take_hit: a tie keeps the lower index
// either way, and the inclusive tmax of take_hit matters only for a first hit
// at t = tmax = +inf, which no test returns (an infinite t fails the
// barycentric test).  Default arithmetic: two primitive records per scalar
// round trip (one wait and one loop step per pair: +1 %), and a triangle's
// update made inside the test from its own compares (bw_closest_update: no
// second t < bt compare, no -0 fix -- a -0 t only feeds compares and the hit
// point; CBempty +1.5 %, then +1.6 %, CBspheres' triangles +2.6 %, round 4).
template <bool REFA, bool SPH = true>
__device__ __forceinline__ void leaf_closest(const float4* prims, int pstart, int pcount, const RayV& r,
                                             uint32_t& prim, float& t) {
  float bt = r.tmax;
  int bp = -1;
  constexpr int PS = prim_stride<REFA>();
  const CPTR(f4v) P = (const CPTR(f4v))(prims + (size_t)pstart * PS);
  int k0 = 0;
  if constexpr (!REFA) {
    auto step = [&](const Prim& q, int k) {
      if (!SPH || !prim_sphere<REFA>(q)) {
        // the update straight from the test's compares (no -1 sentinel)
        bw_closest_update(r.o, r.d, q, pstart + k, bt, bp);
        return;
      }
      // (a sphere's t is checked against bt here)
      const float tt = sphere_test(r.o, r.d, q.q0, q.q1);
      const bool take = (tt >= 0.0f) & (tt < bt);
      bt = take ? tt : bt;
      bp = take ? pstart + k : bp;
    };
    for (; k0 + 1 < pcount; k0 += 2, P += 2 * PS) {
      Prim qa, qb;
      load_prim_pair(P, qa, qb);
      step(qa, k0);
      step(qb, k0 + 1);
    }
  }
  for (int k = k0; k < pcount; ++k, P += PS) {
    // the whole record in one scalar round trip (load_prim)
    const Prim q = load_prim<REFA>(P);
    // (a tri_outside pre-test does not pay here: extension rays of one wave
    // rarely all miss a plane, measured -7 % on CBempty)
    const float tt = (SPH && prim_sphere<REFA>(q)) ? sphere_test(r.o, r.d, q.q0, q.q1)
                                                   : tri_test<REFA, true>(r.o, r.d, q, bt);
    const bool take = (tt >= 0.0f) & (tt < bt);
    bt = take ? tt : bt;
    bp = take ? pstart + k : bp;
  }
  prim = bp < 0 ? PT_PRIM_NONE : (uint32_t)bp;
  t = bt;
}

// PT_FLAG_COUNT_TESTS: the primitive tests and cluster box tests a lane
// executes (the counting variant of k_path_leaf only, CNT; the timed kernels
// carry none of it)
struct TestCount {
  uint32_t tri, sph, box;
};

// Candidate clusters: the closest-hit loop tests the leaf's primitive clusters
// (one primitive, or two consecutive triangles with nearly the same box: a
// Cornell wall's halves; ShadeArgs::cbox, host-built, widened by the BVH
// boxes' guard band: conservative as a leaf box is) only where the lane's ray
// enters the cluster's box, from records staged in LDS (s_rec; per-lane
// candidates, so vector reads).  An extension ray inside the Cornell box
// enters the boxes of the wall it leaves through (and of the light in front of
// the ceiling): 1-2 clusters of 6.  Candidates run in increasing index with
// the strict test: the same hit as the full loop (a box missed holds no hit).
// CBempty 85,000 -> 93,400 Mrays/s, CBspheres 56,950 -> 59,100 (interleaved
// A/B, 2 runs each; fixed pairs (2i, 2i + 1) instead: CBspheres 50,200, a
// sphere paired with the ceiling).  Extension rays pick their candidates by
// the slab test: by the overlap of the box of their segment to the exit from
// the clusters' union box instead (as the shadow rays do), CBempty 17.9 ->
// 18.7 ms per frame, CBspheres likewise -- a room-crossing segment's box
// overlaps more walls than its slab test enters, and each extra candidate
// costs a division (round 5).
constexpr int PATH_CL_PRIMS = 32;  // primitives staged in LDS at most
template <bool SPH, bool CNT = false>
__device__ __forceinline__ void leaf_closest_cl(const ShadeArgs& S, const float4* s_rec, const uint32_t* s_cl,
                                                int pstart, int pcount, const RayV& r, uint32_t& prim, float& t,
                                                TestCount* tc = nullptr) {
  const f3 inv = mk(__builtin_amdgcn_rcpf(safe_dir(r.d.x)), __builtin_amdgcn_rcpf(safe_dir(r.d.y)),
                    __builtin_amdgcn_rcpf(safe_dir(r.d.z)));
  const f3 oi = mk(r.o.x * inv.x, r.o.y * inv.y, r.o.z * inv.z);
  const CPTR(f4v) B = (const CPTR(f4v))S.cbox;
  uint32_t cm = 0u;
  for (int c = 0; c < S.nclus; ++c) {
    const float4 b0 = f4(B[2 * c]), b1 = f4(B[2 * c + 1]);
    cm = mask_bit(cm, box_hit_open(b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, oi, inv), c);
  }
  if constexpr (CNT) tc->box += (uint32_t)S.nclus;
  float bt = r.tmax;
  int bp = -1;
  auto step = [&](int k) {
    Prim q;
    q.q0 = s_rec[4 * k];
    q.q1 = s_rec[4 * k + 1];
    q.q2 = s_rec[4 * k + 2];
    q.q3 = s_rec[4 * k + 3];
    if constexpr (CNT) {
      if (SPH && prim_sphere<false>(q)) ++tc->sph;
      else ++tc->tri;
    }
    if (SPH && prim_sphere<false>(q)) {
      const float tt = sphere_test(r.o, r.d, q.q0, q.q1);
      const bool take = (tt >= 0.0f) & (tt < bt);
      bt = take ? tt : bt;
      bp = take ? pstart + k : bp;
    } else {
      bw_closest_update(r.o, r.d, q, pstart + k, bt, bp);
    }
  };
  if constexpr (SPH) {
    // the triangle candidates, then the spheres: two per-lane loops instead
    // of one whose iterations ran both tests whenever a wave's lanes were at
    // a triangle and at a sphere.  A sphere takes a tie with the best so far
    // by the lower index: the hit of the loop in index order.
    uint32_t cs = cm & S.sph_cl;
    cm &= ~S.sph_cl;
    while (cm) {
      const int c = __builtin_ctz(cm);
      cm &= cm - 1u;
      const uint32_t fc = s_cl[c];  // first primitive | count << 16
      Prim q;
      const int k = (int)(fc & 0xFFFFu);
      q.q0 = s_rec[4 * k];
      q.q1 = s_rec[4 * k + 1];
      q.q2 = s_rec[4 * k + 2];
      q.q3 = s_rec[4 * k + 3];
      if constexpr (CNT) ++tc->tri;
      bw_closest_update(r.o, r.d, q, pstart + k, bt, bp);
      if (fc >> 17) {
        q.q0 = s_rec[4 * k + 4];
        q.q1 = s_rec[4 * k + 5];
        q.q2 = s_rec[4 * k + 6];
        q.q3 = s_rec[4 * k + 7];
        if constexpr (CNT) ++tc->tri;
        bw_closest_update(r.o, r.d, q, pstart + k + 1, bt, bp);
      }
    }
    while (cs) {
      const int c = __builtin_ctz(cs);
      cs &= cs - 1u;
      const int k = (int)(s_cl[c] & 0xFFFFu);
      if constexpr (CNT) ++tc->sph;
      const float tt = sphere_test(r.o, r.d, s_rec[4 * k], s_rec[4 * k + 1]);
      const int gi = pstart + k;
      const bool take = (tt >= 0.0f) & ((tt < bt) | ((tt == bt) & (gi < bp)));
      bt = take ? tt : bt;
      bp = take ? gi : bp;
    }
  } else {
    while (cm) {
      const int c = __builtin_ctz(cm);
      cm &= cm - 1u;
      const uint32_t fc = s_cl[c];  // first primitive | count << 16
      step((int)(fc & 0xFFFFu));
      if (fc >> 17) step((int)(fc & 0xFFFFu) + 1);
    }
  }
  prim = bp < 0 ? PT_PRIM_NONE : (uint32_t)bp;
  t = bt;
}

// The shadow rays' occlusion query over the same clusters, done at the first
// hit (round 5: CBempty 93,200 -> 101,000 Mrays/s, CBspheres 59,080 ->
// 61,050).  A shadow segment is tested against the clusters as an overlap
// test of its bounding box with each cluster's box (6 compares with scalar
// bounds, combined on the scalar unit) instead of the slab test, then the
// same per-lane candidate loop.
// Conservative as the slab test: a hit point fma(t, d, o) with t in [0, tmax]
// lies between o and e = fma(tmax, d, o) on every axis (fma is monotone in
// t), so within the segment's box; a cluster's box holds every point where
// its triangles' tests can report a hit (the guard band).  CBempty 105,400 ->
// 111,600 Mrays/s, CBspheres 64,800 -> 66,800 (interleaved A/B, 2 runs each;
// looping over the clusters wave-uniformly instead, testing a cluster for the
// lanes that overlap it whenever any lane does, lost 8 %: a wave's 64 lanes
// lie on every wall, and a grazing incident ray leaves its shadow ray's
// origin within the band of its own wall)
template <bool SPH, bool CNT = false>
__device__ __forceinline__ bool leaf_occluded_aabb(const ShadeArgs& S, const float4* s_rec, const uint32_t* s_cl,
                                                   const RayV& r, TestCount* tc = nullptr) {
  // (an unbounded segment -- a directional or hemisphere light -- as one of
  // length 2^127: no hit lies beyond it, and e stays finite for a unit d)
  const float tm = fminf(r.tmax, 0x1p127f);
  const f3 e = mk(__builtin_fmaf(tm, r.d.x, r.o.x), __builtin_fmaf(tm, r.d.y, r.o.y), __builtin_fmaf(tm, r.d.z, r.o.z));
  const f3 lo = mk(fminf(r.o.x, e.x), fminf(r.o.y, e.y), fminf(r.o.z, e.z));
  const f3 hi = mk(fmaxf(r.o.x, e.x), fmaxf(r.o.y, e.y), fmaxf(r.o.z, e.z));
  const CPTR(f4v) B = (const CPTR(f4v))S.cbox;
  bool hit = false;
  auto test = [&](int k) -> bool {
    Prim q;
    q.q0 = s_rec[4 * k];
    q.q1 = s_rec[4 * k + 1];
    q.q2 = s_rec[4 * k + 2];
    q.q3 = s_rec[4 * k + 3];
    if constexpr (CNT) {
      if (SPH && prim_sphere<false>(q)) ++tc->sph;
      else ++tc->tri;
    }
    if (SPH && prim_sphere<false>(q)) {
      const float tt = sphere_test(r.o, r.d, q.q0, q.q1);
      return (tt >= 0.0f) & (tt <= r.tmax);
    }
    float ndd, num;
    plane_nd<false>(r.o, r.d, q, ndd, num);
    return !tri_outside<false>(ndd, num, r.tmax) && bw_occludes(r.o, r.d, q, num, ndd, r.tmax);
  };
  if constexpr (CNT) tc->box += (uint32_t)S.nclus;
  uint32_t cm = 0u;
  for (int c = 0; c < S.nclus; ++c) {
    const float4 b0 = f4(B[2 * c]), b1 = f4(B[2 * c + 1]);
    const bool ov = !((hi.x < b0.x) | (lo.x > b0.y) | (hi.y < b0.z) | (lo.y > b0.w) | (hi.z < b1.x) | (lo.z > b1.y));
    cm = mask_bit(cm, ov, c);
  }
  // (SPH: the triangle candidates, then the spheres, as in leaf_closest_cl)
  uint32_t cs = 0u;
  if constexpr (SPH) {
    cs = cm & S.sph_cl;
    cm &= ~S.sph_cl;
  }
  while (cm && !hit) {
    const int c = __builtin_ctz(cm);
    cm &= cm - 1u;
    const uint32_t fc = s_cl[c];
    hit = test((int)(fc & 0xFFFFu));
    if (!hit && (fc >> 17)) hit = test((int)(fc & 0xFFFFu) + 1);
  }
  if constexpr (SPH) {
    while (cs && !hit) {
      const int c = __builtin_ctz(cs);
      cs &= cs - 1u;
      const int k = (int)(s_cl[c] & 0xFFFFu);
      if constexpr (CNT) ++tc->sph;
      const float tt = sphere_test(r.o, r.d, s_rec[4 * k], s_rec[4 * k + 1]);
      hit = (tt >= 0.0f) & (tt <= r.tmax);
    }
  }
  return hit;
}

// any primitive at t in [0, tmax]; triangles whose plane hit is certainly
// outside [0, tmax] for every lane (tri_outside: shadow rays toward the light
// mostly point away from the walls or end before them) cost no division;
// the answer is a bitwise mask update (no exec-mask branch per primitive:
// +1-2 %, round 4), a triangle's straight from the test's own compares
// (bw_occludes) on the pre-test's num / ndd (+1.4 % CBempty, round 4)
template <bool REFA, bool SPH = true>
__device__ __forceinline__ bool leaf_occluded(const float4* prims, int pstart, int pcount, const RayV& r) {
  constexpr int PS = prim_stride<REFA>();
  const CPTR(f4v) P = (const CPTR(f4v))(prims + (size_t)pstart * PS);
  bool hit = false;
  int k0 = 0;
  if constexpr (!REFA) {
    auto test = [&](const Prim& q) -> bool {
      if (!SPH || !prim_sphere<REFA>(q)) {
        float ndd, num;
        plane_nd<REFA>(r.o, r.d, q, ndd, num);
        return !tri_outside<REFA>(ndd, num, r.tmax) && bw_occludes(r.o, r.d, q, num, ndd, r.tmax);
      }
      const float tt = sphere_test(r.o, r.d, q.q0, q.q1);
      return (tt >= 0.0f) & (tt <= r.tmax);
    };
    for (; k0 + 1 < pcount; k0 += 2, P += 2 * PS) {
      Prim qa, qb;
      load_prim_pair(P, qa, qb);
      hit = hit | test(qa);
      hit = hit | test(qb);
      if (__ballot(!hit) == 0ull) return hit;  // every active lane is occluded
    }
  }
  for (int k = k0; k < pcount; ++k, P += PS) {
    const Prim q = load_prim<REFA>(P);
    float tt = -1.0f;
    if (SPH && prim_sphere<REFA>(q)) {
      tt = sphere_test(r.o, r.d, q.q0, q.q1);
    } else {
      float ndd, num;
      plane_nd<REFA>(r.o, r.d, q, ndd, num);
      if (!tri_outside<REFA>(ndd, num, r.tmax)) tt = tri_test<REFA>(r.o, r.d, q, r.tmax);
    }
    // (no short-circuit: one mask update, no exec-mask branch per primitive)
    hit = hit | ((tt >= 0.0f) & (tt <= r.tmax));
    if (__ballot(!hit) == 0ull) break;  // every active lane is occluded
  }
  return hit;
}

// Path regeneration (persistent waves).  A wave of 64 independent paths would
// run as long as its longest path (up to max_bounces + 2 vertices) while the
// mean path has ~4: most lanes would sit idle.  Instead every lane whose path
// has ended takes the next unstarted path from its wave's pool, and the wave
// refills the pool from a global counter in chunks of PATH_CHUNK paths; the
// grid is sized to the resident wave count, every wave exits once the counter
// passes N and its lanes are idle.  Results do not depend on which lane runs a
// path: random numbers are keyed by (pixel, sample, vertex) and each path
// writes only its own slot ps1[p].
// Philox products as v_mad_u64_u32 (CBempty +1.4 %).  The vertex's Philox
// words are computed where they are used, not early as in k_shade_push (in
// k_path_leaf the shading record is an L2 hit and nothing waits on it long);
// with the light held in registers, at the final round-5 code: CBempty 17.66
// -> 17.2 ms per frame, CBspheres 28.6 -> 26.6 (v_mul_hi_u32 + v_mul_lo_u32
// instead of v_mad_u64_u32 measured slower in that configuration).
constexpr bool PATH_MAD64 = true, PATH_RNG_EARLY = false;
// paths a wave takes from the global counter at a time for a whole frame
// (CBempty: 128: -1.3 %, 512: +1.6 %, 1024: +1.4 %, 2048: +0.1 % against 256;
// re-measured in round 3: 1024 -0.3 %, 256 -1.2 % against 512; round 5: 1024
// -0.5 %, 256 -1.6 %); the guided schedule's largest chunk.  The plain grabs
// take the launch's `chunk` (pt_ctx::path_chunk_for: smaller for a small
// launch, whose tail is about one chunk's time)
constexpr uint32_t PATH_CHUNK = 512;

// With all path state in registers: 6 waves per SIMD (80 VGPRs, no spills);
// 7 waves (72 VGPRs) ran within 0.6 % of it but spilled ~20 VGPRs around the
// shading code (~35 GB of scratch write-back per 1024^2 x 256 spp frame, PMC
// WRITE_SIZE); 8 waves spilled ~60 and lost 10 %.  8 waves per SIMD with the
// radiance and the throughput in LDS (16 KB per workgroup while the pending
// shadow rays were kept there too): 64 VGPRs; CBempty 51,700 -> 54,700
// Mrays/s, CBspheres 38,500 -> 40,800 (7 waves: 68 VGPRs without spills,
// 54,000).
constexpr int PATH_WAVES = 8;
// The light: held in registers (round 5, at the final code: CBempty 17.55 ->
// 17.25 ms per frame, CBspheres 28.48 -> 27.03 against re-reading it from the
// kernel arguments at each NEE sample, which had cut SGPR spills 34 -> 13 in
// round 2); the extended-light variants (XL) keep the re-read (their
// registers).  The camera is re-read from the kernel arguments at each path
// start (cam_of).  Both re-reads read the kernel-argument segment at
// offsetof(ShadeArgs, ...): S must stay this kernel's FIRST parameter (checked
// at every launch, below).  Refilling idle lanes only once k of a wave's 64
// are idle measured slower (k = 4, 8, 16: CBempty -0.6 / +0.0 / -0.9 %,
// CBspheres -0.2 / -0.2 / -2.3 %, round 5): every idle lane refills.
// Path grabs (round 6): the launch's paths are split into `grab_nreg`
// contiguous path regions of `grab_region` paths, one counter each (128 B
// apart); a wave takes `grab_chunk` paths at a time from its region (its
// workgroup's, blockIdx % nreg) and moves on to the next region when that one
// is dry; it exits once every region is.  One counter for the whole launch
// saturated near 90 M grabs/s (a CBempty frame in 128-path chunks took 24.5
// instead of 16.8 ms), and a launch's tail is about one chunk's time: the
// host picks the chunk by the launch's paths per resident lane (pt_render).
// The grab's operands are re-read from the kernel-argument segment and the
// wave's region state lives in LDS, so the path loop holds none of them in
// SGPRs (held there they spilled 64 SGPRs to VGPR lanes instead of 28, and a
// whole frame ran 8 % slower).  Round 2-5's guided schedule (chunks halving
// from 512 to 64 as the paths ran out, its phase arithmetic in SGPRs) is gone:
// it lost on whole frames (2.6 %) and, at the round-5 kernels, on the 1/8
// share too.
constexpr uint32_t PATH_REGIONS_MAX = 32;
constexpr uint32_t PATH_CTR_STRIDE = 32;  // u32s between region counters (128 B)

// PT_PATH_TIMING (diagnostic build only): per-wave wall-clock marks (entry,
// first empty grab, exit, chunks taken) for pt_dbg_path_timing
#ifndef PT_PATH_TIMING
#define PT_PATH_TIMING 0
#endif
#if PT_PATH_TIMING
constexpr uint32_t PT_TIMING_WAVES = 16384;
static __device__ unsigned long long g_path_timing[PT_TIMING_WAVES * 8];
#endif
// SPH: the leaf holds spheres (false: the sphere test is not compiled in; the
// host picks the variant, pt_ctx::has_sphere)
// CNT: the counting variant (PT_FLAG_COUNT_TESTS): executed tests into
// rcount's lines (words 1-3 of each 128-B counter line)
template <int NSH, bool REFA, bool SPH = true, bool XL = false, bool CNT = false>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(PATH_WAVES, 8))) void k_path_leaf(
    ShadeArgs S, int pstart, int pcount, int passes, unsigned long long* __restrict__ rcount,
    uint32_t* __restrict__ err) {
  const uint32_t lid = lane_id();
  // light_of<true> reads the light at offsetof(ShadeArgs, light) of the
  // kernel-argument segment, so S must stay this kernel's FIRST parameter:
  // checked at every launch (wave-uniform, a few cached scalar loads); a
  // mismatch sets ERR_KERNARG and the kernel does nothing (pt_render fails)
  {
    const pt_light a = light_of<true>(S), b = S.light;
    const pt_camera ca = cam_of<true>(S), cb = S.cam;
    uint32_t wa[sizeof a / 4], wb[sizeof b / 4], wc[sizeof ca / 4], wd[sizeof cb / 4];
    __builtin_memcpy(wa, &a, sizeof a);
    __builtin_memcpy(wb, &b, sizeof b);
    __builtin_memcpy(wc, &ca, sizeof ca);
    __builtin_memcpy(wd, &cb, sizeof cb);
    bool same = true;
#pragma unroll
    for (uint32_t i = 0; i < sizeof a / 4; ++i) same = same && wa[i] == wb[i];
#pragma unroll
    for (uint32_t i = 0; i < sizeof ca / 4; ++i) same = same && wc[i] == wd[i];
    if (!same) {
      if (threadIdx.x == 0) atomicOr(err, ERR_KERNARG);
      return;
    }
  }
  // Pipelined frames (pt_render, PT_FLAG_ASYNC): the first acc_blocks
  // workgroups sum the previous launch's results (k_accum's work, its sums
  // bit for bit) and exit.  Dispatched first, they hold a few of the slots
  // the path workgroups would take while the rest start paths; the path
  // workgroups behind them start as they exit (persistent waves grab their
  // paths, so a late start only means fewer grabs).  Memory-bound sums beside
  // the VALU-bound paths instead of a bandwidth-bound k_accum after them.
  // (Measured and rejected: the frame's copy to the host carried the same way
  // by leading workgroups writing the pinned buffer -- 16.53 against 16.42 ms
  // per CBempty frame with the copy on the copy stream.)
  {
    const uint32_t na = S.acc_blocks;
    if (blockIdx.x < na) {
      const uint32_t n = S.acc_npix;
      for (uint32_t q = blockIdx.x * TPB + threadIdx.x; q < n; q += na * TPB)
        accum_pixel(S.acc_res, S.acc_dst, S.acc_slot, n, S.acc_spp, q);
      return;
    }
  }
  const uint32_t wg = blockIdx.x - S.acc_blocks;  // (the path workgroup's index)
  // candidate clusters: the leaf's records in LDS for the per-lane candidate loop
  __shared__ float4 s_rec[PATH_CL_PRIMS * 4];
  __shared__ uint32_t s_cl[PATH_CL_PRIMS];
  const bool use_cl = !REFA && S.nclus > 0 && pcount <= PATH_CL_PRIMS;
  if (use_cl) {
    for (int i = threadIdx.x; i < pcount * 4; i += TPB) s_rec[i] = S.prims[(size_t)pstart * 4 + i];
    for (int i = threadIdx.x; i < S.nclus; i += TPB)
      s_cl[i] = __float_as_uint(S.cbox[8 * i + 6]) | (__float_as_uint(S.cbox[8 * i + 7]) << 16);
    __syncthreads();
  }
  // rays traced by the wave (wave-uniform, counted from ballots: no VGPR)
  uint32_t nrays = 0;
  // per wave: the path region it grabs from (its workgroup's, then the next
  // ones as they run dry) and how many regions it has found dry
  __shared__ uint32_t s_grab[TPB / 64][2];
  if (lid == 0) {
    s_grab[threadIdx.x >> 6][0] = wg % S.grab_nreg;
    s_grab[threadIdx.x >> 6][1] = 0u;
  }
#if PT_PATH_TIMING
  const unsigned long long tm0 = wall_clock64();
  unsigned long long tm_drain = 0, tm_grab = 0, tm_grab_max = 0;
  uint32_t nchunks = 0;
#endif
  // wave-uniform pool [next, end) of unstarted paths; `drained`: the global
  // counter has passed N
  uint32_t next = 0, end = 0;
  bool drained = false;
  bool active = false;
  // Camera rays made in batches (round 6): the wave computes the camera rays
  // of the pool's next up to 64 paths with every lane at once into a ring in
  // LDS (s_cam: {dir, pixel} and the path, per wave), and idle lanes start
  // their paths from the ring's head -- the same path for the same lane as
  // taking them straight from the pool.  Made where a lane refills, the camera
  // ray cost the wave a whole divergent camera_dir per iteration (~15 of 64
  // lanes refill at each vertex of a ~4-vertex mean path).
  __shared__ float4 s_cam[TPB / 64][64];
  __shared__ uint32_t s_camp[TPB / 64][64];
  float4* const cam_ring = s_cam[threadIdx.x >> 6];
  uint32_t* const camp_ring = s_camp[threadIdx.x >> 6];
  uint32_t fhead = 0, fcount = 0;  // (wave-uniform) ring head and entries
  // the lane's path index lives in LDS between its uses (camera ray, sample
  // index, result): one VGPR less across the vertex loop
  __shared__ uint32_t sh_p[TPB];
  PathState st{mk(0, 0, 0), 0u, mk(0, 0, 0), 0u};
  RayV ext{mk(0, 0, 0), mk(0, 0, 1), -1.0f}, shr[NSH];
  f3 C[NSH];
#pragma unroll
  for (int s = 0; s < NSH; ++s) {
    shr[s] = RayV{mk(0, 0, 0), mk(0, 0, 1), -1.0f};
    C[s] = mk(0, 0, 0);
  }
  // Shadow rays are tested where their NEE sample makes them (shade_vertex's
  // IMM), none pending between vertices (round 5: no shadow ray in LDS, 16 ->
  // 6 KB of LDS per workgroup, no iteration that only resolves a path's last
  // shadow ray; CBempty 18.07 -> 17.73 ms per frame).  The path's radiance and
  // throughput live in LDS (sh_lds, stride-1 columns).
  // (XL: the light re-read keeps the extended-light variants' registers down,
  // 136 B of scratch without it)
  constexpr bool M64P = PATH_MAD64, LRP = XL, EARLYP = PATH_RNG_EARLY;
  __shared__ float sh_lds[6 * TPB];
  float* const Lq = sh_lds + threadIdx.x;  // (the radiance, then the throughput)
  TestCount tc{0u, 0u, 0u};  // (CNT only)
  // the occlusion query of one shadow ray
  auto occluded = [&](const RayV& r) -> bool {
    if (use_cl) return leaf_occluded_aabb<SPH, CNT>(S, s_rec, s_cl, r, &tc);
    if constexpr (CNT) tc.tri += (uint32_t)pcount;  // (the full loop: an upper bound)
    return leaf_occluded<REFA, SPH>(S.prims, pstart, pcount, r);
  };
  for (;;) {
    // ---- refill idle lanes from the camera-ray ring (new paths start at their camera ray)
    const unsigned long long idle = __ballot(!active);
    const uint32_t nidle = (uint32_t)__popcll(idle);
    // top the ring up in batches until it holds a ray for every idle lane (or
    // the paths have run out): at most a few rounds, fully active
    while (idle && fcount < nidle && !(drained && next == end)) {
      if (next < end) {
        const uint32_t m = min(64u - fcount, end - next);
        if (lid < m) {
          const uint32_t p = next + lid;
          uint32_t g;
          const f3 dir = camera_dir<M64P, REFA, true>(S, p, g);
          const uint32_t at = (fhead + fcount + lid) & 63u;
          cam_ring[at] = make_float4(dir.x, dir.y, dir.z, __uint_as_float(g));
          camp_ring[at] = p;
        }
        fcount += m;
        next += m;
        continue;
      }
#if PT_PATH_TIMING
      const unsigned long long tg = wall_clock64();
#endif
      uint32_t b = 0, e = 0, dry = 0;
      if (lid == 0) {
        // (the grab's operands from the kernel-argument segment, opaque to the
        // compiler: not held in SGPRs across the path loop)
        const CPTR(char) kp = (const CPTR(char))__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        const CPTR(uint32_t) ga = (const CPTR(uint32_t))(kp + offsetof(ShadeArgs, grab_chunk));
        const uint32_t chunk = ga[0], region = ga[1], nreg = ga[2];
        typedef uint32_t* wptr_t;
        uint32_t* const work = *(const CPTR(wptr_t))(kp + offsetof(ShadeArgs, grab_work));
        uint32_t* const gs = s_grab[threadIdx.x >> 6];
        uint32_t reg = gs[0], tried = gs[1];
        while (tried < nreg) {
          const uint32_t lo = reg * region, hi = min(lo + region, S.N);
          const uint32_t k = atomicAdd(work + reg * PATH_CTR_STRIDE, chunk);
          if (k < hi - lo) {
            b = lo + k;
            e = min(b + chunk, hi);
            break;
          }
          reg = reg + 1 == nreg ? 0u : reg + 1;
          ++tried;
        }
        gs[0] = reg;
        gs[1] = tried;
        dry = tried >= nreg ? 1u : 0u;
      }
      b = __builtin_amdgcn_readfirstlane(b);
      e = __builtin_amdgcn_readfirstlane(e);
      drained = __builtin_amdgcn_readfirstlane(dry) != 0u;
      next = drained ? 0u : b;
      end = drained ? 0u : e;
#if PT_PATH_TIMING
      const unsigned long long dt = wall_clock64() - tg;
      tm_grab += dt;
      tm_grab_max = dt > tm_grab_max ? dt : tm_grab_max;
      if (drained) tm_drain = wall_clock64();
      else ++nchunks;
#endif
    }
    if (idle && fcount) {
      const uint32_t r = mbcnt64(idle);
      if (!active && r < fcount) {
        const uint32_t at = (fhead + r) & 63u;
        const float4 c = cam_ring[at];
        const uint32_t p = camp_ring[at];
        sh_p[threadIdx.x] = p;
        active = true;
        const f3 dir = mk(c.x, c.y, c.z);
        st.g = __float_as_uint(c.w);
        st.T = mk(1.0f, 1.0f, 1.0f);
        st.L = mk(0.0f, 0.0f, 0.0f);
        Lq[0] = 0.0f;
        Lq[TPB] = 0.0f;
        Lq[2 * TPB] = 0.0f;
        Lq[3 * TPB] = 1.0f;  // (the throughput)
        Lq[4 * TPB] = 1.0f;
        Lq[5 * TPB] = 1.0f;
        st.flags = F_EXT | (1u << 8);
        ext = RayV{ld3(cam_of<true>(S).origin), dir, __builtin_inff()};
      }
      const uint32_t used = min(nidle, fcount);
      fhead = (fhead + used) & 63u;
      fcount -= used;
    }
    if (!__any(active)) break;  // (the paths have run out: the ring is filled whenever any remain)
    // ---- one vertex of every active path: leaf tests, then shade
    nrays += (uint32_t)__popcll(__ballot(active && (st.flags & F_EXT)));
    uint32_t cast_sh = 0u;  // (the shadow rays this vertex cast, counted below in uniform control flow)
    if (active) {
      uint32_t prim = PT_PRIM_NONE;
      float t = 0.0f;
      if (st.flags & F_EXT) {
        // (extension rays have tmax = inf: not carried across iterations)
        if (use_cl) {
          leaf_closest_cl<SPH, CNT>(S, s_rec, s_cl, pstart, pcount, RayV{ext.o, ext.d, __builtin_inff()}, prim, t, &tc);
        } else {
          if constexpr (CNT) tc.tri += (uint32_t)pcount;
          leaf_closest<REFA, SPH>(S.prims, pstart, pcount, RayV{ext.o, ext.d, __builtin_inff()}, prim, t);
        }
      }
      bool clear[NSH];
#pragma unroll
      for (int s = 0; s < NSH; ++s) {
        clear[s] = false;  // (no shadow ray pending from the last vertex)
        shr[s] = RayV{mk(0, 0, 0), mk(0, 0, 1), -1.0f};  // (no value carried across iterations in registers)
        C[s] = mk(0, 0, 0);
      }
      bool new_ext, new_sh[NSH];
      RayV e2, s2[NSH];
      // (the sample index is recomputed, not carried: one register less)
      shade_vertex<NSH, M64P, LRP, REFA, true, XL, decltype(occluded), EARLYP>(
          S, S.sample_base + udiv_q(sh_p[threadIdx.x], S.div_npix), st, ext.o, ext.d, prim, t, clear, C, new_ext, e2,
          new_sh, s2, sh_lds, occluded);
#pragma unroll
      for (int s = 0; s < NSH; ++s) cast_sh |= new_sh[s] ? 1u << s : 0u;  // (cast and resolved)
      // (unconditional: without a new extension ray F_EXT is clear and ext is
      // not read again before the lane's next camera ray -- the old ray need
      // not stay live through shade_vertex)
      ext = e2;
      // vertices done = vtx - 1 (shade_vertex advanced it); the path ends
      // after `passes` of them or when it has no ray left to trace
      const uint32_t done = ((st.flags >> 8) & 0xffu) - 1u;
      if (!(st.flags & (F_EXT | F_SHADOW | F_SHADOW2)) || done >= (uint32_t)passes) {
        st.L = mk(Lq[0], Lq[TPB], Lq[2 * TPB]);
        put_res(S.ps1, sh_p[threadIdx.x], st.L);
        active = false;
      }
    }
#pragma unroll
    for (int s = 0; s < NSH; ++s) nrays += (uint32_t)__popcll(__ballot((cast_sh >> s) & 1u));
  }
  // rays traced (R): one fire-and-forget atomic per wave into its lane's counter
  const uint32_t w = __builtin_amdgcn_readfirstlane(nrays);
  if (lid == 0 && w)
    atomicAdd(rcount + (size_t)((wg * 4 + (threadIdx.x >> 6)) & (RCOUNT_SLOTS - 1)) * 16,
              (unsigned long long)w);
  if constexpr (CNT) {  // the wave's executed tests (64-bit sums: a lane's u32 counts cannot overflow them)
    unsigned long long v[3] = {tc.tri, tc.sph, tc.box};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v[j] += __shfl_xor(v[j], o);
    }
    if (lid == 0) {
      unsigned long long* line = rcount + (size_t)((wg * 4 + (threadIdx.x >> 6)) & (RCOUNT_SLOTS - 1)) * 16;
      for (int j = 0; j < 3; ++j)
        if (v[j]) atomicAdd(line + 1 + j, v[j]);
    }
  }
#if PT_PATH_TIMING
  const uint32_t gw = wg * (TPB / 64) + (threadIdx.x >> 6);
  if (lid == 0 && gw < PT_TIMING_WAVES) {
    unsigned long long* o = g_path_timing + (size_t)gw * 8;
    o[0] = tm0;
    o[1] = tm_drain;
    o[2] = wall_clock64();
    o[3] = nchunks;
    o[4] = tm_grab;
    o[5] = tm_grab_max;
  }
#endif
}

// (accum_pixel for every active pixel of a batch)
__global__ __launch_bounds__(TPB) void k_accum(const float4* __restrict__ ps1, float4* accum,
                                               const uint32_t* __restrict__ slot, uint32_t npix, uint32_t spp_b) {
  const uint32_t q = blockIdx.x * TPB + threadIdx.x;
  if (q < npix) accum_pixel(ps1, accum, slot, npix, spp_b, q);
}

// Repack pt_intersect's 8-float rays {o, tmax, d, 0} into ray records.
__global__ __launch_bounds__(TPB) void k_load_rays(const float4* __restrict__ in, float4* ray, uint32_t n) {
  const uint32_t i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const float4 a = in[2 * i], b = in[2 * i + 1];
  ray[RSTRIDE * i] = make_float4(a.x, a.y, a.z, b.x);
  ray[RSTRIDE * i + 1] = rec_r1(b.y, b.z, a.w);
}

// Closest-hit keys of pt_intersect: {t bits, prim} or PT_HIT_NONE.
__global__ __launch_bounds__(TPB) void k_store_hits(const float4* __restrict__ ray, unsigned long long* out,
                                                    uint32_t n) {
  const uint32_t i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const float4 r1 = ray[RSTRIDE * i + 1];
  const uint32_t prim = __float_as_uint(r1.z);
  out[i] = prim == PT_PRIM_NONE ? PT_HIT_NONE
                                : (((unsigned long long)__float_as_uint(r1.w) << 32) | (unsigned long long)prim);
}

}  // namespace pt
