// Shared definitions of the traversal and shading kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_api.h"
#include "ptmath.h"

// Pointer into the constant address space: uniform loads through it become
// scalar (s_load) instead of per-lane vector loads.
#define CPTR(T) __attribute__((address_space(4))) T*

namespace pt {

typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 f4(f4v v) { return make_float4(v.x, v.y, v.z, v.w); }

// A ray record is 32 B, two float4 (a scattered gather of one ray touches one
// 64-B half line):  r0 = {o.x, o.y, o.z, d.x},  r1 = {d.y, d.z, prim, t}.
// {prim (low dword), t bits (high dword)} is the 64-bit closest-hit key: it
// starts as {PT_PRIM_NONE, tmax} (t < 0 marks an empty slot) and leaves lower
// it with atomicMin, so t is also the ray's current tmax (inclusive).
constexpr int RSTRIDE = 2;        // float4 per ray record
constexpr uint32_t PT_PRIM_NONE = 0xFFFFFFFFu;
constexpr int TPB = 256;          // threads per workgroup (4 waves)
constexpr int RPT = 4;            // rays per thread in a traversal item
constexpr int TILE = TPB * RPT;   // rays per traversal item
// a level runs 1024-ray workgroup items when its (node, lane) queues hold
// this many rays on average, wave items otherwise (BLOCK_MODE_RAYS_PER_PAIR;
// dragon proxy levels: 512: 135 ms, 1024: 130, 4096: 130, 16384: 131, wave
// items only: 132).  Level-kernel workgroups LEVEL_GRID: 16384 (vs 8192:
// dragon proxy levels -4 %; 2048 -15 %, 32768 within noise).  Rays per lane of
// a wave item RPTW (2: same, 8: -30 % on the dragon proxy).
constexpr int RPTW = 4;           // rays per lane in a wave-sized item
constexpr int WTILE = 64 * RPTW;  // rays per wave item (levels >= 1)
constexpr int NLANE = 8;          // queue lanes (one per XCD)
constexpr int CSTRIDE = 32;       // u32 per queue counter: each (node, lane) counter owns a 128-B line
constexpr uint32_t MODE_WAVE = 0, MODE_BLOCK = 1;
constexpr uint32_t BLOCK_MODE_RAYS_PER_PAIR = 4096;  // level mode threshold (mean rays per queue lane)
constexpr int LEVEL_GRID = 16384;  // workgroups of the level kernel (64 per CU: the
                                   // dispatcher's refill balances uneven items)
constexpr int RCOUNT_SLOTS = 64;  // ray counters (u64, 128 B apart), indexed by workgroup & 63

// device statistics slots (unsigned long long)
enum {
  STAT_R = 0,
  STAT_V = 1,
  STAT_PEAKQ = 2,
  STAT_LV0 = 8,     // 16 per-level visit counters
  STAT_LEAF0 = 24,  // 16 per-level leaf-visit counters
  STAT_ITEMS0 = 40, // 16 per-level item counters
  STAT_SHADED = 56, // path vertices shaded by k_shade_push
  STAT_COUNT = 64
};

struct TraceArgs {
  const pt_node* __restrict__ nodes;
  const float4* __restrict__ prims;  // 6 float4 per primitive
  float4* ray;                       // ray records (RSTRIDE float4 each)
  uint32_t* cnt;                     // [node][lane] rays pushed into the node
  uint32_t* qoff;                    // [node][lane] absolute queue offset
  uint32_t* q;                       // ray-id queues of the root pass's targets (4 B ids)
  float4* qe;                        // ray-entry queues of the levels below (two parity halves):
                                     // QESTRIDE float4 per entry, {o, d.x}{d.y, d.z, id, tmax}
  uint32_t shadow_base;              // ray slots >= shadow_base are shadow rays (any hit ends them);
                                     // 0xFFFFFFFF: every ray wants its closest hit (pt_intersect)
  const float* __restrict__ tmin;    // per ray slot t_min (pt_intersect, TMIN kernels only; else unused)
  // capacities, checked only by a -DPT_DBG_BOUNDS build (a debugging aid)
  uint32_t dbg_nslots;               // ray records
  uint32_t dbg_nnodes;
  uint64_t dbg_qids;                 // ids in q (all regions)
  uint32_t dbg_nprims;               // primitives (hit keys, shading records)
};
#ifdef PT_DBG_BOUNDS
#define PT_CHECK(cond, what, a, b)                                                                  \
  if (!(cond)) {                                                                                    \
    printf("PT_DBG_BOUNDS %s: %llu vs %llu (block %d thread %d)\n", what, (unsigned long long)(a), \
           (unsigned long long)(b), (int)blockIdx.x, (int)threadIdx.x);                             \
    return;                                                                                         \
  }
#else
#define PT_CHECK(cond, what, a, b)
#endif
constexpr int QESTRIDE = 2;

// A leaf's hit {t, prim} for ray id.  Closest-hit rays: atomicMin on the
// record's key (its t is the tmax of every later box test).  Shadow rays only
// need to know that something blocks them: a plain store of {prim, t = -1}
// marks the ray occluded (prim != PT_PRIM_NONE) and fails every later box
// test (tmax < 0), so an occluded shadow ray leaves the traversal at once.
__device__ __forceinline__ unsigned long long* rec_key(float4* ray, uint32_t id);
__device__ __forceinline__ void report_hit(float4* ray, uint32_t shadow_base, uint32_t id, float t, uint32_t prim) {
  if (id >= shadow_base) {
    *rec_key(ray, id) = ((unsigned long long)__float_as_uint(-1.0f) << 32) | (unsigned long long)prim;
  } else {
    atomicMin(rec_key(ray, id), ((unsigned long long)__float_as_uint(t) << 32) | (unsigned long long)prim);
  }
}
__device__ __forceinline__ unsigned long long* rec_key(float4* ray, uint32_t id) {
  return reinterpret_cast<unsigned long long*>(ray + (size_t)RSTRIDE * id + 1) + 1;
}
__device__ __forceinline__ float4 rec_r1(float dy, float dz, float tmax) {
  return make_float4(dy, dz, __uint_as_float(PT_PRIM_NONE), tmax);
}

__host__ __device__ inline size_t cnt_idx(int node, int lane) { return ((size_t)node * NLANE + lane) * CSTRIDE; }

// The root pass (fused into the ray producers, or k_trace_root): small leaves
// among the root's children / grandchildren are tested right there ("inline
// leaves": their closest hit becomes the ray's initial key and tmax, and a
// shadow ray occluded by one is never queued); every other ray is pushed into
// the queues of the targets (nodes of one level, 1 or 2) whose boxes it hits.
constexpr int MAX_ROOT_TARGETS = 16, MAX_INLINE_LEAVES = 4;
struct RootTable {
  int nt;                          // queue targets
  int tnode[MAX_ROOT_TARGETS];     // target node ids
  int tbox[MAX_ROOT_TARGETS];      // parent * 4 + slot: where the target's box is stored
  int ni;                          // inline leaves
  int ibox[MAX_INLINE_LEAVES];     // parent * 4 + slot of the leaf's box
  int istart[MAX_INLINE_LEAVES];   // its primitives
  int icount[MAX_INLINE_LEAVES];
  // the boxes themselves ({bmin_x, bmax_x, bmin_y, bmax_y, bmin_z, bmax_z}
  // rows), so the root pass reads them from the kernel arguments in a few wide
  // scalar loads instead of six dword loads per box from the node array
  float tb[6][MAX_ROOT_TARGETS];
  float ib[6][MAX_INLINE_LEAVES];
  // candidate clusters of the inline leaves' primitives (PT_ROOT_CLUSTER,
  // pt_device.hip root_clusters; nc = 0: none): cbox, 8 floats per cluster,
  // its box as the rows above; cinfo[c] = first member | member count << 16,
  // cinfo[ROOT_CL_MAX + m] = member m's primitive, its record at cmem[4m ..
  // 4m + 3] (cmem: 4 ROOT_CL_MAX records, cinfo: 2 ROOT_CL_MAX words, zero-padded:
  // copied whole into LDS by the shade kernel)
  int nc;
  int nc_shadow;  // nc, or 0: shadow rays take the leaf loop (PT_NO_ROOT_CLUSTER_SHADOW)
  const float* cbox;
  const float4* cmem;
  const float4* cmem_ref;  // the members' PT_FLAG_REF_ARITH records, 6 float4 each (6 ROOT_CL_MAX)
  const uint32_t* cinfo;
};
constexpr int ROOT_CL_MAX = 32;  // members (and so clusters) at most

struct LevelArgs {
  int first;  // first node id of the level
  int nl;     // nodes in the level
  int maxln;  // row stride - 1 of iprefix
  const uint32_t* iprefix;  // [lane][maxln+1] exclusive item prefix (read)
  uint32_t* iprefix_w;      // same array (written by the scan)
  const uint32_t* icnt;     // [lane][maxln+1] ray count snapshot of the level (read)
  uint32_t* icnt_w;
  const uint32_t* nitems;   // items of the level (read)
  uint32_t* nitems_w;
  const uint32_t* mode;  // MODE_WAVE / MODE_BLOCK, chosen by the scan
  uint32_t* mode_w;
  int ids;      // 1: the level's queues hold ray ids, 0: ray entries
  int out_ids;  // format of the queues it pushes into (the next level's ids)
  // two-level traversal (pt_device.hip trace_levels): on a "real" level an
  // interior node's rays go straight to its leaf children and to the children
  // of its interior children (two BVH levels per visit); interior nodes of the
  // levels in between are never queued and allocate nothing
  int real;       // interior nodes of this level receive rays and allocate their targets
  int two_level;  // their targets are leaf children + grandchildren (else the 4 children)
};

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

}  // namespace pt
