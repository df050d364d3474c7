// GPU BVH build: a binary BVH built on the device,
// collapsed to the reference's 4-wide, level-major node layout.
//
// The reference builds on the host (bvh.cpp:48-337: per-node full re-sorts on
// three axes and a 12-bucket SAH, O(n log^2 n), 0.84 s for CBbunny) and then
// compacts binary depth 2 into 4-wide nodes (compactTree, DEPTH=2).  Here:
//   1. primitive boxes and centroids             k_prim_bounds
//   2. centroid bounds (ordered-int atomics)     k_reduce_bounds
//   3. 63-bit Morton codes, radix sort           k_morton + hipcub
//   4. binary tree: top-down binned SAH with the reference's split rule
//      (default since round 6, PT_GPU_BVH_SAH, k_sah_*: 12 planes per axis
//      over each node's centroid extent, cost 5 + 2 (SA_l n_l + SA_r n_r) /
//      SA, level-synchronous; the dragon proxy's frames as fast as on the
//      host SAH tree), PLOC agglomerative clustering over Morton order
//      (PT_GPU_BVH_PLOC, k_ploc_*: mutual nearest neighbours by union box
//      area in a Morton-order window, then a depth-first renumbering of the
//      primitives), or the radix tree of Karras 2012 (PT_GPU_BVH_LBVH;
//      k_karras)
//   5. node boxes: made by the merges (PLOC) or bottom-up (k_bottom_up)
//   6. 4-wide collapse, one kernel per level:    k_wide_count / scan / k_wide_emit
//      a node with <= max_leaf primitives is a leaf; otherwise its wide
//      children are its binary grandchildren (binary children that are
//      leaves or small enough stay children) -- the reference's DEPTH=2
//      compaction applied to the LBVH
//   7. primitive records in sorted order         k_prim_records (the exact
//      fp32 operands of bvh_ref.cpp / cu:223-237)
// The result is a pt_scene whose arrays have the same layout as a host-built
// one (pt_scene_get_desc), so everything downstream (pt_load_scene, the
// oracle, pt_intersect) is unchanged.  The tree differs from the reference's
// SAH tree; closest hits do not depend on it.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <climits>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pt_api.h"
#include "scene/scene_internal.h"

namespace ptb {

constexpr int TPB = 256;

struct Box {
  float lo[3], hi[3];
};

__device__ __forceinline__ uint32_t f2ord(float f) {  // order-preserving float -> u32
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
__device__ __forceinline__ float rdown(double v) {
  float f = (float)v;
  if ((double)f > v) f = nextafterf(f, -FLT_MAX);
  return f;
}
__device__ __forceinline__ float rup(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, FLT_MAX);
  return f;
}

// 1. per-primitive box (exact fp32 min/max of the vertices; spheres rounded
//    outward from double like bvh_ref.cpp) and centroid; the stored box is
//    widened by the guard band G (scene_internal.h box_guard: the traversal's
//    fp32 slab test is then conservative), the centroid is the unwidened one
__global__ void k_prim_bounds(const float* __restrict__ pos, int n_tris, const float* __restrict__ sph, int n,
                              double G, Box* __restrict__ box, float* __restrict__ cen) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  Box b;
  if (i < n_tris) {
    const float* p = pos + (size_t)i * 9;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      b.lo[k] = fminf(fminf(p[k], p[3 + k]), p[6 + k]);
      b.hi[k] = fmaxf(fmaxf(p[k], p[3 + k]), p[6 + k]);
    }
  } else {
    const float* s = sph + (size_t)(i - n_tris) * 4;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      b.lo[k] = rdown((double)s[k] - (double)s[3]);
      b.hi[k] = rup((double)s[k] + (double)s[3]);
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) cen[(size_t)i * 3 + k] = 0.5f * (b.lo[k] + b.hi[k]);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    b.lo[k] = rdown((double)b.lo[k] - G);
    b.hi[k] = rup((double)b.hi[k] + G);
  }
  box[i] = b;
}

// 2. centroid bounds: lo[3], hi[3] as ordered u32 (init lo = ~0, hi = 0)
__global__ void k_reduce_bounds(const float* __restrict__ cen, int n, uint32_t* bounds) {
  __shared__ uint32_t s[6];
  if (threadIdx.x < 3) s[threadIdx.x] = 0xFFFFFFFFu;
  else if (threadIdx.x < 6) s[threadIdx.x] = 0u;
  __syncthreads();
  for (int i = blockIdx.x * TPB + threadIdx.x; i < n; i += gridDim.x * TPB) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint32_t o = f2ord(cen[(size_t)i * 3 + k]);
      atomicMin(&s[k], o);
      atomicMax(&s[3 + k], o);
    }
  }
  __syncthreads();
  if (threadIdx.x < 3) atomicMin(&bounds[threadIdx.x], s[threadIdx.x]);
  else if (threadIdx.x < 6) atomicMax(&bounds[threadIdx.x], s[threadIdx.x]);
}

__device__ __forceinline__ uint64_t spread21(uint64_t x) {
  x &= 0x1FFFFFull;
  x = (x | x << 32) & 0x1F00000000FFFFull;
  x = (x | x << 16) & 0x1F0000FF0000FFull;
  x = (x | x << 8) & 0x100F00F00F00F00Full;
  x = (x | x << 4) & 0x10C30C30C30C30C3ull;
  x = (x | x << 2) & 0x1249249249249249ull;
  return x;
}

// 3. 63-bit Morton code of the normalised centroid
__global__ void k_morton(const float* __restrict__ cen, int n, const uint32_t* __restrict__ bounds,
                         uint64_t* __restrict__ key, uint32_t* __restrict__ idx) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  uint64_t m = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float lo = ord2f(bounds[k]), hi = ord2f(bounds[3 + k]);
    const float ext = hi - lo;
    float u = ext > 0.0f ? (cen[(size_t)i * 3 + k] - lo) / ext : 0.5f;
    u = fminf(fmaxf(u, 0.0f), 1.0f);
    const uint64_t q = (uint64_t)fminf(u * 2097152.0f, 2097151.0f);
    m |= spread21(q) << (2 - k);
  }
  key[i] = m;
  idx[i] = (uint32_t)i;
}

// common prefix length of sorted keys i and j (index breaks ties), -1 outside
__device__ __forceinline__ int delta(const uint64_t* __restrict__ k, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  const uint64_t a = k[i], b = k[j];
  if (a == b) return 64 + __clz((uint32_t)(i ^ j));
  return __clzll((long long)(a ^ b));
}

// 4. internal node i of the radix tree: children (leaf c encoded as n-1+c),
//    covered range [first, last] of sorted primitives, parent links
__global__ void k_karras(const uint64_t* __restrict__ k, int n, int2* __restrict__ child, int2* __restrict__ range,
                         int* __restrict__ parent) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n - 1) return;
  const int d = (delta(k, n, i, i + 1) - delta(k, n, i, i - 1)) >= 0 ? 1 : -1;
  const int dmin = delta(k, n, i, i - d);
  int lmax = 2;
  while (delta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
  int l = 0;
  for (int t = lmax >> 1; t >= 1; t >>= 1)
    if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(k, n, i, j);
  int s = 0;
  for (int div = 2;; div <<= 1) {
    const int t = (l + div - 1) / div;
    if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
    if (t == 1) break;
  }
  const int g = i + s * d + min(d, 0);
  const int lo = min(i, j), hi = max(i, j);
  const int left = (lo == g) ? (n - 1 + g) : g;
  const int right = (hi == g + 1) ? (n - 1 + g + 1) : g + 1;
  child[i] = make_int2(left, right);
  range[i] = make_int2(lo, hi);
  parent[left] = i;
  parent[right] = i;
}

// 5. boxes bottom-up: every leaf walks to the root; the second thread to
//    reach a node unions its children's boxes (agent-scope fences publish the
//    boxes across XCDs before the arrival counter is bumped)
__global__ void k_bottom_up(const Box* __restrict__ pbox, const uint32_t* __restrict__ sorted, int n,
                            const int2* __restrict__ child, const int* __restrict__ parent, Box* nbox,
                            uint32_t* arrivals) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  int node = n - 1 + i;
  nbox[node] = pbox[sorted[i]];
  while (node != 0) {
    __threadfence();
    const int p = parent[node];
    if (atomicAdd(&arrivals[p], 1u) == 0) return;
    __threadfence();
    const int2 c = child[p];
    const Box a = nbox[c.x], b = nbox[c.y];
    Box u;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      u.lo[k] = fminf(a.lo[k], b.lo[k]);
      u.hi[k] = fmaxf(a.hi[k], b.hi[k]);
    }
    nbox[p] = u;
    node = p;
  }
}

// sah: the top-down SAH tree (every node id has a range; a node of more than
// max_leaf primitives always has two children), else leaves are the ids
// n - 1 .. 2n - 2 (radix tree, PLOC)
__device__ __forceinline__ int2 node_range(int v, int n, const int2* __restrict__ range, bool sah = false) {
  return (!sah && v >= n - 1) ? make_int2(v - (n - 1), v - (n - 1)) : range[v];
}

// the wide children (binary node ids) of binary node v; 0 for a wide leaf.
// Greedy collapse: starting from v's two children, the child with the largest
// box surface area that is still an internal node of more than max_leaf
// primitives is replaced by its two children until there are 4 (a Morton tree
// is often unbalanced: the fixed two-level collapse leaves 3-child nodes).
__device__ __forceinline__ float box_area(const Box& b) {
  const float x = b.hi[0] - b.lo[0], y = b.hi[1] - b.lo[1], z = b.hi[2] - b.lo[2];
  return x * y + y * z + z * x;
}
__device__ __forceinline__ int wide_children(int v, int n, int max_leaf, const int2* __restrict__ child,
                                             const int2* __restrict__ range, const Box* __restrict__ nbox,
                                             int (&out)[4], bool sah) {
  const int2 r = node_range(v, n, range, sah);
  if ((!sah && v >= n - 1) || r.y - r.x + 1 <= max_leaf) return 0;
  const int2 c = child[v];
  out[0] = c.x;
  out[1] = c.y;
  int m = 2;
  while (m < 4) {
    int best = -1;
    float ba = -1.0f;
    for (int j = 0; j < m; ++j) {
      const int u = out[j];
      if (!sah && u >= n - 1) continue;
      const int2 ru = range[u];
      if (ru.y - ru.x + 1 <= max_leaf) continue;
      const float a = box_area(nbox[u]);
      if (a > ba) {
        ba = a;
        best = j;
      }
    }
    if (best < 0) break;
    const int2 cu = child[out[best]];
    out[best] = cu.x;
    out[m++] = cu.y;
  }
  return m;
}

// 6a. children per frontier node
__global__ void k_wide_count(const int* __restrict__ front, int m, int n, int max_leaf,
                             const int2* __restrict__ child, const int2* __restrict__ range,
                             const Box* __restrict__ nbox, uint32_t* __restrict__ cnt, bool sah) {
  const int f = blockIdx.x * TPB + threadIdx.x;
  if (f >= m) return;
  int out[4];
  cnt[f] = (uint32_t)wide_children(front[f], n, max_leaf, child, range, nbox, out, sah);
}

// 6b. write the level's pt_node records and the next frontier
__global__ void k_wide_emit(const int* __restrict__ front, int m, int n, int max_leaf, int level, int base,
                            int next_base, const int2* __restrict__ child, const int2* __restrict__ range,
                            const Box* __restrict__ nbox, const uint32_t* __restrict__ off, pt_node* __restrict__ nodes,
                            int* __restrict__ next, bool sah) {
  const int f = blockIdx.x * TPB + threadIdx.x;
  if (f >= m) return;
  const int v = front[f];
  int out[4];
  const int k = wide_children(v, n, max_leaf, child, range, nbox, out, sah);
  pt_node d;
  d.level = level;
  d.ref_id = v;
  const int2 r = node_range(v, n, range, sah);
  d.prim_start = k ? 0 : r.x;
  d.prim_count = k ? 0 : r.y - r.x + 1;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c < k) {
      const Box b = nbox[out[c]];
      d.child[c] = next_base + (int)off[f] + c;
      d.bmin_x[c] = b.lo[0];
      d.bmin_y[c] = b.lo[1];
      d.bmin_z[c] = b.lo[2];
      d.bmax_x[c] = b.hi[0];
      d.bmax_y[c] = b.hi[1];
      d.bmax_z[c] = b.hi[2];
      next[off[f] + c] = out[c];
    } else {
      d.child[c] = -1;
      d.bmin_x[c] = d.bmin_y[c] = d.bmin_z[c] = FLT_MAX;
      d.bmax_x[c] = d.bmax_y[c] = d.bmax_z[c] = -FLT_MAX;
    }
  }
  nodes[base + f] = d;
}

// 7. primitive records in sorted order (bvh_ref.cpp's fp32 operands)
__global__ void k_prim_records(const float* __restrict__ pos, const float* __restrict__ nrm,
                               const int32_t* __restrict__ tri_bsdf, int n_tris, const float* __restrict__ sph,
                               const int32_t* __restrict__ sph_bsdf, const uint32_t* __restrict__ sorted, int n,
                               pt_prim* __restrict__ prims, pt_prim_shading* __restrict__ shading) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const int src = (int)sorted[i];
  pt_prim d;
  pt_prim_shading sh;
  for (int k = 0; k < 24; ++k) d.q[k] = 0.0f;
  for (int k = 0; k < 4; ++k) sh.n0[k] = sh.n1[k] = sh.n2[k] = 0.0f;
  if (src >= n_tris) {
    const int s = src - n_tris;
    const uint32_t meta = (PT_PRIM_SPHERE << 28) | ((uint32_t)(sph_bsdf ? sph_bsdf[s] : 0) & 0x0FFFFFFFu);
    const float* q = sph + (size_t)s * 4;
    d.q[0] = q[0];
    d.q[1] = q[1];
    d.q[2] = q[2];
    d.q[3] = __uint_as_float(meta);
    d.q[4] = q[3];
    d.q[5] = q[3] * q[3];
  } else {
    const uint32_t meta = (PT_PRIM_TRIANGLE << 28) | ((uint32_t)(tri_bsdf ? tri_bsdf[src] : 0) & 0x0FFFFFFFu);
    const float* p = pos + (size_t)src * 9;
    float v[3][3];
    for (int a = 0; a < 3; ++a)
      for (int k = 0; k < 3; ++k) v[a][k] = p[a * 3 + k];
    float e0[3], e1[3], e2[3], v02[3], N[3];
    for (int k = 0; k < 3; ++k) {
      e0[k] = v[1][k] - v[0][k];
      v02[k] = v[2][k] - v[0][k];
      e1[k] = v[2][k] - v[1][k];
      e2[k] = v[0][k] - v[2][k];
    }
    N[0] = e0[1] * v02[2] - e0[2] * v02[1];
    N[1] = e0[2] * v02[0] - e0[0] * v02[2];
    N[2] = e0[0] * v02[1] - e0[1] * v02[0];
    const float dN = N[0] * v[0][0] + N[1] * v[0][1] + N[2] * v[0][2];
    float m[3][3];  // edge normals m_k = N x e_k (pt_api.h)
    const float* ek[3] = {e0, e1, e2};
    for (int k = 0; k < 3; ++k) {
      m[k][0] = N[1] * ek[k][2] - N[2] * ek[k][1];
      m[k][1] = N[2] * ek[k][0] - N[0] * ek[k][2];
      m[k][2] = N[0] * ek[k][1] - N[1] * ek[k][0];
    }
    float* q = d.q;
    q[0] = v[0][0]; q[1] = v[0][1]; q[2] = v[0][2]; q[3] = __uint_as_float(meta);
    q[4] = v[1][0]; q[5] = v[1][1]; q[6] = v[1][2]; q[7] = dN;
    q[8] = v[2][0]; q[9] = v[2][1]; q[10] = v[2][2]; q[11] = m[0][0];
    q[12] = N[0]; q[13] = N[1]; q[14] = N[2]; q[15] = m[0][1];
    q[16] = m[1][0]; q[17] = m[1][1]; q[18] = m[1][2]; q[19] = m[0][2];
    q[20] = m[2][0]; q[21] = m[2][1]; q[22] = m[2][2]; q[23] = 0.f;
    if (nrm) {
      const float* m = nrm + (size_t)src * 9;
      for (int k = 0; k < 3; ++k) {
        sh.n0[k] = m[k];
        sh.n1[k] = m[3 + k];
        sh.n2[k] = m[6 + k];
      }
    } else {
      // face normal, normalised in double like pt_scene_from_mesh
      const double fx = (double)e0[1] * v02[2] - (double)e0[2] * v02[1];
      const double fy = (double)e0[2] * v02[0] - (double)e0[0] * v02[2];
      const double fz = (double)e0[0] * v02[1] - (double)e0[1] * v02[0];
      const double len = sqrt(fx * fx + fy * fy + fz * fz);
      const float nx = len > 0 ? (float)(fx / len) : 0.f, ny = len > 0 ? (float)(fy / len) : 0.f,
                  nz = len > 0 ? (float)(fz / len) : 1.f;
      sh.n0[0] = sh.n1[0] = sh.n2[0] = nx;
      sh.n0[1] = sh.n1[1] = sh.n2[1] = ny;
      sh.n0[2] = sh.n1[2] = sh.n2[2] = nz;
    }
  }
  prims[i] = d;
  shading[i] = sh;
}

// ---- 4'-5'. PLOC: parallel locally-ordered clustering (Meister & Bittner,
// TVCG 2018) instead of the radix tree.  Clusters start as the primitives in
// Morton order; in every iteration each cluster finds its nearest neighbour
// (smallest union box area) among the PLOC_R clusters on either side, mutual
// nearest neighbours merge into a new internal node, and the cluster list is
// compacted (order kept).  Pairs compare by (area, lower position, higher
// position), a strict total order, so the globally closest pair is always
// mutual and every iteration merges at least once.  Internal node ids count
// down from n - 2 in creation order (the root, created last, is 0); leaves
// are n - 1 + Morton position until k_ploc_remap renumbers them to the
// final depth-first primitive order, in which every node covers a contiguous
// range (as the radix tree's nodes do).
// search window radius; visits per ray on the dragon proxy: 2: 5.16, 3: 5.22,
// 4: 4.89, 8: 5.11, 16: 5.21, 32: 5.22 (the radix tree: 6.93, host SAH: 4.36)
constexpr int PLOC_R = 4;

__device__ __forceinline__ float union_area(const Box& a, const Box& b) {
  const float x = fmaxf(a.hi[0], b.hi[0]) - fminf(a.lo[0], b.lo[0]);
  const float y = fmaxf(a.hi[1], b.hi[1]) - fminf(a.lo[1], b.lo[1]);
  const float z = fmaxf(a.hi[2], b.hi[2]) - fminf(a.lo[2], b.lo[2]);
  return x * y + y * z + z * x;
}

__global__ void k_ploc_init(const Box* __restrict__ pbox, const uint32_t* __restrict__ sorted, int n,
                            int* __restrict__ clus, Box* __restrict__ nbox) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  clus[i] = n - 1 + i;
  nbox[n - 1 + i] = pbox[sorted[i]];
}

__global__ void k_ploc_nn(const int* __restrict__ clus, int m, const Box* __restrict__ nbox, int* __restrict__ nn) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= m) return;
  const Box bi = nbox[clus[i]];
  int best = -1;
  float ba = FLT_MAX;
  const int j0 = max(0, i - PLOC_R), j1 = min(m - 1, i + PLOC_R);
  // candidates in increasing position: for equal areas the first one found
  // has the smaller (lower, higher) position pair, so strict < keeps it
  for (int j = j0; j <= j1; ++j) {
    if (j == i) continue;
    const float a = union_area(bi, nbox[clus[j]]);
    if (a < ba || best < 0) {
      ba = a;
      best = j;
    }
  }
  nn[i] = best;
}

__global__ void k_ploc_flags(const int* __restrict__ nn, int m, uint32_t* __restrict__ lead,
                             uint32_t* __restrict__ keep) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= m) return;
  const int j = nn[i];
  const bool mutual = nn[j] == i;
  lead[i] = mutual && i < j;
  keep[i] = !mutual || i < j;
}

__device__ __forceinline__ uint32_t subtree_prims(int v, int n, const uint32_t* __restrict__ cnt) {
  return v >= n - 1 ? 1u : cnt[v];
}

// merges (new node id idbase - rank) and compaction; the last thread writes
// {clusters left, merges}
__global__ void k_ploc_merge(const int* __restrict__ clus, const int* __restrict__ nn, int m, int n,
                             const uint32_t* __restrict__ lead, const uint32_t* __restrict__ lrank,
                             const uint32_t* __restrict__ keep, const uint32_t* __restrict__ kpos, int idbase,
                             int2* __restrict__ child, Box* __restrict__ nbox, uint32_t* __restrict__ cnt,
                             int* __restrict__ clus2, uint32_t* __restrict__ totals) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= m) return;
  if (i == m - 1) {
    totals[0] = kpos[i] + keep[i];
    totals[1] = lrank[i] + lead[i];
  }
  if (!keep[i]) return;
  int c = clus[i];
  if (lead[i]) {
    const int a = c, b = clus[nn[i]];
    const int p = idbase - (int)lrank[i];
    child[p] = make_int2(a, b);
    const Box x = nbox[a], y = nbox[b];
    Box u;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      u.lo[k] = fminf(x.lo[k], y.lo[k]);
      u.hi[k] = fmaxf(x.hi[k], y.hi[k]);
    }
    nbox[p] = u;
    cnt[p] = subtree_prims(a, n, cnt) + subtree_prims(b, n, cnt);
    c = p;
  }
  clus2[kpos[i]] = c;
}

// depth-first primitive offsets, top-down over the nodes of one iteration
// (ids [lo, hi]; their parents were made in later iterations)
__global__ void k_ploc_offsets(int lo, int hi, int n, const int2* __restrict__ child,
                               const uint32_t* __restrict__ cnt, uint32_t* __restrict__ start,
                               int2* __restrict__ range, uint32_t* __restrict__ pos) {
  const int p = lo + blockIdx.x * TPB + threadIdx.x;
  if (p > hi) return;
  const uint32_t s = start[p];
  range[p] = make_int2((int)s, (int)(s + cnt[p] - 1));
  const int2 c = child[p];
  const uint32_t ca = subtree_prims(c.x, n, cnt);
  if (c.x >= n - 1) pos[c.x - (n - 1)] = s;
  else start[c.x] = s;
  if (c.y >= n - 1) pos[c.y - (n - 1)] = s + ca;
  else start[c.y] = s + ca;
}

// leaves renumbered to their depth-first position: child links, leaf boxes
// (into nbox2) and the final primitive order
__global__ void k_ploc_remap(int n, int2* __restrict__ child, const uint32_t* __restrict__ pos,
                             const Box* __restrict__ nbox, Box* __restrict__ nbox2,
                             const uint32_t* __restrict__ sorted, uint32_t* __restrict__ sorted2) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i < n - 1) {
    int2 c = child[i];
    if (c.x >= n - 1) c.x = n - 1 + (int)pos[c.x - (n - 1)];
    if (c.y >= n - 1) c.y = n - 1 + (int)pos[c.y - (n - 1)];
    child[i] = c;
  }
  if (i < n) {
    nbox2[n - 1 + pos[i]] = nbox[n - 1 + i];
    sorted2[pos[i]] = sorted[i];
  }
}

// ---- 4''-5''. top-down binned SAH (the reference's split rule, bvh.cpp:48-230,
// level-synchronous on the device).  A node of more than max_leaf primitives
// is split by one of 12 planes per axis, evenly spaced over its centroids'
// extent (plane p at lo + p (hi - lo) / 13), minimising the reference's cost
// 5 + 2 (SA_l / SA) n_l + 2 (SA_r / SA) n_r; a node whose planes all cost at
// least a leaf's 2 n (coincident centroids) is split at the middle of its
// range instead (the reference keeps it as a larger leaf).  Per level: the
// centroid extents of the nodes being split (k_sah_cbounds), their 13 bins per
// axis (count and box: k_sah_bin), the best plane and the two children
// (k_sah_split), then a stable partition of each node's primitive range
// (k_sah_flags, a scan, k_sah_scatter).  Node ids count up in creation order
// (the root is 0); every node has a range of the sorted primitives, and the
// 4-wide collapse reads the tree in its `sah` mode.
constexpr int SAH_BINS = 13;  // 12 planes
constexpr int SAH_CNT = 2 * 3 * SAH_BINS;  // bin records per node: counts (u32) and boxes (6 ordered u32)

struct SahSplit {  // per node being split
  int axis;        // -1: split at the middle of the range
  int plane;       // 1..12: the left child holds bins 0 .. plane - 1
  int nl;          // primitives of the left child
  int pad;
  Box bl, br;
};

// the slot (index into the level's list of nodes being split, sorted by range
// start) whose range holds position i, or -1
__device__ __forceinline__ int sah_slot(const int2* __restrict__ srange, int m, int i) {
  int lo = 0, hi = m - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (srange[mid].x <= i) lo = mid;
    else hi = mid - 1;
  }
  return (m > 0 && srange[lo].x <= i && i <= srange[lo].y) ? lo : -1;
}

// (the accumulating kernels below reduce in LDS when all of a workgroup's
// positions lie in one node's range -- every workgroup of the top levels,
// where one node's bins would otherwise take ~10^5 same-address atomics --
// and flush once; mixed workgroups use global atomics)
__device__ __forceinline__ int block_uniform_slot(int s) {
  __shared__ int lo, hi;
  if (threadIdx.x == 0) {
    lo = INT_MAX;
    hi = INT_MIN;
  }
  __syncthreads();
  atomicMin(&lo, s);
  atomicMax(&hi, s);
  __syncthreads();
  return lo == hi ? lo : -2;  // (-1: no slot in the whole workgroup)
}

__global__ void k_sah_cbounds(const uint32_t* __restrict__ P, int n, const float* __restrict__ cen,
                              const int2* __restrict__ srange, int m, uint32_t* __restrict__ cb) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  const int s = i < n ? sah_slot(srange, m, i) : -1;
  const int u = block_uniform_slot(i < n ? s : (blockIdx.x * TPB < n ? sah_slot(srange, m, blockIdx.x * TPB) : -1));
  __shared__ uint32_t L[6];
  if (u >= 0 && threadIdx.x < 6) L[threadIdx.x] = threadIdx.x < 3 ? 0xFFFFFFFFu : 0u;
  __syncthreads();
  if (s >= 0) {
    const uint32_t pr = P[i];
    uint32_t* const dst = u >= 0 ? L : cb + s * 6;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint32_t o = f2ord(cen[(size_t)pr * 3 + k]);
      atomicMin(&dst[k], o);
      atomicMax(&dst[3 + k], o);
    }
  }
  if (u >= 0) {
    __syncthreads();
    if (threadIdx.x < 3) atomicMin(&cb[u * 6 + threadIdx.x], L[threadIdx.x]);
    else if (threadIdx.x < 6) atomicMax(&cb[u * 6 + threadIdx.x], L[threadIdx.x]);
  }
}

// bin of centroid c among the 12 planes of [lo, hi]: the number of planes
// strictly below c (0 .. 12); a primitive is left of plane p iff its bin < p
__device__ __forceinline__ int sah_bin(float c, float lo, float hi) {
  const float step = (hi - lo) / 13.0f;
  int b = 0;
#pragma unroll
  for (int p = 1; p <= 12; ++p) b += (fmaf((float)p, step, lo) < c) ? 1 : 0;
  return b;
}

__global__ void k_sah_bin(const uint32_t* __restrict__ P, int n, const float* __restrict__ cen,
                          const Box* __restrict__ pbox, const int2* __restrict__ srange, int m,
                          const uint32_t* __restrict__ cb, uint32_t* __restrict__ bins) {
  constexpr int NB = SAH_CNT * 4;  // u32 per node: [axis][bin]: count, then lo[3], hi[3] (ordered), pad
  const int i = blockIdx.x * TPB + threadIdx.x;
  const int s = i < n ? sah_slot(srange, m, i) : -1;
  const int u = block_uniform_slot(i < n ? s : (blockIdx.x * TPB < n ? sah_slot(srange, m, blockIdx.x * TPB) : -1));
  __shared__ uint32_t L[NB];
  if (u >= 0)
    for (int t = threadIdx.x; t < NB; t += TPB) {
      const int f = t & 7;
      L[t] = (f >= 1 && f <= 3) ? 0xFFFFFFFFu : 0u;
    }
  __syncthreads();
  if (s >= 0) {
    const uint32_t pr = P[i];
    const Box b = pbox[pr];
    uint32_t* const B = u >= 0 ? L : bins + (size_t)s * NB;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int j = sah_bin(cen[(size_t)pr * 3 + k], ord2f(cb[s * 6 + k]), ord2f(cb[s * 6 + 3 + k]));
      uint32_t* const r = B + (k * SAH_BINS + j) * 8;
      atomicAdd(&r[0], 1u);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        atomicMin(&r[1 + a], f2ord(b.lo[a]));
        atomicMax(&r[4 + a], f2ord(b.hi[a]));
      }
    }
  }
  if (u >= 0) {
    __syncthreads();
    uint32_t* const G = bins + (size_t)u * NB;
    for (int t = threadIdx.x; t < NB; t += TPB) {
      const int f = t & 7;
      if (f == 0) {
        if (L[t]) atomicAdd(&G[t], L[t]);
      } else if (f <= 3) {
        if (L[t] != 0xFFFFFFFFu) atomicMin(&G[t], L[t]);
      } else if (f <= 6) {
        if (L[t]) atomicMax(&G[t], L[t]);
      }
    }
  }
}

__device__ __forceinline__ float box_sa(const Box& b) {
  const float x = b.hi[0] - b.lo[0], y = b.hi[1] - b.lo[1], z = b.hi[2] - b.lo[2];
  return 2.0f * (x * y + y * z + z * x);
}
__device__ __forceinline__ void box_grow(Box& a, const uint32_t* r) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    a.lo[k] = fminf(a.lo[k], ord2f(r[1 + k]));
    a.hi[k] = fmaxf(a.hi[k], ord2f(r[4 + k]));
  }
}

// one thread per node being split: the best plane (axes in order, strict <:
// the first minimum, as the reference's loops), the children's boxes
__global__ void k_sah_split(const int* __restrict__ snode, int m, const int2* __restrict__ srange,
                            const Box* __restrict__ nbox, const uint32_t* __restrict__ bins,
                            SahSplit* __restrict__ out) {
  const int s = blockIdx.x * TPB + threadIdx.x;
  if (s >= m) return;
  const int2 r = srange[s];
  const int cnt = r.y - r.x + 1;
  const double total_sa = (double)box_sa(nbox[snode[s]]);
  const uint32_t* const B = bins + (size_t)s * SAH_CNT * 4;
  const float leaf_cost = 2.0f * (float)cnt;
  double best = leaf_cost;
  SahSplit o;
  o.axis = -1;
  o.plane = 0;
  o.nl = cnt / 2;
  o.pad = 0;
  for (int k = 0; k < 3; ++k) {
    Box L[SAH_BINS], R;
    uint32_t nL[SAH_BINS];
    Box acc;
    uint32_t c = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      acc.lo[a] = FLT_MAX;
      acc.hi[a] = -FLT_MAX;
    }
    for (int j = 0; j < SAH_BINS; ++j) {  // L[j]: bins 0 .. j - 1 (left of plane j)
      L[j] = acc;
      nL[j] = c;
      const uint32_t* rr = B + (k * SAH_BINS + j) * 8;
      if (rr[0]) {
        box_grow(acc, rr);
        c += rr[0];
      }
    }
    R.lo[0] = R.lo[1] = R.lo[2] = FLT_MAX;
    R.hi[0] = R.hi[1] = R.hi[2] = -FLT_MAX;
    Box Rp[SAH_BINS];
    for (int j = SAH_BINS - 1; j >= 1; --j) {  // Rp[j]: bins j .. 12 (right of plane j)
      const uint32_t* rr = B + (k * SAH_BINS + j) * 8;
      if (rr[0]) box_grow(R, rr);
      Rp[j] = R;
    }
    for (int p = 1; p < SAH_BINS; ++p) {
      const int nl = (int)nL[p], nr = cnt - nl;
      if (nl == 0 || nr == 0) continue;
      const double cost = 5.0 + ((double)box_sa(L[p]) / total_sa) * nl * 2 + ((double)box_sa(Rp[p]) / total_sa) * nr * 2;
      if (cost < best) {
        best = cost;
        o.axis = k;
        o.plane = p;
        o.nl = nl;
        o.bl = L[p];
        o.br = Rp[p];
      }
    }
  }
  out[s] = o;
}

// children of the split nodes: ids base + 2 s, base + 2 s + 1; a child of
// more than max_leaf primitives is split at the next level (flag)
__global__ void k_sah_children(const int* __restrict__ snode, int m, const int2* __restrict__ srange,
                                  const SahSplit* __restrict__ sp, int base, int max_leaf, int2* __restrict__ child,
                               int2* __restrict__ range, uint32_t* __restrict__ more) {
  const int s = blockIdx.x * TPB + threadIdx.x;
  if (s >= m) return;
  const int2 r = srange[s];
  const SahSplit o = sp[s];
  const int l = base + 2 * s, rr = l + 1;
  child[snode[s]] = make_int2(l, rr);
  range[l] = make_int2(r.x, r.x + o.nl - 1);
  range[rr] = make_int2(r.x + o.nl, r.y);
  child[l] = child[rr] = make_int2(-1, -1);
  more[2 * s] = o.nl > max_leaf ? 1u : 0u;
  more[2 * s + 1] = (r.y - r.x + 1 - o.nl) > max_leaf ? 1u : 0u;
}

// left flags of the positions in split ranges (0 elsewhere)
__global__ void k_sah_flags(const uint32_t* __restrict__ P, int n, const float* __restrict__ cen,
                            const int2* __restrict__ srange, int m, const uint32_t* __restrict__ cb,
                            const SahSplit* __restrict__ sp, uint32_t* __restrict__ left) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const int s = sah_slot(srange, m, i);
  uint32_t f = 0;
  if (s >= 0) {
    const SahSplit o = sp[s];
    if (o.axis < 0) {
      f = (i - srange[s].x) < o.nl ? 1u : 0u;
    } else {
      const int k = o.axis;
      f = sah_bin(cen[(size_t)P[i] * 3 + k], ord2f(cb[s * 6 + k]), ord2f(cb[s * 6 + 3 + k])) < o.plane ? 1u : 0u;
    }
  }
  left[i] = f;
}

// stable partition of each split range (left primitives first, in order)
__global__ void k_sah_scatter(const uint32_t* __restrict__ P, int n, const int2* __restrict__ srange, int m,
                              const SahSplit* __restrict__ sp, const uint32_t* __restrict__ left,
                              const uint32_t* __restrict__ lscan, uint32_t* __restrict__ P2) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const int s = sah_slot(srange, m, i);
  if (s < 0) {
    P2[i] = P[i];
    return;
  }
  const int first = srange[s].x;
  const uint32_t lr = lscan[i] - lscan[first];  // left primitives before i in the range
  const int pos = left[i] ? first + (int)lr : first + sp[s].nl + (i - first - (int)lr);
  P2[pos] = P[i];
}

// the children's boxes as the unions of their primitives' boxes, after the
// partition (the middle split of coincident centroids has no bins to take
// them from): ordered-u32 atomics into cbu[6 per child], then k_sah_child_box
__global__ void k_sah_child_acc(const uint32_t* __restrict__ P, int n, const Box* __restrict__ pbox,
                                const int2* __restrict__ srange, int m, const SahSplit* __restrict__ sp,
                                uint32_t* __restrict__ cbu) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  const int s = i < n ? sah_slot(srange, m, i) : -1;
  const int c = s >= 0 ? 2 * s + ((i - srange[s].x) < sp[s].nl ? 0 : 1) : -1;
  // (uniform child: the workgroup's positions in one child's range)
  const int u = block_uniform_slot(i < n ? c : (blockIdx.x * TPB < n ? c : -1));
  __shared__ uint32_t L[6];
  if (u >= 0 && threadIdx.x < 6) L[threadIdx.x] = threadIdx.x < 3 ? 0xFFFFFFFFu : 0u;
  __syncthreads();
  if (c >= 0) {
    const Box b = pbox[P[i]];
    uint32_t* const dst = u >= 0 ? L : cbu + c * 6;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      atomicMin(&dst[k], f2ord(b.lo[k]));
      atomicMax(&dst[3 + k], f2ord(b.hi[k]));
    }
  }
  if (u >= 0) {
    __syncthreads();
    if (threadIdx.x < 3) atomicMin(&cbu[u * 6 + threadIdx.x], L[threadIdx.x]);
    else if (threadIdx.x < 6) atomicMax(&cbu[u * 6 + threadIdx.x], L[threadIdx.x]);
  }
}
__global__ void k_sah_child_box(int m2, int base, const uint32_t* __restrict__ cbu, Box* __restrict__ nbox) {
  const int c = blockIdx.x * TPB + threadIdx.x;
  if (c >= m2) return;
  Box b;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    b.lo[k] = ord2f(cbu[c * 6 + k]);
    b.hi[k] = ord2f(cbu[c * 6 + 3 + k]);
  }
  nbox[base + c] = b;
}
__global__ void k_sah_init_cbu(int m2, uint32_t* __restrict__ cbu) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i < m2 * 6) cbu[i] = (i % 6) < 3 ? 0xFFFFFFFFu : 0u;
}

// the root's box: the union of the primitive boxes
__global__ void k_root_box(const Box* __restrict__ pbox, int n, uint32_t* __restrict__ rb) {
  __shared__ uint32_t s[6];
  if (threadIdx.x < 3) s[threadIdx.x] = 0xFFFFFFFFu;
  else if (threadIdx.x < 6) s[threadIdx.x] = 0u;
  __syncthreads();
  for (int i = blockIdx.x * TPB + threadIdx.x; i < n; i += gridDim.x * TPB) {
    const Box b = pbox[i];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      atomicMin(&s[k], f2ord(b.lo[k]));
      atomicMax(&s[3 + k], f2ord(b.hi[k]));
    }
  }
  __syncthreads();
  if (threadIdx.x < 3) atomicMin(&rb[threadIdx.x], s[threadIdx.x]);
  else if (threadIdx.x < 6) atomicMax(&rb[threadIdx.x], s[threadIdx.x]);
}
__global__ void k_root_init(const uint32_t* __restrict__ rb, int n, Box* __restrict__ nbox, int2* __restrict__ range,
                            int2* __restrict__ child) {
  Box b;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    b.lo[k] = ord2f(rb[k]);
    b.hi[k] = ord2f(rb[3 + k]);
  }
  nbox[0] = b;
  range[0] = make_int2(0, n - 1);
  child[0] = make_int2(-1, -1);
}
__global__ void k_sah_init_bins(int m, uint32_t* __restrict__ cb, uint32_t* __restrict__ bins) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i < m * 6) cb[i] = (i % 6) < 3 ? 0xFFFFFFFFu : 0u;
  if (i < m * SAH_CNT * 4) {
    const int f = i & 7;  // count, lo[3] (min: init high), hi[3] (max: init low), pad
    bins[i] = (f >= 1 && f <= 3) ? 0xFFFFFFFFu : 0u;
  }
}
// the next level's split list: compacted children with more than max_leaf
// primitives (their ids base + t and ranges), kept in range order
__global__ void k_sah_next(int m2, int base, const uint32_t* __restrict__ more, const uint32_t* __restrict__ mscan,
                           const int2* __restrict__ range, int* __restrict__ snode2, int2* __restrict__ srange2) {
  const int t = blockIdx.x * TPB + threadIdx.x;
  if (t >= m2) return;
  if (more[t]) {
    snode2[mscan[t]] = base + t;
    srange2[mscan[t]] = range[base + t];
  }
}

struct DevBuf {
  std::vector<void*> ptrs;
  ~DevBuf() {
    for (void* p : ptrs) hipFree(p);
  }
  template <class T>
  T* alloc(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    return (T*)p;
  }
};

}  // namespace ptb

using namespace ptb;

#define BCHK(x)                         \
  do {                                  \
    if ((x) != hipSuccess) return PT_E_HIP; \
  } while (0)

static int build_on_device(const pt_mesh_desc* md, int max_leaf, int builder, ptscene::Scene& S, hipStream_t st) {
  const int n_tris = md->n_tris, n = md->n_tris + md->n_spheres;
  DevBuf B;
  float* d_pos = B.alloc<float>((size_t)n_tris * 9);
  float* d_nrm = md->normals ? B.alloc<float>((size_t)n_tris * 9) : nullptr;
  int32_t* d_tb = md->tri_bsdf ? B.alloc<int32_t>(n_tris) : nullptr;
  float* d_sph = B.alloc<float>((size_t)md->n_spheres * 4);
  int32_t* d_sb = md->sphere_bsdf ? B.alloc<int32_t>(md->n_spheres) : nullptr;
  Box* d_pbox = B.alloc<Box>(n);
  float* d_cen = B.alloc<float>((size_t)n * 3);
  uint32_t* d_bounds = B.alloc<uint32_t>(6);
  uint64_t *d_key = B.alloc<uint64_t>(n), *d_key2 = B.alloc<uint64_t>(n);
  uint32_t *d_idx = B.alloc<uint32_t>(n), *d_idx2 = B.alloc<uint32_t>(n);
  int2* d_child = B.alloc<int2>(n);
  int2* d_range = B.alloc<int2>(n);
  int* d_parent = B.alloc<int>(2 * (size_t)n);
  Box* d_nbox = B.alloc<Box>(2 * (size_t)n);
  uint32_t* d_arr = B.alloc<uint32_t>(n);
  pt_node* d_nodes = B.alloc<pt_node>(2 * (size_t)n);
  int *d_front = B.alloc<int>(2 * (size_t)n), *d_next = B.alloc<int>(2 * (size_t)n);
  uint32_t *d_cnt = B.alloc<uint32_t>(2 * (size_t)n), *d_off = B.alloc<uint32_t>(2 * (size_t)n + 1);
  pt_prim* d_prims = B.alloc<pt_prim>(n);
  pt_prim_shading* d_shading = B.alloc<pt_prim_shading>(n);
  for (void* p : B.ptrs)
    if (!p) return PT_E_HIP;
  if (n_tris) BCHK(hipMemcpyAsync(d_pos, md->positions, (size_t)n_tris * 36, hipMemcpyHostToDevice, st));
  if (d_nrm) BCHK(hipMemcpyAsync(d_nrm, md->normals, (size_t)n_tris * 36, hipMemcpyHostToDevice, st));
  if (d_tb) BCHK(hipMemcpyAsync(d_tb, md->tri_bsdf, (size_t)n_tris * 4, hipMemcpyHostToDevice, st));
  if (md->n_spheres) BCHK(hipMemcpyAsync(d_sph, md->spheres, (size_t)md->n_spheres * 16, hipMemcpyHostToDevice, st));
  if (d_sb) BCHK(hipMemcpyAsync(d_sb, md->sphere_bsdf, (size_t)md->n_spheres * 4, hipMemcpyHostToDevice, st));
  const uint32_t binit[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
  BCHK(hipMemcpyAsync(d_bounds, binit, sizeof(binit), hipMemcpyHostToDevice, st));
  BCHK(hipMemsetAsync(d_arr, 0, (size_t)n * 4, st));
  const dim3 g((n + TPB - 1) / TPB);
  hipLaunchKernelGGL(k_prim_bounds, g, dim3(TPB), 0, st, d_pos, n_tris, d_sph, n, ptscene::box_guard(S), d_pbox,
                     d_cen);
  hipLaunchKernelGGL(k_reduce_bounds, dim3(std::min(1024, (n + TPB - 1) / TPB)), dim3(TPB), 0, st, d_cen, n,
                     d_bounds);
  // binary tree: top-down SAH, PLOC or the radix tree (the last two over
  // the primitives in Morton order)
  const bool sah = builder == PT_GPU_BVH_SAH;
  if (!sah) {
    hipLaunchKernelGGL(k_morton, g, dim3(TPB), 0, st, d_cen, n, d_bounds, d_key, d_idx);
    size_t tmp_bytes = 0;
    BCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, d_key, d_key2, d_idx, d_idx2, n, 0, 63, st));
    void* d_tmp = B.alloc<uint8_t>(tmp_bytes);
    if (!d_tmp) return PT_E_HIP;
    BCHK(hipcub::DeviceRadixSort::SortPairs(d_tmp, tmp_bytes, d_key, d_key2, d_idx, d_idx2, n, 0, 63, st));
  }
  const bool ploc = n > 1 && builder == PT_GPU_BVH_PLOC;
  uint32_t* d_sorted = d_idx2;  // final primitive order
  if (sah) {
    // ids count up from the root (0): at most 2 n - 1 nodes, each with a range
    int2* d_child2 = B.alloc<int2>(2 * (size_t)n);
    int2* d_range2 = B.alloc<int2>(2 * (size_t)n);
    const int smax = n / (max_leaf + 1) + 1;  // nodes split in one level (disjoint ranges of > max_leaf)
    uint32_t *d_P = B.alloc<uint32_t>(n), *d_P2 = B.alloc<uint32_t>(n), *d_left = B.alloc<uint32_t>(n + 1),
             *d_lscan = B.alloc<uint32_t>(n + 1), *d_more = B.alloc<uint32_t>(2 * (size_t)smax + 1),
             *d_mscan = B.alloc<uint32_t>(2 * (size_t)smax + 1), *d_cb = B.alloc<uint32_t>(6 * (size_t)smax),
             *d_bins = B.alloc<uint32_t>((size_t)smax * SAH_CNT * 4), *d_rb = B.alloc<uint32_t>(6),
             *d_cbu = B.alloc<uint32_t>(12 * (size_t)smax);
    int *d_snode = B.alloc<int>(smax), *d_snode2 = B.alloc<int>(smax);
    int2 *d_srange = B.alloc<int2>(smax), *d_srange2 = B.alloc<int2>(smax);
    SahSplit* d_sp = B.alloc<SahSplit>(smax);
    size_t sb = 0;
    BCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, sb, d_left, d_lscan, n + 1, st));
    void* d_sscan = B.alloc<uint8_t>(sb);
    if (!d_child2 || !d_range2 || !d_P || !d_P2 || !d_left || !d_lscan || !d_more || !d_mscan || !d_cb || !d_bins ||
        !d_rb || !d_cbu || !d_snode || !d_snode2 || !d_srange || !d_srange2 || !d_sp || !d_sscan)
      return PT_E_HIP;
    d_child = d_child2;
    d_range = d_range2;
    std::vector<uint32_t> iota(n);
    for (int i = 0; i < n; ++i) iota[i] = (uint32_t)i;
    BCHK(hipMemcpyAsync(d_P, iota.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    BCHK(hipMemcpyAsync(d_rb, binit, sizeof(binit), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_root_box, dim3(std::min(1024, (n + TPB - 1) / TPB)), dim3(TPB), 0, st, d_pbox, n, d_rb);
    hipLaunchKernelGGL(k_root_init, dim3(1), dim3(1), 0, st, d_rb, n, d_nbox, d_range, d_child);
    int m = n > max_leaf ? 1 : 0, next_id = 1;
    if (m) {
      const int zero = 0;
      const int2 r0 = make_int2(0, n - 1);
      BCHK(hipMemcpyAsync(d_snode, &zero, 4, hipMemcpyHostToDevice, st));
      BCHK(hipMemcpyAsync(d_srange, &r0, sizeof(r0), hipMemcpyHostToDevice, st));
    }
    for (int level = 0; m > 0; ++level) {
      if (level > 4 * 64 || m > smax) return PT_E_INVALID;
      const dim3 gm((m + TPB - 1) / TPB), gb(((size_t)m * SAH_CNT * 4 + TPB - 1) / TPB);
      hipLaunchKernelGGL(k_sah_init_bins, gb, dim3(TPB), 0, st, m, d_cb, d_bins);
      hipLaunchKernelGGL(k_sah_cbounds, g, dim3(TPB), 0, st, d_P, n, d_cen, d_srange, m, d_cb);
      hipLaunchKernelGGL(k_sah_bin, g, dim3(TPB), 0, st, d_P, n, d_cen, d_pbox, d_srange, m, d_cb, d_bins);
      hipLaunchKernelGGL(k_sah_split, gm, dim3(TPB), 0, st, d_snode, m, d_srange, d_nbox, d_bins, d_sp);
      hipLaunchKernelGGL(k_sah_children, gm, dim3(TPB), 0, st, d_snode, m, d_srange, d_sp, next_id, max_leaf, d_child,
                         d_range, d_more);
      hipLaunchKernelGGL(k_sah_flags, g, dim3(TPB), 0, st, d_P, n, d_cen, d_srange, m, d_cb, d_sp, d_left);
      BCHK(hipcub::DeviceScan::ExclusiveSum(d_sscan, sb, d_left, d_lscan, n, st));
      hipLaunchKernelGGL(k_sah_scatter, g, dim3(TPB), 0, st, d_P, n, d_srange, m, d_sp, d_left, d_lscan, d_P2);
      std::swap(d_P, d_P2);
      const int m2 = 2 * m;
      hipLaunchKernelGGL(k_sah_init_cbu, dim3((m2 * 6 + TPB - 1) / TPB), dim3(TPB), 0, st, m2, d_cbu);
      hipLaunchKernelGGL(k_sah_child_acc, g, dim3(TPB), 0, st, d_P, n, d_pbox, d_srange, m, d_sp, d_cbu);
      hipLaunchKernelGGL(k_sah_child_box, dim3((m2 + TPB - 1) / TPB), dim3(TPB), 0, st, m2, next_id, d_cbu, d_nbox);
      BCHK(hipMemsetAsync(d_more + m2, 0, 4, st));
      BCHK(hipcub::DeviceScan::ExclusiveSum(d_sscan, sb, d_more, d_mscan, m2 + 1, st));
      uint32_t next_m = 0;
      BCHK(hipMemcpyAsync(&next_m, d_mscan + m2, 4, hipMemcpyDeviceToHost, st));
      hipLaunchKernelGGL(k_sah_next, dim3((m2 + TPB - 1) / TPB), dim3(TPB), 0, st, m2, next_id, d_more, d_mscan,
                         d_range, d_snode2, d_srange2);
      BCHK(hipStreamSynchronize(st));
      BCHK(hipGetLastError());
      next_id += m2;
      m = (int)next_m;
      std::swap(d_snode, d_snode2);
      std::swap(d_srange, d_srange2);
    }
    d_sorted = d_P;
  } else if (ploc) {
    int *d_clus = B.alloc<int>(n), *d_clus2 = B.alloc<int>(n), *d_nn = B.alloc<int>(n);
    uint32_t *d_lead = B.alloc<uint32_t>(n), *d_lrank = B.alloc<uint32_t>(n), *d_keep = B.alloc<uint32_t>(n),
             *d_kpos = B.alloc<uint32_t>(n), *d_pcnt = B.alloc<uint32_t>(n), *d_start = B.alloc<uint32_t>(n),
             *d_ppos = B.alloc<uint32_t>(n), *d_sorted2 = B.alloc<uint32_t>(n), *d_tot = B.alloc<uint32_t>(2);
    Box* d_nbox2 = B.alloc<Box>(2 * (size_t)n);
    size_t sb = 0;
    BCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, sb, d_lead, d_lrank, n, st));
    void* d_pscan = B.alloc<uint8_t>(sb);
    if (!d_clus || !d_clus2 || !d_nn || !d_lead || !d_lrank || !d_keep || !d_kpos || !d_pcnt || !d_start ||
        !d_ppos || !d_sorted2 || !d_tot || !d_nbox2 || !d_pscan)
      return PT_E_HIP;
    hipLaunchKernelGGL(k_ploc_init, g, dim3(TPB), 0, st, d_pbox, d_idx2, n, d_clus, d_nbox);
    std::vector<std::pair<int, int>> made_ranges;  // internal ids made per iteration
    int m = n, made = 0;
    while (m > 1) {
      const dim3 gm((m + TPB - 1) / TPB);
      hipLaunchKernelGGL(k_ploc_nn, gm, dim3(TPB), 0, st, d_clus, m, d_nbox, d_nn);
      hipLaunchKernelGGL(k_ploc_flags, gm, dim3(TPB), 0, st, d_nn, m, d_lead, d_keep);
      BCHK(hipcub::DeviceScan::ExclusiveSum(d_pscan, sb, d_lead, d_lrank, m, st));
      BCHK(hipcub::DeviceScan::ExclusiveSum(d_pscan, sb, d_keep, d_kpos, m, st));
      const int idbase = n - 2 - made;
      hipLaunchKernelGGL(k_ploc_merge, gm, dim3(TPB), 0, st, d_clus, d_nn, m, n, d_lead, d_lrank, d_keep, d_kpos,
                         idbase, d_child, d_nbox, d_pcnt, d_clus2, d_tot);
      uint32_t tot[2] = {0, 0};
      BCHK(hipMemcpyAsync(tot, d_tot, 8, hipMemcpyDeviceToHost, st));
      BCHK(hipStreamSynchronize(st));
      BCHK(hipGetLastError());
      if (tot[1] == 0 || (int)tot[0] >= m) return PT_E_INVALID;  // cannot happen (see above)
      made_ranges.push_back({idbase - (int)tot[1] + 1, idbase});
      made += (int)tot[1];
      m = (int)tot[0];
      std::swap(d_clus, d_clus2);
    }
    if (made != n - 1) return PT_E_INVALID;
    BCHK(hipMemsetAsync(d_start, 0, 4, st));  // root 0 starts at 0
    for (size_t t = made_ranges.size(); t-- > 0;) {
      const int lo = made_ranges[t].first, hi = made_ranges[t].second;
      hipLaunchKernelGGL(k_ploc_offsets, dim3((hi - lo + 1 + TPB - 1) / TPB), dim3(TPB), 0, st, lo, hi, n, d_child,
                         d_pcnt, d_start, d_range, d_ppos);
    }
    hipLaunchKernelGGL(k_ploc_remap, g, dim3(TPB), 0, st, n, d_child, d_ppos, d_nbox, d_nbox2, d_idx2, d_sorted2);
    BCHK(hipMemcpyAsync(d_nbox + (n - 1), d_nbox2 + (n - 1), (size_t)n * sizeof(Box), hipMemcpyDeviceToDevice, st));
    d_sorted = d_sorted2;
  } else {
    if (n > 1)
      hipLaunchKernelGGL(k_karras, dim3((n - 1 + TPB - 1) / TPB), dim3(TPB), 0, st, d_key2, n, d_child, d_range,
                         d_parent);
    hipLaunchKernelGGL(k_bottom_up, g, dim3(TPB), 0, st, d_pbox, d_idx2, n, d_child, d_parent, d_nbox, d_arr);
  }
  hipLaunchKernelGGL(k_prim_records, g, dim3(TPB), 0, st, d_pos, d_nrm, d_tb, n_tris, d_sph, d_sb, d_sorted, n,
                     d_prims, d_shading);
  BCHK(hipGetLastError());

  // 6. level-synchronous 4-wide collapse
  const int root = (n > 1 || sah) ? 0 : n - 1;  // a single primitive: the root is leaf 0
  BCHK(hipMemcpyAsync(d_front, &root, 4, hipMemcpyHostToDevice, st));
  size_t scan_bytes = 0;
  BCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, d_cnt, d_off, 2 * n + 1, st));
  void* d_scan = B.alloc<uint8_t>(scan_bytes);
  if (!d_scan) return PT_E_HIP;
  std::vector<int32_t> level_start = {0};
  int m = 1, base = 0;
  for (int level = 0; m > 0; ++level) {
    if (level > 1000) return PT_E_INVALID;
    const dim3 gm((m + TPB - 1) / TPB);
    BCHK(hipMemsetAsync(d_cnt + m, 0, 4, st));
    hipLaunchKernelGGL(k_wide_count, gm, dim3(TPB), 0, st, d_front, m, n, max_leaf, d_child, d_range, d_nbox,
                       d_cnt, sah);
    BCHK(hipcub::DeviceScan::ExclusiveSum(d_scan, scan_bytes, d_cnt, d_off, m + 1, st));
    uint32_t next_m = 0;
    BCHK(hipMemcpyAsync(&next_m, d_off + m, 4, hipMemcpyDeviceToHost, st));
    hipLaunchKernelGGL(k_wide_emit, gm, dim3(TPB), 0, st, d_front, m, n, max_leaf, level, base, base + m, d_child,
                       d_range, d_nbox, d_off, d_nodes, d_next, sah);
    BCHK(hipStreamSynchronize(st));
    BCHK(hipGetLastError());
    base += m;
    level_start.push_back(base);
    m = (int)next_m;
    std::swap(d_front, d_next);
  }

  // results to the host scene
  std::vector<uint32_t> sorted(n);
  S.dprims.resize(n);
  S.dshading.resize(n);
  S.dnodes.resize(base);
  BCHK(hipMemcpyAsync(sorted.data(), d_sorted, (size_t)n * 4, hipMemcpyDeviceToHost, st));
  BCHK(hipMemcpyAsync(S.dprims.data(), d_prims, (size_t)n * sizeof(pt_prim), hipMemcpyDeviceToHost, st));
  BCHK(hipMemcpyAsync(S.dshading.data(), d_shading, (size_t)n * sizeof(pt_prim_shading), hipMemcpyDeviceToHost,
                      st));
  BCHK(hipMemcpyAsync(S.dnodes.data(), d_nodes, (size_t)base * sizeof(pt_node), hipMemcpyDeviceToHost, st));
  BCHK(hipStreamSynchronize(st));
  S.sorted_to_input.assign(sorted.begin(), sorted.end());
  S.level_start = level_start;
  S.level_counts.clear();
  for (size_t l = 0; l + 1 < level_start.size(); ++l) S.level_counts.push_back(level_start[l + 1] - level_start[l]);
  return PT_OK;
}

extern "C" int pt_scene_build_gpu(const pt_mesh_desc* mesh, int32_t device, int32_t max_leaf, pt_scene** out,
                                  double* build_ms) {
  return pt_scene_build_gpu_ex(mesh, device, max_leaf, PT_GPU_BVH_SAH, out, build_ms);
}

extern "C" int pt_scene_build_gpu_ex(const pt_mesh_desc* mesh, int32_t device, int32_t max_leaf, int32_t builder,
                                     pt_scene** out, double* build_ms) {
  if (!out) return PT_E_INVALID;
  *out = nullptr;
  if (max_leaf < 1 || max_leaf > 64) return PT_E_INVALID;
  if (builder != PT_GPU_BVH_PLOC && builder != PT_GPU_BVH_LBVH && builder != PT_GPU_BVH_SAH) return PT_E_INVALID;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return PT_E_NODEVICE;
  if (device < 0 || device >= ndev) return PT_E_INVALID;
  auto* sc = new pt_scene();
  int rc = ptscene::scene_from_mesh(mesh, sc->s);
  if (rc) {
    delete sc;
    return rc;
  }
  ptscene::flatten_bsdfs(sc->s);
  hipSetDevice(device);
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
    delete sc;
    return PT_E_HIP;
  }
  const auto t0 = std::chrono::steady_clock::now();
  rc = build_on_device(mesh, max_leaf, builder, sc->s, st);
  const auto t1 = std::chrono::steady_clock::now();
  hipStreamDestroy(st);
  if (rc) {
    delete sc;
    return rc;
  }
  if (build_ms) *build_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  *out = sc;
  return PT_OK;
}
