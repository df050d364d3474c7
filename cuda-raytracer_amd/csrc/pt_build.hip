// GPU BVH build: a binary BVH built on the device,
// collapsed to the reference's 4-wide, level-major node layout.
//
// The reference builds on the host (bvh.cpp:48-337: per-node full re-sorts on
// three axes and a 12-bucket SAH, O(n log^2 n), 0.84 s for CBbunny) and then
// compacts binary depth 2 into 4-wide nodes (compactTree, DEPTH=2).  Here:
//   1. primitive boxes and centroids             k_prim_bounds
//   2. centroid bounds (ordered-int atomics)     k_reduce_bounds
//   3. 63-bit Morton codes, radix sort           k_morton + hipcub
//   4. binary tree: PLOC agglomerative clustering (default, k_ploc_*: mutual
//      nearest neighbours by union box area in a Morton-order window, then a
//      depth-first renumbering of the primitives), or the radix tree of
//      Karras 2012 (PT_GPU_BVH=lbvh; k_karras)
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

__device__ __forceinline__ int2 node_range(int v, int n, const int2* __restrict__ range) {
  return v >= n - 1 ? make_int2(v - (n - 1), v - (n - 1)) : range[v];
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
                                             int (&out)[4]) {
  const int2 r = node_range(v, n, range);
  if (v >= n - 1 || r.y - r.x + 1 <= max_leaf) return 0;
  const int2 c = child[v];
  out[0] = c.x;
  out[1] = c.y;
  int m = 2;
  while (m < 4) {
    int best = -1;
    float ba = -1.0f;
    for (int j = 0; j < m; ++j) {
      const int u = out[j];
      if (u >= n - 1) continue;
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
                             const Box* __restrict__ nbox, uint32_t* __restrict__ cnt) {
  const int f = blockIdx.x * TPB + threadIdx.x;
  if (f >= m) return;
  int out[4];
  cnt[f] = (uint32_t)wide_children(front[f], n, max_leaf, child, range, nbox, out);
}

// 6b. write the level's pt_node records and the next frontier
__global__ void k_wide_emit(const int* __restrict__ front, int m, int n, int max_leaf, int level, int base,
                            int next_base, const int2* __restrict__ child, const int2* __restrict__ range,
                            const Box* __restrict__ nbox, const uint32_t* __restrict__ off, pt_node* __restrict__ nodes,
                            int* __restrict__ next) {
  const int f = blockIdx.x * TPB + threadIdx.x;
  if (f >= m) return;
  const int v = front[f];
  int out[4];
  const int k = wide_children(v, n, max_leaf, child, range, nbox, out);
  pt_node d;
  d.level = level;
  d.ref_id = v;
  const int2 r = node_range(v, n, range);
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
  hipLaunchKernelGGL(k_morton, g, dim3(TPB), 0, st, d_cen, n, d_bounds, d_key, d_idx);
  size_t tmp_bytes = 0;
  BCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, d_key, d_key2, d_idx, d_idx2, n, 0, 63, st));
  void* d_tmp = B.alloc<uint8_t>(tmp_bytes);
  if (!d_tmp) return PT_E_HIP;
  BCHK(hipcub::DeviceRadixSort::SortPairs(d_tmp, tmp_bytes, d_key, d_key2, d_idx, d_idx2, n, 0, 63, st));
  // binary tree: PLOC or the radix tree
  const bool ploc = n > 1 && builder == PT_GPU_BVH_PLOC;
  uint32_t* d_sorted = d_idx2;  // final primitive order
  if (ploc) {
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
  const int root = n > 1 ? 0 : n - 1;  // a single primitive: the root is leaf 0
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
                       d_cnt);
    BCHK(hipcub::DeviceScan::ExclusiveSum(d_scan, scan_bytes, d_cnt, d_off, m + 1, st));
    uint32_t next_m = 0;
    BCHK(hipMemcpyAsync(&next_m, d_off + m, 4, hipMemcpyDeviceToHost, st));
    hipLaunchKernelGGL(k_wide_emit, gm, dim3(TPB), 0, st, d_front, m, n, max_leaf, level, base, base + m, d_child,
                       d_range, d_nbox, d_off, d_nodes, d_next);
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
  return pt_scene_build_gpu_ex(mesh, device, max_leaf, PT_GPU_BVH_PLOC, out, build_ms);
}

extern "C" int pt_scene_build_gpu_ex(const pt_mesh_desc* mesh, int32_t device, int32_t max_leaf, int32_t builder,
                                     pt_scene** out, double* build_ms) {
  if (!out) return PT_E_INVALID;
  *out = nullptr;
  if (max_leaf < 1 || max_leaf > 64) return PT_E_INVALID;
  if (builder != PT_GPU_BVH_PLOC && builder != PT_GPU_BVH_LBVH) return PT_E_INVALID;
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
