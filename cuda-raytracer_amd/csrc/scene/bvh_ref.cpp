// Restated reference BVH build, 4-wide compaction, DFS serialisation and the
// flattening CudaRenderer::loadScene performs, followed by a breadth-first
// (level-major) renumbering for the device.
//
//   Triangle::get_bbox (1e-3 padding)      src/static_scene/triangle.cpp:13-47
//   Sphere::get_bbox                       src/static_scene/sphere.h:30-32
//   BVHAccel::BVHAccel (sort by x, split)  src/bvh.cpp:339-365
//   splitBVHNode (12 planes x 3 axes)      src/bvh.cpp:48-230
//   BVHNode::compactTree (DEPTH 2, 4 way)  src/bvh.cpp:275-337
//   BVHSubTree::compress (DFS ids, levels) src/bvh.cpp:234-273
//   triangle / BSDF flattening             src/cudaRenderer.cu:1694-1827
//
// Deliberate deviations (none changes which primitive a ray hits):
//  - no MAX_LEVELS=16 / LEVEL_INDEX_SIZE=6000 / 4 KB-LDS leaf caps (cu:1801,
//    cudaRenderer.h:62-69); leaves may hold more than 32 primitives when the
//    SAH refuses to split (bvh.cpp:209-212).
//  - child boxes are rounded OUTWARD when converted to fp32 (the reference
//    rounds to nearest, make_float3 at cu:1822-1823) so that the fp32 slab test
//    is conservative for every primitive in the subtree.
#include <algorithm>
#include <cstdlib>
#include <cfloat>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <stack>

#include "scene_internal.h"

namespace ptscene {

void BBox::expand(const BBox& b) {
  min.x = std::min(min.x, b.min.x);
  min.y = std::min(min.y, b.min.y);
  min.z = std::min(min.z, b.min.z);
  max.x = std::max(max.x, b.max.x);
  max.y = std::max(max.y, b.max.y);
  max.z = std::max(max.z, b.max.z);
  extent = max - min;
}

namespace {

struct BuildCtx {
  const Scene* S;
  std::vector<BBox> boxes;  // per input prim, computed once (pure function)
  std::vector<double> cx, cy, cz;
};

BBox prim_bbox(const Scene& S, const Prim& p) {
  if (p.kind == PT_PRIM_SPHERE) {
    V3 r(p.radius, p.radius, p.radius);
    V3 lo = p.centre - r, hi = p.centre + r;
    return BBox(lo.x, lo.y, lo.z, hi.x, hi.y, hi.z);
  }
  const auto& psns = S.meshes[p.mesh].positions;
  V3 p1 = psns[p.v[0]], p2 = psns[p.v[1]], p3 = psns[p.v[2]];
  double maxX = (p1.x > p2.x) ? p1.x : p2.x;
  double maxY = (p1.y > p2.y) ? p1.y : p2.y;
  double maxZ = (p1.z > p2.z) ? p1.z : p2.z;
  maxX = (maxX > p3.x) ? maxX : p3.x;
  maxY = (maxY > p3.y) ? maxY : p3.y;
  maxZ = (maxZ > p3.z) ? maxZ : p3.z;
  double minX = (p1.x < p2.x) ? p1.x : p2.x;
  double minY = (p1.y < p2.y) ? p1.y : p2.y;
  double minZ = (p1.z < p2.z) ? p1.z : p2.z;
  minX = (minX < p3.x) ? minX : p3.x;
  minY = (minY < p3.y) ? minY : p3.y;
  minZ = (minZ < p3.z) ? minZ : p3.z;
  const double PADDING = 1e-3;
  minX -= PADDING;
  maxX += PADDING;
  minY -= PADDING;
  maxY += PADDING;
  minZ -= PADDING;
  maxZ += PADDING;
  return BBox(minX, minY, minZ, maxX, maxY, maxZ);
}

struct BNode {  // BVHNode (bvh.h:49-63)
  BBox bb;
  size_t start, range;
  BNode *l = nullptr, *r = nullptr;
  bool leaf() const { return !l && !r; }
};

struct WNode {  // BVHSubTree (bvh.h:35-47), TREE_BRANCHES = 4
  WNode* outlets[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t start = 0, range = 0;
  V3 min[4], max[4];
};

class RefBuilder {
 public:
  RefBuilder(BuildCtx& c, std::vector<int>& prims) : C(c), P(prims) {}

  // splitBVHNode, bvh.cpp:48-230.  Primitive identity is the input index.
  BNode* split(size_t max_leaf, size_t start, size_t end, BBox _bb) {
    BNode* node = new BNode{_bb, start, end - start};
    pool.emplace_back(node);
    if (end - start <= max_leaf) return node;
    double total_sa = _bb.surface_area();
    if (total_sa < 1e-15) return node;

    float current_cost = 2 * (end - start);
    float bestcost = current_cost;
    int besti = 0;
    float bestk = 0;
    BBox boxl, boxr;
    for (int i = 0; i < 3; i++) {
      sort_axis(i, start, end);
      std::vector<BBox> ltor, rtol;
      BBox b1, b2;
      double startval = cen(i, P[start]);
      double endval = cen(i, P[end - 1]);
      const int numparts = 12;
      int lastidx = (int)start;
      std::vector<int> indices;
      for (long part = 1; part <= numparts; part++) {
        double divider = startval + part * ((endval - startval) / (numparts + 1));
        // upper_bound with cmpd{X,Y,Z}(d, prim) = d < centroid
        int idx = (int)(std::upper_bound(P.begin() + start, P.begin() + end, divider,
                                         [&](double d, int b) { return d < cen(i, b); }) -
                        P.begin());
        for (int j = lastidx; j < idx; j++) b1.expand(C.boxes[P[j]]);
        indices.push_back(idx);
        lastidx = idx;
        ltor.push_back(b1);
      }
      lastidx = (int)end;
      for (long part = 1; part <= numparts; part++) {
        double divider = endval - part * ((endval - startval) / (numparts + 1));
        // lower_bound with cmpd{X,Y,Z}2(prim, d) = centroid < d
        int idx = (int)(std::lower_bound(P.begin() + start, P.begin() + end, divider,
                                         [&](int b, double d) { return cen(i, b) < d; }) -
                        P.begin());
        for (int j = lastidx - 1; j >= idx; j--) b2.expand(C.boxes[P[j]]);
        lastidx = idx;
        rtol.push_back(b2);
      }
      double mincost = current_cost;
      size_t mink = 1;
      BBox minboxl, minboxr;
      for (size_t k = 0; k < (size_t)numparts; k++) {
        int count = indices[k] - (int)start;
        int count2 = (int)(end - start) - count;
        double sa1 = ltor[k].surface_area();
        double sa2 = rtol[numparts - k - 1].surface_area();
        double cost = 5 + (sa1 / total_sa) * count * 2 + (sa2 / total_sa) * count2 * 2;
        if (mincost > cost) {
          mincost = cost;
          mink = indices[k];
          minboxl = ltor[k];
          minboxr = rtol[numparts - k - 1];
        }
      }
      if (mincost == current_cost) {
        mink = indices[1];
        minboxl = ltor[1];
        minboxr = rtol[numparts - 2];
      }
      if (mincost < bestcost) {
        bestcost = mincost;
        bestk = mink;
        besti = i;
        boxl = minboxl;
        boxr = minboxr;
      }
    }
    if (bestcost == current_cost) return node;
    sort_axis(besti, start, end);
    node->l = split(max_leaf, start, (size_t)bestk, boxl);
    node->r = split(max_leaf, (size_t)bestk, end, boxr);
    return node;
  }

  void sort_axis(int i, size_t start, size_t end) {
    const std::vector<double>& c = (i == 0) ? C.cx : (i == 1 ? C.cy : C.cz);
    std::sort(P.begin() + start, P.begin() + end, [&](int a, int b) { return c[a] < c[b]; });
  }
  double cen(int i, int p) const { return i == 0 ? C.cx[p] : (i == 1 ? C.cy[p] : C.cz[p]); }

  // BVHNode::compactTree, bvh.cpp:275-337 (DEPTH = 2, TREE_BRANCHES = 4)
  WNode* compact(BNode* n0) {
    WNode* st = new WNode();
    wpool.emplace_back(st);
    if (n0->leaf()) {
      st->range = n0->range;
      st->start = n0->start;
      return st;
    }
    int curr = 0;
    std::stack<std::pair<int, BNode*>> stk;
    stk.push({0, n0});
    while (!stk.empty()) {
      auto dn = stk.top();
      stk.pop();
      int depth = dn.first;
      BNode* n = dn.second;
      if (depth == 2) {
        if (curr >= 4) throw std::runtime_error("compactTree: more than 4 branches");
        int t = curr++;
        st->outlets[t] = compact(n);
        st->min[t] = n->bb.min;
        st->max[t] = n->bb.max;
        continue;
      }
      if (n->l) stk.push({depth + 1, n->l});
      if (n->r) stk.push({depth + 1, n->r});
      if (!n->l && !n->r && depth != 2) {
        if (curr >= 4) throw std::runtime_error("compactTree: more than 4 branches");
        int t = curr++;
        st->outlets[t] = compact(n);
        st->min[t] = n->bb.min;
        st->max[t] = n->bb.max;
        continue;
      }
    }
    return st;
  }

  std::vector<std::unique_ptr<BNode>> pool;
  std::vector<std::unique_ptr<WNode>> wpool;

 private:
  BuildCtx& C;
  std::vector<int>& P;
};

struct CNode {  // C_BVHSubTree (bvh.h:24-32) in DFS pre-order
  int64_t outlets[4];
  size_t start, range;
  V3 min[4], max[4];
  int depth;
};

// BVHSubTree::compress, bvh.cpp:234-273 (without the 16-level exit)
int compress(const WNode* w, std::vector<CNode>& tree, std::vector<std::vector<int>>& levels,
             int depth) {
  int idx = (int)tree.size();
  tree.push_back(CNode());
  if ((int)levels.size() <= depth) levels.push_back({});
  levels[depth].push_back(idx);
  tree[idx].range = w->range;
  tree[idx].start = w->start;
  tree[idx].depth = depth;
  for (int i = 0; i < 4; i++) {
    if (w->outlets[i]) {
      int off = compress(w->outlets[i], tree, levels, depth + 1);
      tree[idx].outlets[i] = off;
      tree[idx].min[i] = w->min[i];
      tree[idx].max[i] = w->max[i];
    } else {
      tree[idx].outlets[i] = -1;
    }
  }
  return idx;
}

float round_down(double v) {
  float f = (float)v;
  if ((double)f > v) f = nextafterf(f, -FLT_MAX);
  return f;
}
float round_up(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, FLT_MAX);
  return f;
}

}  // namespace

double box_guard(const Scene& S) {
  double m = 0.0;
  auto upd = [&](double v) { m = std::max(m, std::fabs(v)); };
  for (const Mesh& me : S.meshes)
    for (const V3& p : me.positions) {
      upd(p.x);
      upd(p.y);
      upd(p.z);
    }
  for (const Prim& p : S.prims)
    if (p.kind == PT_PRIM_SPHERE) {
      upd(std::fabs(p.centre.x) + p.radius);
      upd(std::fabs(p.centre.y) + p.radius);
      upd(std::fabs(p.centre.z) + p.radius);
    }
  for (int k = 0; k < 3; ++k) {
    upd(S.camera.origin[k]);
    upd(S.light.position[k]);
  }
  // PT_BOX_GUARD=0 turns the band off (diagnostics: scripts/dev/guard_off.py)
  const char* e = getenv("PT_BOX_GUARD");
  if (e && atoi(e) == 0) return 0.0;
  return std::ldexp(m, -14);
}

// BSDF table: one entry per scene object (cu:1694-1723)
void flatten_bsdfs(Scene& S) {
  S.dbsdfs.clear();
  for (const Material& m : S.materials) {
    pt_bsdf b{};
    b.type = m.type;
    for (int k = 0; k < 3; ++k) {
      b.albedo[k] = m.albedo[k];
      b.transmittance[k] = m.trans[k];
    }
    b.ior = m.ior;
    b.roughness = m.roughness;
    S.dbsdfs.push_back(b);
  }
}

void build_bvh_and_flatten(Scene& S, size_t max_leaf) {
  const int n = (int)S.prims.size();
  BuildCtx C;
  C.S = &S;
  C.boxes.resize(n);
  C.cx.resize(n);
  C.cy.resize(n);
  C.cz.resize(n);
  BBox bb;
  for (int i = 0; i < n; ++i) {
    C.boxes[i] = prim_bbox(S, S.prims[i]);
    V3 c = C.boxes[i].centroid();
    C.cx[i] = c.x;
    C.cy[i] = c.y;
    C.cz[i] = c.z;
    bb.expand(C.boxes[i]);
  }
  std::vector<int> order(n);
  for (int i = 0; i < n; ++i) order[i] = i;
  RefBuilder B(C, order);
  std::sort(order.begin(), order.end(), [&](int a, int b) { return C.cx[a] < C.cx[b]; });  // bvh.cpp:358
  BNode* root = n ? B.split(max_leaf, 0, n, bb) : nullptr;

  // sorted primitive arrays (cu:1760-1792): v0,v1,v2 and n0..n2 in fp32
  S.sorted_to_input = order;
  S.dprims.assign(n, pt_prim{});
  S.dshading.assign(n, pt_prim_shading{});
  for (int i = 0; i < n; ++i) {
    const Prim& p = S.prims[order[i]];
    pt_prim& d = S.dprims[i];
    pt_prim_shading& sh = S.dshading[i];
    uint32_t meta = ((uint32_t)p.kind << 28) | ((uint32_t)p.object & 0x0FFFFFFFu);
    if (p.kind == PT_PRIM_SPHERE) {
      d.q[0] = (float)p.centre.x;
      d.q[1] = (float)p.centre.y;
      d.q[2] = (float)p.centre.z;
      memcpy(&d.q[3], &meta, 4);
      float r = (float)p.radius;
      d.q[4] = r;
      d.q[5] = r * r;
      continue;
    }
    const Mesh& m = S.meshes[p.mesh];
    float v[3][3], nn[3][3];
    for (int k = 0; k < 3; ++k) {
      v[k][0] = (float)m.positions[p.v[k]].x;
      v[k][1] = (float)m.positions[p.v[k]].y;
      v[k][2] = (float)m.positions[p.v[k]].z;
      nn[k][0] = (float)m.normals[p.v[k]].x;
      nn[k][1] = (float)m.normals[p.v[k]].y;
      nn[k][2] = (float)m.normals[p.v[k]].z;
    }
    // fp32 operands of intersectRayTriangle (cu:223-237), same operation order
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
    float dN = N[0] * v[0][0] + N[1] * v[0][1] + N[2] * v[0][2];
    // edge normals m_k = N x e_k (pt_api.h): dot(m_k, P - v_k) is the
    // reference's dot(N, cross(e_k, P - v_k))
    float en[3][3];
    const float* ek[3] = {e0, e1, e2};
    for (int k = 0; k < 3; ++k) {
      en[k][0] = N[1] * ek[k][2] - N[2] * ek[k][1];
      en[k][1] = N[2] * ek[k][0] - N[0] * ek[k][2];
      en[k][2] = N[0] * ek[k][1] - N[1] * ek[k][0];
    }
    float* q = d.q;
    q[0] = v[0][0]; q[1] = v[0][1]; q[2] = v[0][2]; memcpy(&q[3], &meta, 4);
    q[4] = v[1][0]; q[5] = v[1][1]; q[6] = v[1][2]; q[7] = dN;
    q[8] = v[2][0]; q[9] = v[2][1]; q[10] = v[2][2]; q[11] = en[0][0];
    q[12] = N[0]; q[13] = N[1]; q[14] = N[2]; q[15] = en[0][1];
    q[16] = en[1][0]; q[17] = en[1][1]; q[18] = en[1][2]; q[19] = en[0][2];
    q[20] = en[2][0]; q[21] = en[2][1]; q[22] = en[2][2]; q[23] = 0.f;
    for (int k = 0; k < 3; ++k) {
      sh.n0[k] = nn[0][k];
      sh.n1[k] = nn[1][k];
      sh.n2[k] = nn[2][k];
    }
  }

  flatten_bsdfs(S);

  // wide tree + DFS compress + BFS renumbering
  S.dnodes.clear();
  S.level_start.clear();
  S.level_counts.clear();
  if (!root) {
    S.level_start = {0};
    return;
  }
  WNode* wroot = B.compact(root);
  const double G = box_guard(S);  // scene_internal.h: conservative fp32 slab tests
  std::vector<CNode> tree;
  std::vector<std::vector<int>> levels;
  compress(wroot, tree, levels, 0);
  std::vector<int> dfs_to_bfs(tree.size(), -1);
  int next = 0;
  for (auto& lv : levels) {
    S.level_start.push_back(next);
    S.level_counts.push_back((int)lv.size());
    for (int id : lv) dfs_to_bfs[id] = next++;
  }
  S.level_start.push_back(next);
  S.dnodes.assign(tree.size(), pt_node{});
  for (size_t lv = 0; lv < levels.size(); ++lv) {
    for (int id : levels[lv]) {
      const CNode& c = tree[id];
      pt_node& d = S.dnodes[dfs_to_bfs[id]];
      d.level = (int32_t)lv;
      d.ref_id = id;
      d.prim_start = (int32_t)c.start;
      d.prim_count = (int32_t)c.range;
      for (int i = 0; i < 4; ++i) {
        if (c.range == 0 && c.outlets[i] >= 0) {
          d.child[i] = dfs_to_bfs[c.outlets[i]];
          d.bmin_x[i] = round_down(c.min[i].x - G);
          d.bmin_y[i] = round_down(c.min[i].y - G);
          d.bmin_z[i] = round_down(c.min[i].z - G);
          d.bmax_x[i] = round_up(c.max[i].x + G);
          d.bmax_y[i] = round_up(c.max[i].y + G);
          d.bmax_z[i] = round_up(c.max[i].z + G);
        } else {
          d.child[i] = -1;
          // empty slot: an inverted box no ray can enter
          d.bmin_x[i] = d.bmin_y[i] = d.bmin_z[i] = FLT_MAX;
          d.bmax_x[i] = d.bmax_y[i] = d.bmax_z[i] = -FLT_MAX;
        }
      }
    }
  }
}

}  // namespace ptscene
