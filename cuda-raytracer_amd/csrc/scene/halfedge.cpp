// Restatement of the parts of Scotty3D's halfedge mesh that decide what the
// renderer sees: vertex order, the (v1,v2,v3) order of each triangle and the
// area-weighted vertex normals.
//
//   HalfedgeMesh::build            src/halfEdgeMesh.cpp:47-418
//   Vertex::normal / isBoundary    src/halfEdgeMesh.h:619-670
//   StaticScene::Mesh::Mesh        src/static_scene/object.cpp:17-58
//
// The reference keeps elements in std::lists; here they are index arrays in
// the same creation order, which is all the traversal orders depend on.
#include <map>
#include <set>

#include "scene_internal.h"

namespace ptscene {

double V3::norm() const { return std::sqrt(x * x + y * y + z * z); }

namespace {
struct HE {
  int next = -1, twin = -1, vertex = -1, face = -1;
};
}  // namespace

bool build_static_mesh(const std::vector<std::vector<size_t>>& polygons,
                       const std::vector<V3>& vertex_positions, Mesh& out,
                       std::vector<std::array<int, 3>>& tris, std::string& err) {
  typedef size_t Index;
  std::map<Index, int> index_to_vertex;  // HalfedgeMesh.cpp:93
  std::vector<int> vert_he;              // Vertex::_halfedge
  std::vector<int> vert_degree;

  // First pass: allocate vertices in order of first appearance (cpp:100-152).
  for (const auto& p : polygons) {
    if (p.size() < 3) {
      err = "polygon with fewer than three vertices";
      return false;
    }
    std::set<Index> distinct;
    for (Index i : p) {
      distinct.insert(i);
      auto it = index_to_vertex.find(i);
      if (it == index_to_vertex.end()) {
        index_to_vertex[i] = (int)vert_he.size();
        vert_he.push_back(-1);
        vert_degree.push_back(1);
      } else {
        vert_degree[it->second]++;
      }
    }
    if (distinct.size() < p.size()) {
      err = "polygon with repeated vertices";
      return false;
    }
  }
  const int nfaces = (int)polygons.size();
  std::vector<int> face_he(nfaces, -1);
  std::vector<HE> he;
  he.reserve(polygons.size() * 4 + 16);
  std::map<std::pair<Index, Index>, int> pair_to_he;

  // Second pass: halfedges, twins, next pointers (cpp:169-252).
  for (int f = 0; f < nfaces; ++f) {
    const auto& p = polygons[f];
    const size_t degree = p.size();
    std::vector<int> face_hes;
    for (size_t i = 0; i < degree; ++i) {
      Index a = p[i], b = p[(i + 1) % degree];
      if (pair_to_he.count({a, b})) {
        err = "non-manifold or inconsistently oriented mesh";
        return false;
      }
      int hab = (int)he.size();
      he.push_back(HE());
      pair_to_he[{a, b}] = hab;
      he[hab].face = f;
      face_he[f] = hab;  // the face keeps its LAST created halfedge
      he[hab].vertex = index_to_vertex[a];
      vert_he[he[hab].vertex] = hab;
      face_hes.push_back(hab);
      auto iba = pair_to_he.find({b, a});
      if (iba != pair_to_he.end()) {
        he[hab].twin = iba->second;
        he[iba->second].twin = hab;
      } else {
        he[hab].twin = -1;
      }
    }
    for (size_t i = 0; i < degree; ++i) he[face_hes[i]].next = face_hes[(i + 1) % degree];
  }

  // Boundary vertices point at a twinless halfedge (cpp:256-268).
  for (size_t v = 0; v < vert_he.size(); ++v) {
    int h = vert_he[v];
    const int start = h;
    do {
      if (he[h].twin == -1) {
        vert_he[v] = h;
        break;
      }
      h = he[he[h].twin].next;
    } while (h != start);
  }

  // Boundary loops (cpp:271-340).  Faces >= nfaces are boundary faces.
  int nboundary = 0;
  for (size_t h = 0; h < he.size(); ++h) {
    if (he[h].twin != -1) continue;
    const int b = nfaces + nboundary++;
    std::vector<int> bhes;
    int i = (int)h;
    do {
      int t = (int)he.size();
      he.push_back(HE());
      bhes.push_back(t);
      he[i].twin = t;
      he[t].twin = i;
      he[t].face = b;
      he[t].vertex = he[he[i].next].vertex;
      i = he[i].next;
      while (i != (int)h && he[i].twin != -1) {
        i = he[i].twin;
        i = he[i].next;
      }
    } while (i != (int)h);
    const size_t degree = bhes.size();
    for (size_t p = 0; p < degree; ++p) he[bhes[p]].next = bhes[(p - 1 + degree) % degree];
  }

  // First non-boundary halfedge (cpp:346-348).
  for (size_t v = 0; v < vert_he.size(); ++v) vert_he[v] = he[he[vert_he[v]].twin].next;

  // Manifold check (cpp:351-378).
  for (size_t v = 0; v < vert_he.size(); ++v) {
    int count = 0, h = vert_he[v];
    do {
      if (he[h].face < nfaces) count++;
      h = he[he[h].twin].next;
    } while (h != vert_he[v]);
    if (count != vert_degree[v]) {
      err = "non-manifold vertex";
      return false;
    }
  }
  if (vertex_positions.size() < vert_he.size()) {
    err = "fewer vertex positions than vertices";
    return false;
  }
  // Positions: the k-th smallest input index gets vertexPositions[k] (cpp:399-412).
  std::vector<V3> pos(vert_he.size());
  {
    int k = 0;
    for (const auto& e : index_to_vertex) pos[e.second] = vertex_positions[k++];
  }

  auto is_boundary = [&](int v) {
    int h = vert_he[v];
    do {
      if (he[h].face >= nfaces) return true;
      h = he[he[h].twin].next;
    } while (h != vert_he[v]);
    return false;
  };
  // Vertex::normal (halfEdgeMesh.h:619-644).
  out.positions = pos;
  out.normals.resize(pos.size());
  for (size_t v = 0; v < pos.size(); ++v) {
    V3 N(0., 0., 0.);
    const V3 pi = pos[v];
    int h = vert_he[v];
    if (is_boundary((int)v)) {
      do {
        V3 pj = pos[he[he[h].next].vertex];
        V3 pk = pos[he[he[he[h].next].next].vertex];
        N += cross(pj - pi, pk - pi);
        h = he[he[h].next].twin;
      } while (h != vert_he[v]);
    } else {
      do {
        V3 pj = pos[he[he[h].next].vertex];
        V3 pk = pos[he[he[he[h].next].next].vertex];
        N += cross(pj - pi, pk - pi);
        h = he[he[h].twin].next;
      } while (h != vert_he[v]);
    }
    // Vector3D::normalize: (*this) /= norm()  ==  *this *= (1./norm)
    const double s = 1. / N.norm();
    N.x *= s;
    N.y *= s;
    N.z *= s;
    out.normals[v] = N;
  }
  // StaticScene::Mesh: one triangle per face from f->halfedge() (object.cpp:50-55).
  // Vertex labels are the vertex list order, which is our vertex index.
  tris.clear();
  tris.reserve(nfaces);
  for (int f = 0; f < nfaces; ++f) {
    int h = face_he[f];
    tris.push_back({he[h].vertex, he[he[h].next].vertex, he[he[he[h].next].next].vertex});
  }
  return true;
}

}  // namespace ptscene
