// COLLADA subset loader: the CMU462 flavour used by media/pathtracer.
//
// Restates, in the order the reference evaluates them:
//   ColladaParser::load / uri table / up-axis fix   src/collada/collada.cpp:116-210
//   get_element url indirection                    collada.cpp:69-89
//   parse_node (matrix/rotate/translate/scale)      collada.cpp:212-400
//   parse_light / parse_sphere / parse_polymesh     collada.cpp:473-820
//   parse_material (CMU462 profile wins)            collada.cpp:868-950
//   CudaRenderer::loadFromSceneInfo (camera)        src/cudaRenderer.cu:1572-1677
//   DynamicScene::AreaLight / PointLight            src/dynamic_scene/area_light.h:12-24,
//                                                   point_light.h:15-18
//   DynamicScene::Mesh (vertex transform)           src/dynamic_scene/mesh.cpp:21-45
//   DynamicScene::Sphere (centre, radius*scale)     src/dynamic_scene/sphere.cpp:9-17
// The XML reader below is a minimal, self-contained DOM builder (the reference
// vendors tinyxml2, which is not reused).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>

#include "scene_internal.h"

namespace ptscene {

// ---- minimal XML DOM ----------------------------------------------------------
namespace {
struct XNode {
  std::string name;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::string text;
  std::vector<std::unique_ptr<XNode>> kids;
  const char* attr(const char* k) const {
    for (auto& a : attrs)
      if (a.first == k) return a.second.c_str();
    return nullptr;
  }
  XNode* child(const char* n) const {
    for (auto& c : kids)
      if (c->name == n) return c.get();
    return nullptr;
  }
  XNode* first_child() const { return kids.empty() ? nullptr : kids[0].get(); }
};

class XmlParser {
 public:
  explicit XmlParser(const std::string& s) : s_(s) {}
  std::unique_ptr<XNode> parse(std::string& err) {
    auto root = std::make_unique<XNode>();
    root->name = "#document";
    std::vector<XNode*> stack{root.get()};
    while (i_ < s_.size()) {
      if (s_[i_] != '<') {
        size_t j = s_.find('<', i_);
        if (j == std::string::npos) j = s_.size();
        stack.back()->text.append(s_, i_, j - i_);
        i_ = j;
        continue;
      }
      if (s_.compare(i_, 4, "<!--") == 0) {
        size_t j = s_.find("-->", i_);
        if (j == std::string::npos) return fail(err, "unterminated comment");
        i_ = j + 3;
        continue;
      }
      if (s_.compare(i_, 2, "<?") == 0 || s_.compare(i_, 2, "<!") == 0) {
        size_t j = s_.find('>', i_);
        if (j == std::string::npos) return fail(err, "unterminated declaration");
        i_ = j + 1;
        continue;
      }
      if (s_.compare(i_, 2, "</") == 0) {
        size_t j = s_.find('>', i_);
        if (j == std::string::npos) return fail(err, "unterminated end tag");
        std::string nm = trim(s_.substr(i_ + 2, j - i_ - 2));
        if (stack.size() < 2 || stack.back()->name != nm) return fail(err, "mismatched </" + nm + ">");
        stack.pop_back();
        i_ = j + 1;
        continue;
      }
      // start tag
      size_t j = i_ + 1;
      while (j < s_.size() && !isspace((unsigned char)s_[j]) && s_[j] != '>' && s_[j] != '/') j++;
      auto node = std::make_unique<XNode>();
      node->name = s_.substr(i_ + 1, j - i_ - 1);
      bool self_close = false;
      while (true) {
        while (j < s_.size() && isspace((unsigned char)s_[j])) j++;
        if (j >= s_.size()) return fail(err, "unterminated tag");
        if (s_[j] == '/') {
          self_close = true;
          j = s_.find('>', j);
          if (j == std::string::npos) return fail(err, "bad tag");
          j++;
          break;
        }
        if (s_[j] == '>') {
          j++;
          break;
        }
        size_t k = j;
        while (k < s_.size() && s_[k] != '=' && !isspace((unsigned char)s_[k])) k++;
        std::string an = s_.substr(j, k - j);
        while (k < s_.size() && s_[k] != '"' && s_[k] != '\'') k++;
        if (k >= s_.size()) return fail(err, "bad attribute");
        char q = s_[k];
        size_t e = s_.find(q, k + 1);
        if (e == std::string::npos) return fail(err, "bad attribute value");
        node->attrs.push_back({an, s_.substr(k + 1, e - k - 1)});
        j = e + 1;
      }
      XNode* raw = node.get();
      stack.back()->kids.push_back(std::move(node));
      if (!self_close) stack.push_back(raw);
      i_ = j;
    }
    if (stack.size() != 1) return fail(err, "unclosed elements");
    return root;
  }

 private:
  static std::string trim(const std::string& x) {
    size_t a = 0, b = x.size();
    while (a < b && isspace((unsigned char)x[a])) a++;
    while (b > a && isspace((unsigned char)x[b - 1])) b--;
    return x.substr(a, b - a);
  }
  std::unique_ptr<XNode> fail(std::string& err, const std::string& m) {
    err = "XML: " + m;
    return nullptr;
  }
  const std::string& s_;
  size_t i_ = 0;
};

// ---- COLLADA walker -------------------------------------------------------------
struct LightInfo {
  int type = 0;  // 0 none, 1 ambient, 2 directional, 3 area, 4 point, 5 spot
  float spectrum[3] = {1, 1, 1};
};

struct Loader {
  Scene& S;
  std::string& err;
  std::map<std::string, XNode*> uri;
  M4 global = M4::identity();
  V3 up{0, 1, 0};
  // camera state (cudaRenderer.cu:1590-1607): the last camera node wins
  bool cam = false;
  V3 c_pos, c_dir;
  struct PendingLight {
    LightInfo info;
    M4 T;
  };
  std::vector<PendingLight> lights;

  Loader(Scene& s, std::string& e) : S(s), err(e) {}

  void build_uri(XNode* n) {
    if (const char* id = n->attr("id")) uri[id] = n;
    for (auto& k : n->kids) build_uri(k.get());
  }
  XNode* uri_find(const std::string& id) {
    auto it = uri.find(id);
    return it == uri.end() ? nullptr : it->second;
  }
  // collada.cpp:69-89: follow the path, then one level of url indirection
  XNode* get_element(XNode* x, const std::string& query) {
    std::stringstream ss(query);
    std::string tok;
    XNode* e = x;
    while (e && std::getline(ss, tok, '/')) e = e->child(tok.c_str());
    if (e) {
      if (const char* url = e->attr("url")) e = uri_find(url + 1);
    }
    return e;
  }
  XNode* technique_common(XNode* x) {
    if (XNode* p = x->child("profile_COMMON")) {
      for (auto& t : p->kids)
        if (t->name == "technique" && t->attr("sid") && std::string(t->attr("sid")) == "common")
          return t.get();
    }
    return x->child("technique_common");
  }
  XNode* technique_cmu462(XNode* x) {
    XNode* extra = x->child("extra");
    if (!extra) return nullptr;
    for (auto& t : extra->kids)
      if (t->name == "technique" && t->attr("profile") && std::string(t->attr("profile")) == "CMU462")
        return t.get();
    return nullptr;
  }
  static bool spectrum_from(XNode* n, float out[3]) {
    if (!n) return false;
    std::stringstream ss(n->text);
    ss >> out[0] >> out[1] >> out[2];
    return true;
  }

  Material parse_material(XNode* xml) {
    Material m;
    XNode* eff = get_element(xml, "instance_effect");
    if (!eff) return m;
    XNode* cmu = technique_cmu462(eff);
    XNode* com = technique_common(eff);
    if (cmu) {
      // the last recognised element wins (collada.cpp:887-942)
      for (auto& b : cmu->kids) {
        const std::string& t = b->name;
        if (t == "emission") {
          m = Material();
          m.type = PT_BSDF_EMISSION;
          spectrum_from(get_element(b.get(), "radiance"), m.albedo);
        } else if (t == "mirror") {
          m = Material();
          m.type = PT_BSDF_MIRROR;
          spectrum_from(get_element(b.get(), "reflectance"), m.albedo);
        } else if (t == "glass" || t == "refraction") {
          m = Material();
          m.type = t == "glass" ? PT_BSDF_GLASS : PT_BSDF_REFRACTION;
          if (t == "glass")
            spectrum_from(get_element(b.get(), "reflectance"), m.albedo);
          else
            m.albedo[0] = m.albedo[1] = m.albedo[2] = 0.f;
          spectrum_from(get_element(b.get(), "transmittance"), m.trans);
          if (XNode* ior = get_element(b.get(), "ior")) m.ior = (float)atof(ior->text.c_str());
          if (XNode* r = get_element(b.get(), "roughness")) m.roughness = (float)atof(r->text.c_str());
        }
      }
    } else if (com) {
      m.type = PT_BSDF_DIFFUSE;
      if (XNode* d = get_element(com, "phong/diffuse/color")) {
        spectrum_from(d, m.albedo);
      } else {
        m.albedo[0] = m.albedo[1] = m.albedo[2] = .5f;
      }
    } else {
      m.albedo[0] = m.albedo[1] = m.albedo[2] = .5f;
    }
    return m;
  }

  bool parse_light(XNode* xml, LightInfo& L) {
    XNode* com = technique_common(xml);
    XNode* cmu = technique_cmu462(xml);
    XNode* tech = cmu ? cmu : com;
    if (!tech) {
      err = "light without supported profile";
      return false;
    }
    XNode* e = tech->first_child();
    if (!e) return true;
    const std::string& t = e->name;
    if (t == "ambient") L.type = 1;
    else if (t == "directional") L.type = 2;
    else if (t == "area") L.type = 3;
    else if (t == "point") L.type = 4;
    else if (t == "spot") L.type = 5;
    else {
      err = "unsupported light type " + t;
      return false;
    }
    spectrum_from(get_element(e, "color"), L.spectrum);
    return true;
  }

  bool parse_polymesh(XNode* geom, std::vector<std::vector<size_t>>& polys, std::vector<V3>& verts) {
    XNode* mesh = geom->child("mesh");
    if (!mesh) {
      err = "geometry without mesh";
      return false;
    }
    std::map<std::string, std::vector<float>> sources;
    for (auto& src : mesh->kids) {
      if (src->name != "source") continue;
      XNode* fa = src->child("float_array");
      if (!fa) continue;
      size_t n = fa->attr("count") ? (size_t)atol(fa->attr("count")) : 0;
      std::vector<float> v;
      v.reserve(n);
      const char* p = fa->text.c_str();
      char* end;
      for (size_t i = 0; i < n; ++i) {
        // collada.cpp:661-664 reads with `ss >> float`; strtof rounds identically
        float f = strtof(p, &end);
        if (end == p) break;
        v.push_back(f);
        p = end;
      }
      sources[src->attr("id") ? src->attr("id") : ""] = std::move(v);
    }
    XNode* ev = mesh->child("vertices");
    if (!ev) {
      err = "mesh without vertices";
      return false;
    }
    std::string vid = ev->attr("id") ? ev->attr("id") : "";
    std::vector<V3> vertices;
    for (auto& in : ev->kids) {
      if (in->name != "input" || !in->attr("semantic")) continue;
      if (std::string(in->attr("semantic")) == "POSITION") {
        auto it = sources.find(in->attr("source") + 1);
        if (it == sources.end()) {
          err = "undefined POSITION source";
          return false;
        }
        for (size_t i = 0; i + 2 < it->second.size(); i += 3)
          vertices.push_back(V3(it->second[i], it->second[i + 1], it->second[i + 2]));
      }
    }
    XNode* pl = mesh->child("polylist");
    bool is_poly = true;
    if (!pl) {
      pl = mesh->child("triangles");
      is_poly = false;
    }
    if (!pl) {
      err = "mesh uses neither polylist nor triangles";
      return false;
    }
    bool has_v = false, has_n = false, has_t = false;
    size_t voff = 0;
    for (auto& in : pl->kids) {
      if (in->name != "input" || !in->attr("semantic")) continue;
      std::string sem = in->attr("semantic");
      size_t off = in->attr("offset") ? (size_t)atol(in->attr("offset")) : 0;
      if (sem == "VERTEX") {
        has_v = true;
        voff = off;
        if (std::string(in->attr("source") + 1) != vid) {
          err = "undefined VERTEX source";
          return false;
        }
        verts = vertices;
      } else if (sem == "NORMAL") {
        has_n = true;
      } else if (sem == "TEXCOORD") {
        has_t = true;
      }
    }
    size_t npoly = pl->attr("count") ? (size_t)atol(pl->attr("count")) : 0;
    size_t stride = (has_v ? 1 : 0) + (has_n ? 1 : 0) + (has_t ? 1 : 0);
    std::vector<size_t> sizes;
    size_t nidx = 0;
    if (is_poly) {
      XNode* vc = pl->child("vcount");
      if (!vc) {
        err = "polygon sizes undefined";
        return false;
      }
      std::stringstream ss(vc->text);
      for (size_t i = 0; i < npoly; ++i) {
        size_t sz = 0;
        ss >> sz;
        sizes.push_back(sz);
        nidx += sz * stride;
      }
    } else {
      for (size_t i = 0; i < npoly; ++i) {
        sizes.push_back(3);
        nidx += 3 * stride;
      }
    }
    XNode* ep = pl->child("p");
    if (!ep) {
      err = "no index array";
      return false;
    }
    std::vector<size_t> idx;
    idx.reserve(nidx);
    {
      const char* p = ep->text.c_str();
      char* end;
      for (size_t i = 0; i < nidx; ++i) {
        unsigned long v = strtoul(p, &end, 10);
        if (end == p) break;
        idx.push_back(v);
        p = end;
      }
      if (idx.size() != nidx) {
        err = "short index array";
        return false;
      }
    }
    polys.assign(npoly, {});
    if (has_v) {
      size_t k = 0;
      for (size_t i = 0; i < npoly; ++i)
        for (size_t j = 0; j < sizes[i]; ++j) {
          polys[i].push_back(idx[k * stride + voff]);
          k++;
        }
    }
    return true;
  }

  V3 xform_point(const M4& T, const V3& p, bool project) {
    double in[4] = {p.x, p.y, p.z, 1.0}, out[4];
    T.mul4(in, out);
    if (project) {
      double invW = 1.0 / out[3];
      return V3(out[0] * invW, out[1] * invW, out[2] * invW);
    }
    return V3(out[0], out[1], out[2]);
  }
  V3 xform_dir0(const M4& T, const V3& p) {
    double in[4] = {p.x, p.y, p.z, 0.0}, out[4];
    T.mul4(in, out);
    return V3(out[0], out[1], out[2]);
  }

  bool parse_node(XNode* xml, const M4& parent) {
    M4 local = M4::identity();
    for (auto& e : xml->kids) {
      const std::string& nm = e->name;
      if (nm == "matrix") {
        std::stringstream ss(e->text);
        M4 m;
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j) ss >> m(i, j);
        local = m;
        break;
      }
      if (nm == "translate") {
        M4 m = M4::identity();
        std::stringstream ss(e->text);
        ss >> m(0, 3) >> m(1, 3) >> m(2, 3);
        local = m * local;
      } else if (nm == "scale") {
        M4 m = M4::identity();
        std::stringstream ss(e->text);
        ss >> m(0, 0) >> m(1, 1) >> m(1, 1);  // sic: collada.cpp:314-316
        local = m * local;
      }
    }
    M4 T = parent * local;  // node.transform = transform * node.transform
    for (auto& c : xml->kids)
      if (c->name == "node" && !parse_node(c.get(), T)) return false;

    XNode* e_cam = get_element(xml, "instance_camera");
    XNode* e_light = get_element(xml, "instance_light");
    XNode* e_geom = get_element(xml, "instance_geometry");
    if (e_cam) {
      // cudaRenderer.cu:1592-1593 (c_pos starts at 0; view_dir = (0,0,-1), w=1)
      c_pos = xform_point(T, V3(0, 0, 0), false);
      c_dir = xform_point(T, V3(0, 0, -1), false).unit();
      cam = true;
      // optics (collada.cpp:440-462): xfov/yfov default 50/35 degrees, yfov
      // from the aspect ratio when only xfov is given
      if (XNode* persp = get_element(e_cam, "optics/technique_common/perspective")) {
        XNode* xf = persp->child("xfov");
        XNode* yf = persp->child("yfov");
        S.cam_hfov = xf ? atof(xf->text.c_str()) : 50.0f;
        S.cam_vfov = yf ? atof(yf->text.c_str()) : 35.0f;
        if (!yf) {
          XNode* ar = persp->child("aspect_ratio");
          if (!ar) {
            err = "incomplete perspective definition";
            return false;
          }
          const float aspect = (float)atof(ar->text.c_str());
          S.cam_vfov = 2 * (atan(tan((0.5 * S.cam_hfov) * M_PI / 180.0) / aspect) * 180.0 / M_PI);
        }
        S.have_optics = true;
      }
      S.cam_dir = c_dir;
    } else if (e_light) {
      PendingLight pl;
      if (!parse_light(e_light, pl.info)) return false;
      pl.T = T;
      lights.push_back(pl);
    } else if (e_geom) {
      Material mat;
      bool has_mat = false;
      if (XNode* im = get_element(xml, "instance_geometry/bind_material/technique_common/instance_material")) {
        const char* tgt = im->attr("target");
        if (!tgt) {
          err = "instance_material without target";
          return false;
        }
        XNode* em = uri_find(tgt + 1);
        if (!em) {
          err = std::string("invalid material ") + tgt;
          return false;
        }
        mat = parse_material(em);
        has_mat = true;
      }
      if (get_element(e_geom, "mesh")) {
        std::vector<std::vector<size_t>> polys;
        std::vector<V3> verts;
        if (!parse_polymesh(e_geom, polys, verts)) return false;
        for (auto& v : verts) v = xform_point(T, v, true);  // mesh.cpp:28-30
        Mesh m;
        std::vector<std::array<int, 3>> tris;
        if (!build_static_mesh(polys, verts, m, tris, err)) return false;
        if (!has_mat) {  // mesh.cpp:36-37
          mat = Material();
          mat.albedo[0] = mat.albedo[1] = mat.albedo[2] = 1.f;
        }
        const int obj = (int)S.materials.size();
        S.materials.push_back(mat);
        const int mi = (int)S.meshes.size();
        S.meshes.push_back(std::move(m));
        for (auto& t : tris) {
          Prim p;
          p.kind = PT_PRIM_TRIANGLE;
          p.object = obj;
          p.mesh = mi;
          p.v[0] = t[0];
          p.v[1] = t[1];
          p.v[2] = t[2];
          S.prims.push_back(p);
        }
      } else if (get_element(e_geom, "extra")) {
        XNode* tech = technique_cmu462(e_geom);
        XNode* rad = tech ? get_element(tech, "sphere/radius") : nullptr;
        if (!rad) {
          err = "invalid sphere definition";
          return false;
        }
        double radius = atof(rad->text.c_str());
        V3 pos = xform_point(T, V3(0, 0, 0), true);
        double scale = xform_dir0(T, V3(1, 0, 0)).norm();
        if (!has_mat) {  // sphere.cpp:12-16
          mat = Material();
          mat.albedo[0] = mat.albedo[1] = mat.albedo[2] = .5f;
        }
        const int obj = (int)S.materials.size();
        S.materials.push_back(mat);
        Prim p;
        p.kind = PT_PRIM_SPHERE;
        p.object = obj;
        p.centre = pos;
        p.radius = radius * scale;
        S.prims.push_back(p);
      }
    }
    return true;
  }

  bool run(const std::string& text) {
    XmlParser xp(text);
    auto doc = xp.parse(err);
    if (!doc) return false;
    XNode* root = doc->child("COLLADA");
    if (!root) {
      err = "not a COLLADA file";
      return false;
    }
    build_uri(root);
    if (XNode* asset = root->child("asset")) {
      XNode* ua = asset->child("up_axis");
      if (!ua) {
        err = "no up_axis";
        return false;
      }
      std::string upd = ua->text;
      upd.erase(0, upd.find_first_not_of(" \t\r\n"));
      upd.erase(upd.find_last_not_of(" \t\r\n") + 1);
      global = M4::identity();
      if (upd == "X_UP") {
        global(0, 0) = 0;
        global(0, 1) = 1;
        global(1, 0) = 1;
        global(1, 1) = 0;
        global(2, 2) = -1;
        up = V3(1, 0, 0);
      } else if (upd == "Z_UP") {
        global(1, 1) = 0;
        global(1, 2) = 1;
        global(2, 1) = 1;
        global(2, 2) = 0;
        global(0, 0) = -1;
        up = V3(0, 0, 1);
      } else if (upd == "Y_UP") {
        up = V3(0, 1, 0);
      } else {
        err = "invalid up_axis";
        return false;
      }
    }
    XNode* vs = get_element(root, "scene/instance_visual_scene");
    if (!vs) {
      err = "no scene";
      return false;
    }
    for (auto& n : vs->kids)
      if (n->name == "node" && !parse_node(n.get(), global)) return false;

    // camera (cudaRenderer.cu:1595-1599)
    if (cam) {
      V3 look = -c_dir;
      V3 origin = c_pos + V3(0, 0.75, 0);
      V3 left = cross(V3(0.0, 1.0, 0.0), c_dir).unit();
      V3 cup = cross(left, c_dir).unit();
      const V3* vv[4] = {&origin, &look, &left, &cup};
      float* dst[4] = {S.camera.origin, S.camera.look_at, S.camera.left, S.camera.up};
      for (int k = 0; k < 4; ++k) {
        dst[k][0] = (float)vv[k]->x;
        dst[k][1] = (float)vv[k]->y;
        dst[k][2] = (float)vv[k]->z;
      }
      S.have_camera = true;
    }
    // Lights in scene-graph order (application.cpp:370-374 init_light ->
    // DynamicScene::*Light::get_static_light): area (area_light.h:12-24 with
    // the LightInfo defaults), point, directional (directional_light.h:14-19:
    // -(transform * (direction, 1)) -- translation included, as the reference
    // writes it -- then light.cpp:14-16 dirToLight = its negated unit vector),
    // ambient (ambient_light.h -> InfiniteHemisphereLight, light.cpp:27-44).
    // The CUDA path accepts exactly one (cu:1734-1737): `light` is the first
    // area or point light, else the first of the others; with more than one
    // every light is listed (pt_scene_desc.lights, light == lights[0]).
    S.light = pt_light{};
    S.light.type = PT_LIGHT_NONE;
    S.lights.clear();
    // (a spot light is a light instance too: it keeps the default ambient
    // light out, application.cpp:389, though it adds no light itself)
    const bool any_light = !lights.empty();
    for (auto& pl : lights) {
      const M4& T = pl.T;
      pt_light L{};
      if (pl.info.type == 3) {
        V3 position = xform_point(T, V3(0, 0, 0), false);
        V3 direction = xform_point(T, V3(0, 0, -1), false) - position;
        direction = direction / direction.norm();  // Vector3D::normalize: *= 1/norm
        V3 lup(0, 1, 0), ldir(0, 0, -1);
        V3 dim_y = lup;
        V3 dim_x = cross(lup, ldir);
        V3 dx = xform_point(T, dim_x, false) - position;
        V3 dy = xform_point(T, dim_y, false) - position;
        L.type = PT_LIGHT_AREA;
        for (int k = 0; k < 3; ++k) {
          L.radiance[k] = pl.info.spectrum[k];
          L.position[k] = (float)position[k];
          L.direction[k] = (float)direction[k];
          L.dim_x[k] = (float)dx[k];
          L.dim_y[k] = (float)dy[k];
        }
        // area = |dim_x| * |dim_y| in fp32 (cu:1751)
        float ax = L.dim_x[0] * L.dim_x[0] + L.dim_x[1] * L.dim_x[1] + L.dim_x[2] * L.dim_x[2];
        float ay = L.dim_y[0] * L.dim_y[0] + L.dim_y[1] * L.dim_y[1] + L.dim_y[2] * L.dim_y[2];
        L.area = sqrtf(ax) * sqrtf(ay);
      } else if (pl.info.type == 4) {
        V3 position = xform_point(T, V3(0, 0, 0), false);
        L.type = PT_LIGHT_POINT;
        for (int k = 0; k < 3; ++k) {
          L.radiance[k] = pl.info.spectrum[k];
          L.position[k] = (float)position[k];
        }
      } else if (pl.info.type == 2) {
        V3 to_light = xform_point(T, V3(0, 0, -1), false);  // -(-(T (0,0,-1,1)))
        to_light = to_light / to_light.norm();
        L.type = PT_LIGHT_DIRECTIONAL;
        for (int k = 0; k < 3; ++k) {
          L.radiance[k] = pl.info.spectrum[k];
          L.direction[k] = (float)to_light[k];
        }
      } else if (pl.info.type == 1) {
        L.type = PT_LIGHT_HEMISPHERE;
        for (int k = 0; k < 3; ++k) L.radiance[k] = pl.info.spectrum[k];
      } else {
        continue;  // spot lights: a stub in the reference (light.cpp:61-69)
      }
      S.lights.push_back(L);
    }
    // no light instance at all: Application::load adds the default
    // AmbientLight (application.cpp:389-392; LightInfo's spectrum (1, 1, 1),
    // light_info.cpp:11)
    if (!any_light) {
      pt_light L{};
      L.type = PT_LIGHT_HEMISPHERE;
      L.radiance[0] = L.radiance[1] = L.radiance[2] = 1.0f;
      S.lights.push_back(L);
    }
    // `light`: the first area / point light (the CUDA path's), else the first
    for (size_t i = 0; i < S.lights.size(); ++i)
      if (S.lights[i].type == PT_LIGHT_AREA || S.lights[i].type == PT_LIGHT_POINT) {
        std::rotate(S.lights.begin(), S.lights.begin() + i, S.lights.begin() + i + 1);
        break;
      }
    if (!S.lights.empty()) S.light = S.lights[0];
    if (S.lights.size() < 2) S.lights.clear();
    return true;
  }
};
}  // namespace

M4 M4::identity() {
  M4 B;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) B(i, j) = (i == j) ? 1. : 0.;
  return B;
}
M4 M4::operator*(const M4& B) const {
  const M4& A = *this;
  M4 C;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      C(i, j) = 0.;
      for (int k = 0; k < 4; k++) C(i, j) += A(i, k) * B(k, j);
    }
  return C;
}
void M4::mul4(const double x[4], double out[4]) const {
  for (int i = 0; i < 4; ++i) {
    double a = x[0] * e[0][i];
    double b = x[1] * e[1][i];
    double c = x[2] * e[2][i];
    double d = x[3] * e[3][i];
    out[i] = ((a + b) + c) + d;
  }
}

bool load_dae(const std::string& path, Scene& s, std::string& err) {
  std::ifstream in(path, std::ios::binary);
  if (!in.is_open()) {
    err = "could not open " + path;
    return false;
  }
  std::stringstream ss;
  ss << in.rdbuf();
  std::string text = ss.str();
  Loader L(s, err);
  return L.run(text);
}

}  // namespace ptscene
