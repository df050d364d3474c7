// scotty_pt.h -- header-only C++ surface of the reference over the C ABI.
//
// Keeps the class/method names a Scotty3D / CUDA-SCOTTY caller uses so the
// MI355X path drops in behind them:
//   cutracer::CudaRenderer   src/cudaRenderer.h:173-272   -> scotty::CudaRenderer
//   CMU462::Camera::generate_ray   src/camera.h:81          -> scotty::Camera::generate_ray
//   StaticScene::BVHAccel(prims, 32), intersect(ray[, isect])
//                            src/bvh.h:111-149            -> scotty::BVHAccel
//   CMU462::PathTracer set_scene / set_camera / set_frame_size /
//     start_raytracing / is_done / raytrace_tile / raytrace_pixel / save_image,
//     its WorkQueue of 32x32 tiles and worker threads
//                            src/pathtracer.h:51-179, pathtracer.cpp:183-213,
//                            499-558, src/work_queue.h  -> scotty::PathTracerT /
//                                                           scotty::PathTracer
//   the progressive viewer loop  src/display.cpp:99-190 (key handler, renderPicture)
//     + CudaRenderer::renderAccumulate / setViewpoint, cu:1845-1870, 2419-2457
//                                                        -> scotty::Viewer
// Everything is plain C++17 on top of include/pt_api.h; no HIP types here.
// Errors throw scotty::Error carrying the pt_* code and message (the
// reference printf()s and exit()s instead).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "pt_api.h"

namespace scotty {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m + " (pt error " + std::to_string(c) + ")"), code(c) {}
};

struct Vector3D {
  double x = 0, y = 0, z = 0;
  Vector3D() = default;
  Vector3D(double a, double b, double c) : x(a), y(b), z(c) {}
  Vector3D operator+(const Vector3D& b) const { return Vector3D(x + b.x, y + b.y, z + b.z); }
  Vector3D operator-(const Vector3D& b) const { return Vector3D(x - b.x, y - b.y, z - b.z); }
  Vector3D operator*(double s) const { return Vector3D(x * s, y * s, z * s); }
  double norm() const { return std::sqrt(x * x + y * y + z * z); }
  Vector3D unit() const { return *this * (1.0 / norm()); }
};
inline Vector3D operator*(double s, const Vector3D& v) { return v * s; }
inline double dot(const Vector3D& a, const Vector3D& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline Vector3D cross(const Vector3D& a, const Vector3D& b) {
  return Vector3D(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

// CMU462::Ray (src/ray.h): origin, direction, the segment [min_t, max_t]
struct Ray {
  Vector3D o, d;
  double min_t = 0.0, max_t = INFINITY;
  size_t depth = 0;
  Ray() = default;
  Ray(const Vector3D& o_, const Vector3D& d_, int depth_ = 0) : o(o_), d(d_), depth((size_t)depth_) {}
  Ray(const Vector3D& o_, const Vector3D& d_, double maxt, int depth_ = 0)
      : o(o_), d(d_), max_t(maxt), depth((size_t)depth_) {}
  Vector3D at_time(double t) const { return o + d * t; }
};

struct Spectrum {  // CMU462::Spectrum (r, g, b)
  float r = 0, g = 0, b = 0;
  Spectrum() = default;
  Spectrum(float r_, float g_, float b_) : r(r_), g(g_), b(b_) {}
};

// ---- src/bsdf.h: the BSDF kinds the kernels shade (as pt_bsdf records) -------
class BSDF {
 public:
  virtual ~BSDF() = default;
  const pt_bsdf& params() const { return b_; }
  bool is_delta() const {
    return b_.type == PT_BSDF_MIRROR || b_.type == PT_BSDF_GLASS || b_.type == PT_BSDF_REFRACTION;
  }

 protected:
  BSDF(int type, const Spectrum& a) {
    b_.type = type;
    b_.albedo[0] = a.r;
    b_.albedo[1] = a.g;
    b_.albedo[2] = a.b;
  }
  pt_bsdf b_{};
};
struct DiffuseBSDF : BSDF {  // bsdf.h:108
  explicit DiffuseBSDF(const Spectrum& albedo) : BSDF(PT_BSDF_DIFFUSE, albedo) {}
};
struct MirrorBSDF : BSDF {  // bsdf.h:126
  explicit MirrorBSDF(const Spectrum& reflectance) : BSDF(PT_BSDF_MIRROR, reflectance) {}
};
struct GlassBSDF : BSDF {  // bsdf.h:190 (roughness: read only by PT_FLAG_REF_ARITH, pt_api.h pt_bsdf)
  GlassBSDF(const Spectrum& transmittance, const Spectrum& reflectance, float roughness, float ior)
      : BSDF(PT_BSDF_GLASS, reflectance) {
    b_.transmittance[0] = transmittance.r;
    b_.transmittance[1] = transmittance.g;
    b_.transmittance[2] = transmittance.b;
    b_.ior = ior;
    b_.roughness = roughness;
  }
};
struct RefractionBSDF : BSDF {  // bsdf.h:167: glass without reflectance
  RefractionBSDF(const Spectrum& transmittance, float roughness, float ior)
      : BSDF(PT_BSDF_REFRACTION, Spectrum(0.f, 0.f, 0.f)) {
    b_.transmittance[0] = transmittance.r;
    b_.transmittance[1] = transmittance.g;
    b_.transmittance[2] = transmittance.b;
    b_.ior = ior;
    b_.roughness = roughness;
  }
};
struct EmissionBSDF : BSDF {  // bsdf.h:217
  explicit EmissionBSDF(const Spectrum& radiance) : BSDF(PT_BSDF_EMISSION, radiance) {}
};

struct BBox {  // src/bbox.h subset
  Vector3D min{INFINITY, INFINITY, INFINITY}, max{-INFINITY, -INFINITY, -INFINITY};
  BBox() = default;
  BBox(const Vector3D& a, const Vector3D& b) : min(a), max(b) {}
  void expand(const BBox& o) {
    min = Vector3D(std::min(min.x, o.min.x), std::min(min.y, o.min.y), std::min(min.z, o.min.z));
    max = Vector3D(std::max(max.x, o.max.x), std::max(max.y, o.max.y), std::max(max.z, o.max.z));
  }
};

class Primitive;
// CMU462::StaticScene::Intersection (src/intersection.h)
struct Intersection {
  double t = INFINITY;
  const Primitive* primitive = nullptr;  // the primitive hit
  Vector3D n;                            // normal at the hit (see BVHAccel::intersect)
  BSDF* bsdf = nullptr;
  int index = -1;                        // its BVH-sorted index (getSortedPrimitives(); extension)
};

// ---- src/static_scene/primitive.h, object.h, triangle.h, sphere.h -----------
class Primitive {  // primitive.h:15-63 (without the GL draw calls)
 public:
  virtual ~Primitive() = default;
  virtual BBox get_bbox() const = 0;
  virtual bool intersect(const Ray& r) const = 0;
  virtual bool intersect(const Ray& r, Intersection* i) const = 0;
  virtual BSDF* get_bsdf() const = 0;
};

// StaticScene::Mesh: world-space positions and vertex normals, triangles as
// index triples (object.h:15-44; the halfedge conversion is the loader's job).
class Mesh {
 public:
  Mesh(std::vector<Vector3D> positions_, std::vector<Vector3D> normals_, std::vector<size_t> indices_, BSDF* bsdf_)
      : positions(std::move(positions_)), normals(std::move(normals_)), indices(std::move(indices_)), bsdf(bsdf_) {}
  std::vector<Primitive*> get_primitives() const;  // object.cpp:61-70 (caller owns them)
  BSDF* get_bsdf() const { return bsdf; }
  std::vector<Vector3D> positions, normals;
  std::vector<size_t> indices;

 private:
  BSDF* bsdf;
};

class Triangle : public Primitive {
 public:
  Triangle(const Mesh* mesh, size_t v1, size_t v2, size_t v3) : mesh_(mesh), v1_(v1), v2_(v2), v3_(v3) {}
  // triangle.cpp:13-47: the vertices' box padded by 1e-3 on every side
  BBox get_bbox() const override {
    const Vector3D &a = p(v1_), &b = p(v2_), &c = p(v3_);
    const double pad = 1e-3;
    return BBox(Vector3D(std::min({a.x, b.x, c.x}) - pad, std::min({a.y, b.y, c.y}) - pad,
                         std::min({a.z, b.z, c.z}) - pad),
                Vector3D(std::max({a.x, b.x, c.x}) + pad, std::max({a.y, b.y, c.y}) + pad,
                         std::max({a.z, b.z, c.z}) + pad));
  }
  // triangle.cpp:119-209 (fp64 Moller-Trumbore on the host; BVHAccel answers
  // the same question on the GPU with the kernels' test)
  bool intersect(const Ray& r) const override { return intersect(r, nullptr); }
  bool intersect(const Ray& r, Intersection* isect) const override {
    double u, v, t, den;
    barycentric(r, &u, &v, &t, &den);
    if (!(std::fabs(den) <= 1e10) || u < 0 || v < 0 || u + v > 1 || t < r.min_t || t > r.max_t) return false;
    if (isect) {
      isect->t = t;
      isect->primitive = this;
      isect->bsdf = get_bsdf();
      isect->n = shading_normal(r, u, v);
    }
    return true;
  }
  BSDF* get_bsdf() const override { return mesh_->get_bsdf(); }
  void positions(Vector3D& a, Vector3D& b, Vector3D& c) const {
    a = p(v1_);
    b = p(v2_);
    c = p(v3_);
  }
  void normals(Vector3D& a, Vector3D& b, Vector3D& c) const {
    a = mesh_->normals[v1_];
    b = mesh_->normals[v2_];
    c = mesh_->normals[v3_];
  }
  // The normal Triangle::intersect reports for a hit of ray r (triangle.cpp:
  // 195-202): the vertex normals blended with the hit's barycentric weights,
  // oriented toward the side of the ray origin, unit length.
  Vector3D shading_normal(const Ray& r) const {
    double u, v, t, den;
    barycentric(r, &u, &v, &t, &den);
    if (!std::isfinite(u) || !std::isfinite(v)) u = v = 1.0 / 3.0;  // (a ray in the triangle's plane)
    return shading_normal(r, u, v);
  }

 private:
  const Vector3D& p(size_t i) const { return mesh_->positions[i]; }
  // Moller-Trumbore in fp64: barycentric (u, v) of the hit on v2, v3 and its t
  void barycentric(const Ray& r, double* u, double* v, double* t, double* den) const {
    const Vector3D s = r.o - p(v1_), e1 = p(v2_) - p(v1_), e2 = p(v3_) - p(v1_);
    const Vector3D q = cross(e1, r.d), w = cross(s, e2);
    *den = 1.0 / dot(q, e2);
    *u = -dot(w, r.d) * *den;
    *v = dot(q, s) * *den;
    *t = -dot(w, e1) * *den;
  }
  Vector3D shading_normal(const Ray& r, double u, double v) const {
    Vector3D n = mesh_->normals[v2_] * u + mesh_->normals[v3_] * v + mesh_->normals[v1_] * (1 - u - v);
    if (!(dot(r.o - p(v1_), n) > 0)) n = n * -1.0;
    return n.unit();
  }
  const Mesh* mesh_;
  size_t v1_, v2_, v3_;
};

class SphereObject {  // object.h:47-77
 public:
  SphereObject(const Vector3D& o_, double r_, BSDF* bsdf_) : o(o_), r(r_), bsdf(bsdf_) {}
  std::vector<Primitive*> get_primitives() const;  // object.cpp:82-86 (caller owns it)
  BSDF* get_bsdf() const { return bsdf; }
  Vector3D o;
  double r;

 private:
  BSDF* bsdf;
};

class Sphere : public Primitive {  // sphere.h (its intersect is a stub in the reference, sphere.cpp:11-36)
 public:
  Sphere(const SphereObject* object, const Vector3D& o_, double r_) : o(o_), r(r_), r2(r_ * r_), object_(object) {}
  BBox get_bbox() const override { return BBox(o - Vector3D(r, r, r), o + Vector3D(r, r, r)); }
  bool intersect(const Ray& ray) const override { return intersect(ray, nullptr); }
  // nearest root in [min_t, max_t] (d need not be unit length)
  bool intersect(const Ray& ray, Intersection* isect) const override {
    const Vector3D oc = ray.o - o;
    const double a = dot(ray.d, ray.d), b = dot(oc, ray.d), c = dot(oc, oc) - r2;
    const double disc = b * b - a * c;
    if (disc < 0) return false;
    const double sq = std::sqrt(disc);
    double t = (-b - sq) / a;
    if (t < ray.min_t) t = (-b + sq) / a;
    if (t < ray.min_t || t > ray.max_t) return false;
    if (isect) {
      isect->t = t;
      isect->primitive = this;
      isect->bsdf = get_bsdf();
      isect->n = normal(ray.at_time(t));
    }
    return true;
  }
  BSDF* get_bsdf() const override { return object_->get_bsdf(); }
  Vector3D normal(const Vector3D& p) const { return (p - o).unit(); }  // sphere.h: outward
  Vector3D o;
  double r, r2;

 private:
  const SphereObject* object_;
};

inline std::vector<Primitive*> Mesh::get_primitives() const {
  std::vector<Primitive*> out;
  for (size_t i = 0; i + 2 < indices.size(); i += 3) out.push_back(new Triangle(this, indices[i], indices[i + 1], indices[i + 2]));
  return out;
}
inline std::vector<Primitive*> SphereObject::get_primitives() const { return {new Sphere(this, o, r)}; }

class Scene {
 public:
  explicit Scene(const std::string& dae_path) {
    char err[512] = {0};
    int rc = pt_scene_load_dae(dae_path.c_str(), &s_, err, sizeof err);
    if (rc) throw Error(rc, std::string("loadScene: ") + err);
    pt_scene_get_desc(s_, &d_);
  }
  // a flattened scene the caller owns (must outlive this object): e.g. a
  // pt_scene_from_mesh result or a host array scene
  explicit Scene(const pt_scene_desc& d) : d_(d) {}
  // takes ownership of a pt_scene
  explicit Scene(pt_scene* s) : s_(s) { pt_scene_get_desc(s_, &d_); }
  ~Scene() {
    if (s_) pt_scene_free(s_);
  }
  Scene(const Scene&) = delete;
  Scene& operator=(const Scene&) = delete;
  const pt_scene_desc& desc() const { return d_; }
  pt_scene* handle() const { return s_; }

 private:
  pt_scene* s_ = nullptr;
  pt_scene_desc d_{};
};

class Device {
 public:
  explicit Device(int device = 0) {
    int rc = pt_create(&c_, device);
    if (rc) throw Error(rc, "pt_create");
  }
  ~Device() { pt_destroy(c_); }
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;
  pt_ctx* get() const { return c_; }
  void check(int rc, const char* what) const {
    if (rc) throw Error(rc, std::string(what) + ": " + pt_last_error(c_));
  }

 private:
  pt_ctx* c_ = nullptr;
};

// Collada::CameraInfo (fields of view in degrees, clip planes)
struct CameraInfo {
  double hFov = 50.0, vFov = 35.0, nClip = 0.01, fClip = 100.0;
};

// CMU462::Camera (src/camera.h).  One camera model serves both framings:
//  * the reference GPU camera (cu:80-86, set up at cu:1590-1607): origin,
//    lookAt, left, up with a fixed 53.13 degree field of view -- Camera(pt_camera);
//  * the Scotty3D camera: configure() fits the COLLADA fields of view to the
//    screen (camera.cpp:15-33), place() puts it on a sphere around a target
//    (camera.cpp:35-46, compute_position camera.cpp:86-108), and then
//    look_at = -c2w[2], left = c2w[0] * 2 tan(hFov/2), up = -c2w[1] * 2 tan(vFov/2).
// generate_ray(x, y) (camera.h:71-81; its body is a stub in the reference,
// camera.cpp:111-117): (x, y) in [0,1]^2 are normalised sensor coordinates,
// (0.5, 0.5) the centre, y up; the ray starts at the camera position and
// points along (x - 0.5) left - (y - 0.5) up + look_at, normalised -- the
// direction the kernels trace for that sensor point (cu:338-354, where the
// pixel row is y * H and the column x * W).
class Camera {
 public:
  Camera() = default;
  explicit Camera(const pt_camera& c)
      : pos_(v(c.origin)), look_(v(c.look_at)), left_(v(c.left)), up_(v(c.up)) {}
  void configure(const CameraInfo& info, size_t screenW, size_t screenH) {
    const double PI = 3.14159265358979323846;
    auto rad = [&](double d) { return d * (PI / 180); };
    auto deg = [&](double r) { return r * (180 / PI); };
    screenW_ = screenW;
    screenH_ = screenH;
    hFov_ = info.hFov;
    vFov_ = info.vFov;
    const double ar1 = std::tan(rad(hFov_) / 2) / std::tan(rad(vFov_) / 2);
    const double ar = (double)screenW / (double)screenH;
    if (ar1 < ar)
      hFov_ = 2 * deg(std::atan(std::tan(rad(vFov_) / 2) * ar));
    else if (ar1 > ar)
      vFov_ = 2 * deg(std::atan(std::tan(rad(hFov_) / 2) / ar));
    frame();
  }
  void place(const Vector3D& targetPos, double phi, double theta, double r, double minR, double maxR) {
    const double EPS_F = 0.00001f;
    r_ = std::min(std::max(r, minR), maxR);
    phi_ = (std::sin(phi) == 0) ? (phi + EPS_F) : phi;
    theta_ = theta;
    target_ = targetPos;
    double sinPhi = std::sin(phi_);
    if (sinPhi == 0) {
      phi_ += EPS_F;
      sinPhi = std::sin(phi_);
    }
    const Vector3D toCam(r_ * sinPhi * std::sin(theta_), r_ * std::cos(phi_), r_ * sinPhi * std::cos(theta_));
    pos_ = target_ + toCam;
    const Vector3D upVec(0, sinPhi > 0 ? 1 : -1, 0);
    c2w_[0] = cross(upVec, toCam).unit();
    c2w_[1] = cross(toCam, c2w_[0]).unit();
    c2w_[2] = toCam.unit();
    placed_ = true;
    frame();
  }
  Ray generate_ray(double x, double y) const {
    const double kx = x - 0.5, ky = -(y - 0.5);
    const Vector3D d = left_ * kx + up_ * ky + look_;
    return Ray(pos_, d.unit());
  }
  // the pt_camera the kernels use (pt_set_camera)
  pt_camera params() const {
    pt_camera c{};
    f(c.origin, pos_);
    f(c.look_at, look_);
    f(c.left, left_);
    f(c.up, up_);
    return c;
  }
  Vector3D position() const { return pos_; }
  Vector3D view_point() const { return target_; }
  double h_fov() const { return hFov_; }
  double v_fov() const { return vFov_; }

 private:
  static Vector3D v(const float* p) { return Vector3D(p[0], p[1], p[2]); }
  static void f(float* d, const Vector3D& s) {
    d[0] = (float)s.x;
    d[1] = (float)s.y;
    d[2] = (float)s.z;
  }
  void frame() {  // the placed Scotty3D camera as look_at / left / up
    if (!placed_) return;
    const double PI = 3.14159265358979323846;
    const double sx = 2 * std::tan(hFov_ * PI / 180 / 2), sy = 2 * std::tan(vFov_ * PI / 180 / 2);
    look_ = c2w_[2] * -1.0;
    left_ = c2w_[0] * sx;
    up_ = c2w_[1] * -sy;
  }
  Vector3D pos_, look_{0, 0, -1}, left_{1, 0, 0}, up_{0, -1, 0};
  Vector3D target_, c2w_[3];
  double hFov_ = 53.13010235415598, vFov_ = 53.13010235415598, r_ = 1, phi_ = 0, theta_ = 0;
  size_t screenW_ = 0, screenH_ = 0;
  bool placed_ = false;
};

// StaticScene::BVHAccel (bvh.h:99-149) on the GPU.  The constructor takes the
// Scotty3D primitives (Triangles of Meshes, Spheres of SphereObjects), builds
// the reference's BVH over them (bvh.cpp:48-365: binned SAH, leaves of at
// most max_leaf_size, 4-wide compaction; pt_scene_from_mesh_ex) and uploads
// it to GPU `device`; the primitives must outlive the accelerator (bvh.h:105).
// intersect(ray, isect) is the closest hit with min_t <= t <= max_t (both
// inclusive, as Triangle::intersect tests them, triangle.cpp:189), found by
// the breadth-first traversal (pt_intersect) in fp32: the ray's origin and
// direction are rounded to fp32, min_t up and max_t down to the nearest fp32,
// so a reported t (an fp32 value) lies in the double interval exactly.  The
// Intersection carries the primitive, its BSDF, the fp32 t and the normal of
// Triangle::intersect (interpolated vertex normals facing the ray origin's
// side, triangle.cpp:195-202) or the outward sphere normal (sphere.h).
// Single rays work, but each call is a GPU launch: intersect(std::vector<Ray>)
// is the fast form.
class BVHAccel {
 public:
  BVHAccel(const std::vector<Primitive*>& primitives, size_t max_leaf_size = 32, int device = 0) : dev_(device) {
    if (max_leaf_size == 0 || max_leaf_size > (1u << 20)) throw Error(PT_E_INVALID, "BVHAccel: max_leaf_size");
    std::vector<const Triangle*> tris;
    std::vector<const Sphere*> sphs;
    for (Primitive* p : primitives) {
      if (auto* t = dynamic_cast<const Triangle*>(p))
        tris.push_back(t);
      else if (auto* s = dynamic_cast<const Sphere*>(p))
        sphs.push_back(s);
      else
        throw Error(PT_E_UNSUPPORTED, "BVHAccel: primitives must be Triangles or Spheres");
    }
    if (tris.empty() && sphs.empty()) throw Error(PT_E_INVALID, "BVHAccel: no primitives");
    has_spheres_ = !sphs.empty();
    std::vector<float> pos, nrm, sph;
    std::vector<int32_t> tb, sb;
    std::vector<pt_bsdf> bsdfs;
    std::vector<const BSDF*> seen;
    auto bsdf_id = [&](const BSDF* b) -> int32_t {
      for (size_t i = 0; i < seen.size(); ++i)
        if (seen[i] == b) return (int32_t)i;
      seen.push_back(b);
      pt_bsdf d{};
      if (b) d = b->params();
      else d.albedo[0] = d.albedo[1] = d.albedo[2] = 0.5f;  // (no material: grey diffuse)
      bsdfs.push_back(d);
      return (int32_t)seen.size() - 1;
    };
    auto put = [](std::vector<float>& v, const Vector3D& a) {
      v.push_back((float)a.x);
      v.push_back((float)a.y);
      v.push_back((float)a.z);
    };
    for (const Triangle* t : tris) {
      Vector3D a, b, c;
      t->positions(a, b, c);
      put(pos, a);
      put(pos, b);
      put(pos, c);
      t->normals(a, b, c);
      put(nrm, a);
      put(nrm, b);
      put(nrm, c);
      tb.push_back(bsdf_id(t->get_bsdf()));
    }
    for (const Sphere* s : sphs) {
      put(sph, s->o);
      sph.push_back((float)s->r);
      sb.push_back(bsdf_id(s->get_bsdf()));
    }
    pt_mesh_desc m{};
    m.n_tris = (int32_t)tris.size();
    m.positions = pos.data();
    m.normals = nrm.data();
    m.tri_bsdf = tb.data();
    m.n_spheres = (int32_t)sphs.size();
    m.spheres = sph.empty() ? nullptr : sph.data();
    m.sphere_bsdf = sb.empty() ? nullptr : sb.data();
    m.n_bsdfs = (int32_t)bsdfs.size();
    m.bsdfs = bsdfs.data();
    pt_scene* ps = nullptr;
    int rc = pt_scene_from_mesh_ex(&m, (int32_t)max_leaf_size, &ps);
    if (rc) throw Error(rc, "BVHAccel: pt_scene_from_mesh_ex");
    scene_ = std::make_unique<Scene>(ps);
    const pt_scene_desc& d = scene_->desc();
    std::vector<int32_t> s2i((size_t)d.n_prims);
    pt_scene_sorted_to_input(ps, s2i.data(), d.n_prims);
    sorted_.resize((size_t)d.n_prims);
    for (int32_t i = 0; i < d.n_prims; ++i) {
      const int32_t k = s2i[(size_t)i];
      sorted_[(size_t)i] = k < m.n_tris ? (const Primitive*)tris[(size_t)k] : (const Primitive*)sphs[(size_t)(k - m.n_tris)];
    }
    dev_.check(pt_load_scene(dev_.get(), &d), "pt_load_scene");
  }
  // getSortedPrimitives(), bvh.cpp:384: the primitives in BVH leaf order
  const std::vector<const Primitive*>& sorted_primitives() const { return sorted_; }
  BBox get_bbox() const {
    BBox b;
    for (const Primitive* p : sorted_) b.expand(p->get_bbox());
    return b;
  }
  // a batch of closest-hit queries (one traversal pass on the GPU): out[i]
  // is rays[i]'s Intersection, primitive == nullptr for a miss
  //
  // Directions need not be unit length (Scotty3D's shadow rays run o + t (light
  // - o) over [eps, 1]).  The triangle test's t is the parametric t for any |d|,
  // so triangle-only scenes pass the ray as given; the kernels' sphere test
  // assumes a unit d (trace.hip sphere_test), so with spheres in the scene a
  // non-unit ray is traced as (o, d / |d|) over [min_t |d|, max_t |d|] and its
  // t scaled back by 1 / |d|.
  std::vector<Intersection> intersect(const std::vector<Ray>& rays) const {
    std::vector<float> r(rays.size() * 8);
    std::vector<double> scale(rays.size(), 1.0);
    for (size_t i = 0; i < rays.size(); ++i) {
      float* p = &r[i * 8];
      Vector3D d = rays[i].d;
      double lo = rays[i].min_t, hi = rays[i].max_t;
      if (has_spheres_) {
        const double l2 = dot(d, d);
        if (std::fabs(l2 - 1.0) > 1e-6 && l2 > 0.0) {
          const double len = std::sqrt(l2);
          d = d * (1.0 / len);
          lo *= len;
          hi *= len;
          scale[i] = len;
        }
      }
      p[0] = (float)rays[i].o.x;
      p[1] = (float)rays[i].o.y;
      p[2] = (float)rays[i].o.z;
      p[3] = round_down(hi);
      p[4] = (float)d.x;
      p[5] = (float)d.y;
      p[6] = (float)d.z;
      p[7] = round_up(lo);
    }
    std::vector<uint64_t> h(rays.size());
    dev_.check(pt_intersect(dev_.get(), r.data(), (int32_t)rays.size(), h.data()), "pt_intersect");
    std::vector<Intersection> out(rays.size());
    for (size_t i = 0; i < rays.size(); ++i) {
      if (h[i] == PT_HIT_NONE) continue;
      const uint32_t tb = (uint32_t)(h[i] >> 32);
      float t;
      memcpy(&t, &tb, 4);
      Intersection& is = out[i];
      is.index = (int)(uint32_t)h[i];
      is.primitive = sorted_[(size_t)is.index];
      is.t = scale[i] == 1.0 ? (double)t : (double)t / scale[i];
      is.bsdf = is.primitive->get_bsdf();
      if (auto* tri = dynamic_cast<const Triangle*>(is.primitive))
        is.n = tri->shading_normal(rays[i]);
      else
        is.n = static_cast<const Sphere*>(is.primitive)->normal(rays[i].at_time(is.t));
    }
    return out;
  }
  bool intersect(const Ray& r, Intersection* isect) const {
    Intersection i = intersect(std::vector<Ray>{r})[0];
    if (!i.primitive) return false;
    if (isect) *isect = i;
    return true;
  }
  bool intersect(const Ray& r) const { return intersect(r, nullptr); }
  const pt_scene_desc& desc() const { return scene_->desc(); }
  Device& device() { return dev_; }

 private:
  bool has_spheres_ = false;
  // the fp32 interval [round_up(min_t), round_down(max_t)] holds exactly the
  // fp32 values of the double interval [min_t, max_t]
  static float round_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -INFINITY);
    return f;
  }
  static float round_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, INFINITY);
    return f;
  }
  mutable Device dev_;
  std::unique_ptr<Scene> scene_;
  std::vector<const Primitive*> sorted_;
};

struct Image {  // src/cuda_image.h: float RGBA, rows bottom-up
  int width = 0, height = 0;
  std::vector<float> data;
};

// cutracer::CudaRenderer with the reference's member functions.
class CudaRenderer {
 public:
  explicit CudaRenderer(int device = 0) : dev_(device) {}
  void allocOutputImage(int w, int h) {  // cu:2119
    image_.width = w;
    image_.height = h;
    image_.data.assign((size_t)w * h * 4, 0.f);
  }
  void loadScene(const std::string& path) {  // cu:1679
    scene_ = std::make_unique<Scene>(path);
    camera_ = Camera(scene_->desc().camera);
  }
  void loadScene(const pt_scene_desc& desc) {  // an already flattened scene
    scene_ = std::make_unique<Scene>(desc);
    camera_ = Camera(desc.camera);
  }
  void setup() { dev_.check(pt_load_scene(dev_.get(), &scene_->desc()), "pt_load_scene"); }  // cu:1872
  // one progressive frame of spp samples (renderAccumulate, cu:2419-2457)
  void render(int spp = 2, int max_bounces = 2, uint32_t flags = 0) {
    pt_render_params p{};
    p.width = image_.width;
    p.height = image_.height;
    p.spp = spp;
    p.max_bounces = max_bounces;
    p.seed = 15618;
    p.sample_offset = samples_;
    p.tile_size = 32;
    p.nranks = 1;
    p.flags = flags;
    dev_.check(pt_render(dev_.get(), &p), "pt_render");
    samples_ += spp;
  }
  // cu:1539-1569: the median-filtered frame below 32 accumulated samples
  // (POST_PROCESS_THRESHOLD), the accumulated frame afterwards
  const Image* getImage() {
    dev_.check(pt_get_display_image(dev_.get(), image_.data.data(), image_.data.size()), "pt_get_display_image");
    return &image_;
  }
  const Image* getAccumulatedImage() {
    dev_.check(pt_get_image(dev_.get(), image_.data.data(), image_.data.size()), "pt_get_image");
    return &image_;
  }
  // cu:1845-1870: new origin and look-at (float, as v2f3), left/up kept,
  // accumulation cleared
  void setViewpoint(const Vector3D& origin, const Vector3D& lookAt) {
    pt_camera c = camera_.params();
    c.origin[0] = (float)origin.x;
    c.origin[1] = (float)origin.y;
    c.origin[2] = (float)origin.z;
    c.look_at[0] = (float)lookAt.x;
    c.look_at[1] = (float)lookAt.y;
    c.look_at[2] = (float)lookAt.z;
    camera_ = Camera(c);
    dev_.check(pt_set_camera(dev_.get(), &c), "pt_set_camera");
    samples_ = 0;
  }
  void clearImage() {  // cu:2131
    dev_.check(pt_clear(dev_.get()), "pt_clear");
    samples_ = 0;
  }
  Device& device() { return dev_; }
  const Camera& camera() const { return camera_; }

 private:
  Device dev_;
  std::unique_ptr<Scene> scene_;
  Camera camera_;
  Image image_;
  int samples_ = 0;
};

// ---- CMU462::PathTracer surface (pathtracer.h:51-257, pathtracer.cpp:183-213,
// 499-558) ---------------------------------------------------------------------
// The structure of the Scotty3D renderer is kept: start_raytracing() fills a
// work queue with imageTileSize x imageTileSize tiles (row of tiles by row,
// pathtracer.cpp:195-205) and starts numWorkerThreads std::threads running
// worker_thread(), which pull tiles FIFO (work_queue.h) and call raytrace_tile
// -> raytrace_pixel(x, y) for every pixel, writing the sample buffer.  The
// per-pixel estimate comes from an Estimator:
//   * GpuEstimator (the product path): the whole frame is traced on the GPU
//     through the C ABI when raytracing starts (one pt_render: the reference's
//     CudaRenderer path); raytrace_pixel reads the pixel of that frame;
//   * any type with begin(w, h, spp, max_depth, flags) and
//     pixel(x, y, float rgba[4]) (e.g. the CPU oracle's estimator that times
//     the CPU baseline and makes the config-1 golden, oracle/scotty_cpu.cpp).
// Pixel (x, y) is column x of row y, rows counted bottom-up (the frame
// layout of pt_api.h; save_image flips rows like pathtracer.cpp:584-586).

struct WorkItem {  // src/work_queue.h / pathtracer.h WorkItem
  size_t tile_x = 0, tile_y = 0, tile_w = 0, tile_h = 0;
};
class WorkQueue {
 public:
  void put_work(const WorkItem& w) {
    std::lock_guard<std::mutex> g(m_);
    q_.push_back(w);
  }
  bool try_get_work(WorkItem* out) {
    std::lock_guard<std::mutex> g(m_);
    if (next_ >= q_.size()) return false;
    *out = q_[next_++];
    return true;
  }
  void clear() {
    std::lock_guard<std::mutex> g(m_);
    q_.clear();
    next_ = 0;
  }

 private:
  std::mutex m_;
  std::vector<WorkItem> q_;
  size_t next_ = 0;
};

// GPU estimator: a scotty::CudaRenderer on one device.
class GpuEstimator {
 public:
  explicit GpuEstimator(int device = 0) : r_(device) {}
  void set_scene(const std::string& dae_path) {
    r_.loadScene(dae_path);
    r_.setup();
  }
  void set_scene(const pt_scene_desc& desc) {
    r_.loadScene(desc);
    r_.setup();
  }
  void begin(size_t w, size_t h, size_t spp, size_t max_depth, uint32_t flags) {
    r_.allocOutputImage((int)w, (int)h);
    r_.clearImage();
    r_.render((int)spp, (int)max_depth, flags);
    img_ = r_.getAccumulatedImage();
  }
  void pixel(size_t x, size_t y, float rgba[4]) const {
    const float* p = &img_->data[((size_t)y * img_->width + x) * 4];
    for (int k = 0; k < 4; ++k) rgba[k] = p[k];
  }
  CudaRenderer& renderer() { return r_; }

 private:
  CudaRenderer r_;
  const Image* img_ = nullptr;
};

// GPU estimator over several GPUs of one process (pt_group):
// the frame's 32x32 tiles are dealt round-robin to the devices, each renders
// its share on its own host thread, and the sums are gathered into
// devices[0] (RCCL over xGMI when the devices are distinct, pt_api.h).  The
// reference renders on one device only (cu:1874-1897).
class GroupEstimator {
 public:
  explicit GroupEstimator(const std::vector<int>& devices, int gather = PT_GATHER_AUTO) {
    std::vector<int32_t> d(devices.begin(), devices.end());
    int rc = pt_group_create(&g_, d.data(), (int32_t)d.size(), gather);
    if (rc) throw Error(rc, "pt_group_create");
  }
  ~GroupEstimator() { pt_group_destroy(g_); }
  GroupEstimator(const GroupEstimator&) = delete;
  GroupEstimator& operator=(const GroupEstimator&) = delete;
  void set_scene(const std::string& dae_path) {
    scene_ = std::make_unique<Scene>(dae_path);
    check(pt_group_load_scene(g_, &scene_->desc()), "pt_group_load_scene");
  }
  void set_scene(const pt_scene_desc& desc) {
    scene_ = std::make_unique<Scene>(desc);
    check(pt_group_load_scene(g_, &scene_->desc()), "pt_group_load_scene");
  }
  void begin(size_t w, size_t h, size_t spp, size_t max_depth, uint32_t flags) {
    check(pt_group_clear(g_), "pt_group_clear");
    pt_render_params p{};
    p.width = (int32_t)w;
    p.height = (int32_t)h;
    p.spp = (int32_t)spp;
    p.max_bounces = (int32_t)max_depth;
    p.seed = 15618;
    p.tile_size = 32;
    p.nranks = 1;
    p.flags = flags;
    check(pt_group_render(g_, &p), "pt_group_render");
    img_.width = (int)w;
    img_.height = (int)h;
    img_.data.resize(w * h * 4);
    check(pt_group_get_image(g_, img_.data.data(), img_.data.size()), "pt_group_get_image");
  }
  void pixel(size_t x, size_t y, float rgba[4]) const {
    const float* p = &img_.data[((size_t)y * img_.width + x) * 4];
    for (int k = 0; k < 4; ++k) rgba[k] = p[k];
  }
  pt_group* group() const { return g_; }
  int gather_kind() const {
    int32_t k = 0;
    pt_group_gather_kind(g_, &k);
    return k;
  }

 private:
  void check(int rc, const char* what) const {
    if (rc) throw Error(rc, std::string(what) + ": " + pt_group_last_error(g_));
  }
  pt_group* g_ = nullptr;
  std::unique_ptr<Scene> scene_;
  Image img_;
};

template <class Estimator>
class PathTracerT {
 public:
  enum State { INIT, READY, RENDERING, DONE };
  // (ns_aa, max_ray_depth, ns_area_light, ns_diff, ns_glsy, ns_refr,
  // num_threads) as pathtracer.h:57-60; num_threads 0 = hardware_concurrency
  PathTracerT(Estimator& est, size_t ns_aa = 1, size_t max_ray_depth = 4, size_t /*ns_area_light*/ = 1,
              size_t /*ns_diff*/ = 1, size_t /*ns_glsy*/ = 1, size_t /*ns_refr*/ = 1, size_t num_threads = 0)
      : est_(est), ns_aa_(ns_aa), max_depth_(max_ray_depth) {
    num_threads_ = num_threads ? num_threads : std::max(1u, std::thread::hardware_concurrency());
  }
  ~PathTracerT() { join(); }
  PathTracerT(const PathTracerT&) = delete;
  PathTracerT& operator=(const PathTracerT&) = delete;

  void set_frame_size(size_t w, size_t h) {
    w_ = w;
    h_ = h;
    buf_.assign(w * h * 4, 0.0f);
    state_ = READY;
  }
  void set_flags(uint32_t flags) { flags_ = flags; }  // pt_render_params.flags (PT_FLAG_*)
  size_t num_worker_threads() const { return num_threads_; }

  void start_raytracing() {  // pathtracer.cpp:183-213
    if (state_ != READY) throw Error(PT_E_INVALID, "start_raytracing: set_frame_size first");
    join();
    state_ = RENDERING;
    work_.clear();
    std::fill(buf_.begin(), buf_.end(), 0.0f);
    est_.begin(w_, h_, ns_aa_, max_depth_, flags_);
    for (size_t y = 0; y < h_; y += tile_)
      for (size_t x = 0; x < w_; x += tile_) work_.put_work(WorkItem{x, y, tile_, tile_});
    done_ = 0;
    for (size_t i = 0; i < num_threads_; ++i) threads_.emplace_back(&PathTracerT::worker_thread, this);
  }
  // blocks until every worker is done (the reference polls is_done from its
  // GUI loop; here the caller waits)
  bool is_done() {
    join();
    return state_ == DONE;
  }
  void raytrace_tile(size_t tx, size_t ty, size_t tw, size_t th) {  // pathtracer.cpp:510-535
    const size_t xe = std::min(tx + tw, w_), ye = std::min(ty + th, h_);
    for (size_t y = ty; y < ye; ++y)
      for (size_t x = tx; x < xe; ++x) raytrace_pixel(x, y, &buf_[(y * w_ + x) * 4]);
  }
  void raytrace_pixel(size_t x, size_t y, float rgba[4]) { est_.pixel(x, y, rgba); }  // pathtracer.cpp:499-508
  Vector3D raytrace_pixel(size_t x, size_t y) {
    float p[4];
    raytrace_pixel(x, y, p);
    return Vector3D(p[0], p[1], p[2]);
  }
  // the frame of the last start_raytracing(): RGBA floats, rows bottom-up
  const std::vector<float>& frame() {
    if (!is_done()) throw Error(PT_E_INVALID, "frame before start_raytracing");
    return buf_;
  }
  Vector3D pixel(size_t x, size_t y) {
    const float* p = &frame()[(y * w_ + x) * 4];
    return Vector3D(p[0], p[1], p[2]);
  }
  // pathtracer.cpp:577-591 writes a tonemapped PNG; ".pfm" keeps the floats
  void save_image(const std::string& filename) {
    const std::vector<float>& f = frame();
    const bool pfm = filename.size() >= 4 && filename.compare(filename.size() - 4, 4, ".pfm") == 0;
    int rc;
    if (pfm) {
      rc = pt_write_pfm(filename.c_str(), f.data(), (int32_t)w_, (int32_t)h_);
    } else {
      std::vector<uint8_t> rgba8(w_ * h_ * 4);
      rc = pt_tonemap(f.data(), (int32_t)w_, (int32_t)h_, 2.2f, 1.0f, rgba8.data());
      if (!rc) rc = pt_write_png(filename.c_str(), rgba8.data(), (int32_t)w_, (int32_t)h_);
    }
    if (rc) throw Error(rc, "save_image: cannot write " + filename);
  }
  Estimator& estimator() { return est_; }

 private:
  void worker_thread() {  // pathtracer.cpp:537-558
    WorkItem w;
    while (work_.try_get_work(&w)) raytrace_tile(w.tile_x, w.tile_y, w.tile_w, w.tile_h);
    std::lock_guard<std::mutex> g(m_);
    if (++done_ == num_threads_) state_ = DONE;
  }
  void join() {
    for (auto& t : threads_)
      if (t.joinable()) t.join();
    threads_.clear();
  }

  Estimator& est_;
  size_t ns_aa_, max_depth_, num_threads_;
  size_t tile_ = 32;  // imageTileSize, pathtracer.cpp:55
  size_t w_ = 0, h_ = 0;
  uint32_t flags_ = 0;
  std::vector<float> buf_;
  WorkQueue work_;
  std::vector<std::thread> threads_;
  std::mutex m_;
  size_t done_ = 0;
  State state_ = INIT;
};

// The GPU-backed Scotty3D PathTracer (the drop-in): owns its GpuEstimator.
class PathTracer : private GpuEstimator, public PathTracerT<GpuEstimator> {
 public:
  PathTracer(size_t ns_aa = 1, size_t max_ray_depth = 4, size_t ns_area_light = 1, size_t ns_diff = 1,
             size_t ns_glsy = 1, size_t ns_refr = 1, size_t num_threads = 1, int device = 0)
      : GpuEstimator(device),
        PathTracerT<GpuEstimator>(*static_cast<GpuEstimator*>(this), ns_aa, max_ray_depth, ns_area_light, ns_diff,
                                  ns_glsy, ns_refr, num_threads) {}
  void set_scene(const std::string& dae_path) { GpuEstimator::set_scene(dae_path); }
  void set_scene(const pt_scene_desc& desc) { GpuEstimator::set_scene(desc); }
  void set_camera(const Camera&) {}  // the scene's camera is used (cu:1590-1607)
  CudaRenderer& renderer() { return GpuEstimator::renderer(); }
};

// The Scotty3D PathTracer over several GPUs of one process (pt_group).
class MultiGpuPathTracer : private GroupEstimator, public PathTracerT<GroupEstimator> {
 public:
  MultiGpuPathTracer(const std::vector<int>& devices, size_t ns_aa = 1, size_t max_ray_depth = 4,
                     size_t num_threads = 1, int gather = PT_GATHER_AUTO)
      : GroupEstimator(devices, gather),
        PathTracerT<GroupEstimator>(*static_cast<GroupEstimator*>(this), ns_aa, max_ray_depth, 1, 1, 1, 1,
                                    num_threads) {}
  void set_scene(const std::string& dae_path) { GroupEstimator::set_scene(dae_path); }
  void set_scene(const pt_scene_desc& desc) { GroupEstimator::set_scene(desc); }
  int gather_kind() const { return GroupEstimator::gather_kind(); }
  pt_group* group() const { return GroupEstimator::group(); }
};

// ---- the progressive viewer (display.cpp:99-190 without the GLUT window) -----
// Each displayed frame is renderPicture(): one more renderAccumulate of
// samples_per_frame samples on top of the accumulation (sample indices
// continue: sample_offset), then the display image (median filtered below 32
// accumulated samples, cu:1539-1569).  handleKeyPress moves the camera like
// the reference's w/a/s/d keys (origin += (0, 0, -+0.01) / (-+0.01, 0, 0) in
// double, then setViewpoint: the accumulation restarts); p toggles the pause
// flag and + sets the update flag, as display.cpp:104-116 does -- but, as in
// the reference, no frame reads them: renderPicture (display.cpp:145-174)
// renders whatever their state, so p changes no pixel.  A GUI would call these
// from its event loop; the headless loop drives them from a key script
// (ptrender --viewer).
class Viewer {
 public:
  Viewer(CudaRenderer& r, int samples_per_frame = 2, int max_bounces = 2, uint32_t flags = 0)
      : r_(r), spf_(samples_per_frame), bounces_(max_bounces), flags_(flags) {
    const pt_camera& c = r_.camera().params();
    origin_ = Vector3D(c.origin[0], c.origin[1], c.origin[2]);
    look_at_ = Vector3D(c.look_at[0], c.look_at[1], c.look_at[2]);
  }
  // display.cpp:99-139 handleKeyPress (q/Q is the caller's to handle)
  void handleKeyPress(char key) {
    switch (key) {
      case '=':
      case '+':
        update_ = true;
        break;
      case 'p':
      case 'P':
        paused_ = !paused_;
        if (!paused_) update_ = true;
        break;
      case 'w':
      case 'W':
        move(0, 0, -0.01);
        break;
      case 's':
      case 'S':
        move(0, 0, 0.01);
        break;
      case 'a':
      case 'A':
        move(-0.01, 0, 0);
        break;
      case 'd':
      case 'D':
        move(0.01, 0, 0);
        break;
      default:
        break;
    }
  }
  // display.cpp:145-190 renderPicture: returns the frame to display
  const Image* renderPicture() {
    if (paused_) update_ = false;  // display.cpp:163-164 (updateSim is read nowhere)
    r_.render(spf_, bounces_, flags_);
    ++frames_;
    return r_.getImage();
  }
  bool paused() const { return paused_; }
  bool update_requested() const { return update_; }
  int frames() const { return frames_; }
  const Vector3D& origin() const { return origin_; }

 private:
  void move(double dx, double dy, double dz) {
    origin_ = Vector3D(origin_.x + dx, origin_.y + dy, origin_.z + dz);
    r_.setViewpoint(origin_, look_at_);
  }
  CudaRenderer& r_;
  int spf_, bounces_;
  uint32_t flags_;
  Vector3D origin_, look_at_;
  bool paused_ = false, update_ = true;
  int frames_ = 0;
};

}  // namespace scotty
