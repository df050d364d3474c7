// pt_scene_* entry points of pt_api.h: the host-side input adapter that
// CudaRenderer::loadScene implements inline (src/cudaRenderer.cu:1679-1842).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>

#include "scene_internal.h"

using ptscene::Scene;

// Leaf size of the host SAH build: the reference's 32 (BVHAccel(prims, 32));
// PT_MAX_LEAF overrides it for experiments (hits do not depend on the tree).
static size_t host_max_leaf() {
  const char* e = getenv("PT_MAX_LEAF");
  const long v = e ? atol(e) : 0;
  return v > 0 ? (size_t)v : 32;
}

namespace ptscene {

// pt_mesh_desc -> input-order Scene (prims, meshes, materials, light, camera)
int scene_from_mesh(const pt_mesh_desc* md, Scene& S) {
  if (!md || md->n_tris < 0 || md->n_spheres < 0 || md->n_tris + md->n_spheres <= 0 || md->n_bsdfs <= 0 ||
      !md->bsdfs || (md->n_tris > 0 && !md->positions) || (md->n_spheres > 0 && !md->spheres))
    return PT_E_INVALID;
  for (int32_t t = 0; t < md->n_tris; ++t)
    if (md->tri_bsdf && (md->tri_bsdf[t] < 0 || md->tri_bsdf[t] >= md->n_bsdfs)) return PT_E_INVALID;
  for (int32_t t = 0; t < md->n_spheres; ++t)
    if (md->sphere_bsdf && (md->sphere_bsdf[t] < 0 || md->sphere_bsdf[t] >= md->n_bsdfs)) return PT_E_INVALID;
  ptscene::Mesh m;
  for (int32_t t = 0; t < md->n_tris; ++t) {
    const float* q = md->positions + (size_t)t * 9;
    ptscene::V3 p[3];
    for (int k = 0; k < 3; ++k) p[k] = ptscene::V3(q[k * 3 + 0], q[k * 3 + 1], q[k * 3 + 2]);
    ptscene::V3 fn = ptscene::cross(p[1] - p[0], p[2] - p[0]);
    const double len = fn.norm();
    fn = len > 0 ? fn / len : ptscene::V3(0, 0, 1);
    ptscene::Prim pr;
    pr.kind = PT_PRIM_TRIANGLE;
    pr.object = md->tri_bsdf ? md->tri_bsdf[t] : 0;
    pr.mesh = 0;
    for (int k = 0; k < 3; ++k) {
      pr.v[k] = (int)m.positions.size();
      m.positions.push_back(p[k]);
      if (md->normals) {
        const float* n = md->normals + (size_t)t * 9 + k * 3;
        m.normals.push_back(ptscene::V3(n[0], n[1], n[2]));
      } else {
        m.normals.push_back(fn);
      }
    }
    S.prims.push_back(pr);
  }
  S.meshes.push_back(std::move(m));
  for (int32_t t = 0; t < md->n_spheres; ++t) {
    const float* q = md->spheres + (size_t)t * 4;
    ptscene::Prim pr;
    pr.kind = PT_PRIM_SPHERE;
    pr.object = md->sphere_bsdf ? md->sphere_bsdf[t] : 0;
    pr.centre = ptscene::V3(q[0], q[1], q[2]);
    pr.radius = q[3];
    S.prims.push_back(pr);
  }
  for (int32_t b = 0; b < md->n_bsdfs; ++b) {
    ptscene::Material mat;
    mat.type = md->bsdfs[b].type;
    for (int k = 0; k < 3; ++k) {
      mat.albedo[k] = md->bsdfs[b].albedo[k];
      mat.trans[k] = md->bsdfs[b].transmittance[k];
    }
    mat.ior = md->bsdfs[b].ior;
    mat.roughness = md->bsdfs[b].roughness;
    S.materials.push_back(mat);
  }
  if (md->light) S.light = *md->light;
  if (md->camera) {
    S.camera = *md->camera;
    S.have_camera = true;
  }
  return PT_OK;
}

}  // namespace ptscene

extern "C" {

int pt_scene_load_dae(const char* path, pt_scene** out, char* errbuf, size_t errbuf_len) {
  if (!out || !path) return PT_E_INVALID;
  *out = nullptr;
  auto* sc = new pt_scene();
  std::string err;
  bool ok = false;
  try {
    ok = ptscene::load_dae(path, sc->s, err);
    if (ok && sc->s.prims.empty()) {
      err = "scene has no primitives";
      ok = false;
    }
    if (ok) ptscene::build_bvh_and_flatten(sc->s, host_max_leaf());
  } catch (const std::exception& e) {
    err = e.what();
    ok = false;
  }
  if (!ok) {
    if (errbuf && errbuf_len) {
      strncpy(errbuf, err.c_str(), errbuf_len - 1);
      errbuf[errbuf_len - 1] = 0;
    }
    delete sc;
    return PT_E_IO;
  }
  *out = sc;
  return PT_OK;
}

int pt_scene_from_triangles(const float* positions, int32_t n_tris, const pt_bsdf* bsdf0,
                            const pt_light* light, const pt_camera* camera, pt_scene** out) {
  if (!out || !positions || n_tris <= 0) return PT_E_INVALID;
  auto* sc = new pt_scene();
  Scene& S = sc->s;
  ptscene::Mesh m;
  for (int32_t t = 0; t < n_tris; ++t) {
    ptscene::V3 p[3];
    for (int k = 0; k < 3; ++k)
      p[k] = ptscene::V3(positions[t * 9 + k * 3 + 0], positions[t * 9 + k * 3 + 1],
                         positions[t * 9 + k * 3 + 2]);
    ptscene::V3 n = ptscene::cross(p[1] - p[0], p[2] - p[0]);
    double len = n.norm();
    n = len > 0 ? n / len : ptscene::V3(0, 0, 1);
    ptscene::Prim pr;
    pr.kind = PT_PRIM_TRIANGLE;
    pr.object = 0;
    pr.mesh = 0;
    for (int k = 0; k < 3; ++k) {
      pr.v[k] = (int)m.positions.size();
      m.positions.push_back(p[k]);
      m.normals.push_back(n);
    }
    S.prims.push_back(pr);
  }
  S.meshes.push_back(std::move(m));
  ptscene::Material mat;
  if (bsdf0) {
    mat.type = bsdf0->type;
    for (int k = 0; k < 3; ++k) {
      mat.albedo[k] = bsdf0->albedo[k];
      mat.trans[k] = bsdf0->transmittance[k];
    }
    mat.ior = bsdf0->ior;
    mat.roughness = bsdf0->roughness;
  } else {
    mat.albedo[0] = mat.albedo[1] = mat.albedo[2] = 0.5f;
  }
  S.materials.push_back(mat);
  if (light) S.light = *light;
  if (camera) {
    S.camera = *camera;
    S.have_camera = true;
  }
  try {
    ptscene::build_bvh_and_flatten(S, host_max_leaf());
  } catch (const std::exception&) {
    delete sc;
    return PT_E_INVALID;
  }
  *out = sc;
  return PT_OK;
}

int pt_scene_from_mesh(const pt_mesh_desc* md, pt_scene** out) {
  return pt_scene_from_mesh_ex(md, 0, out);
}

int pt_scene_from_mesh_ex(const pt_mesh_desc* md, int32_t max_leaf, pt_scene** out) {
  if (!out || max_leaf < 0) return PT_E_INVALID;
  *out = nullptr;
  auto* sc = new pt_scene();
  int rc = ptscene::scene_from_mesh(md, sc->s);
  if (rc) {
    delete sc;
    return rc;
  }
  try {
    ptscene::build_bvh_and_flatten(sc->s, max_leaf > 0 ? (size_t)max_leaf : host_max_leaf());
  } catch (const std::exception&) {
    delete sc;
    return PT_E_INVALID;
  }
  *out = sc;
  return PT_OK;
}

int pt_scene_camera_scotty(const pt_scene* sc, int32_t width, int32_t height, pt_camera* out) {
  if (!sc || !out || width <= 0 || height <= 0) return PT_E_INVALID;
  const Scene& S = sc->s;
  if (!S.have_optics) return PT_E_UNSUPPORTED;
  const double PI = 3.14159265358979323846;
  auto rad = [&](double d) { return d * (PI / 180); };
  auto deg = [&](double r) { return r * (180 / PI); };
  // Camera::configure (camera.cpp:15-33)
  double hfov = S.cam_hfov, vfov = S.cam_vfov;
  const double ar1 = tan(rad(hfov) / 2) / tan(rad(vfov) / 2);
  const double ar = (double)width / height;
  if (ar1 < ar)
    hfov = 2 * deg(atan(tan(rad(vfov) / 2) * ar));
  else if (ar1 > ar)
    vfov = 2 * deg(atan(tan(rad(hfov) / 2) / ar));
  // scene bbox (DynamicScene::Scene::get_bbox: meshes and spheres)
  ptscene::V3 lo(INFINITY, INFINITY, INFINITY), hi(-INFINITY, -INFINITY, -INFINITY);
  auto grow = [&](const ptscene::V3& a, const ptscene::V3& b) {
    lo = ptscene::V3(std::min(lo.x, a.x), std::min(lo.y, a.y), std::min(lo.z, a.z));
    hi = ptscene::V3(std::max(hi.x, b.x), std::max(hi.y, b.y), std::max(hi.z, b.z));
  };
  for (const auto& m : S.meshes)  // Mesh::get_bbox: every vertex
    for (const auto& v : m.positions) grow(v, v);
  for (const auto& p : S.prims)  // Sphere::get_bbox: centre +- radius
    if (p.kind == PT_PRIM_SPHERE) {
      const ptscene::V3 r(p.radius, p.radius, p.radius);
      grow(p.centre - r, p.centre + r);
    }
  if (!(lo.x <= hi.x)) return PT_E_INVALID;
  const ptscene::V3 target = (lo + hi) * 0.5, extent = hi - lo;
  const double canonical = extent.norm() / 2 * 1.5;  // application.cpp:397-402
  double r = std::min(std::max(canonical * 2, canonical / 10.0), canonical * 20.0);
  // Camera::place + compute_position (camera.cpp:35-46, 86-108)
  const ptscene::V3& c = S.cam_dir;
  double phi = acos(c.y), theta = atan2(c.x, c.z);
  if (sin(phi) == 0) phi += 0.00001f;  // EPS_F
  double sinPhi = sin(phi);
  if (sinPhi == 0) {
    phi += 0.00001f;
    sinPhi = sin(phi);
  }
  const ptscene::V3 dir_to_cam(r * sinPhi * sin(theta), r * cos(phi), r * sinPhi * cos(theta));
  const ptscene::V3 pos = target + dir_to_cam;
  const ptscene::V3 upv(0, sinPhi > 0 ? 1 : -1, 0);
  ptscene::V3 X = ptscene::cross(upv, dir_to_cam);
  X = X / X.norm();
  ptscene::V3 Y = ptscene::cross(dir_to_cam, X);
  Y = Y / Y.norm();
  const ptscene::V3 Z = dir_to_cam / dir_to_cam.norm();
  // generate_ray(x, y): c2w * ((x-.5) 2 tan(hfov/2), (y-.5) 2 tan(vfov/2), -1).
  // The kernels form d = kx*left + ky*up + kz*look_at with (kx, ky, kz) a
  // multiple of (x-.5, .5-y, 1) (cu:338-354), so left/up carry the sensor
  // extents and up is negated.
  const double sx = 2 * tan(rad(hfov) / 2), sy = 2 * tan(rad(vfov) / 2);
  const ptscene::V3 look = Z * -1.0, left = X * sx, up = Y * -sy;
  const ptscene::V3* vv[4] = {&pos, &look, &left, &up};
  float* dst[4] = {out->origin, out->look_at, out->left, out->up};
  for (int k = 0; k < 4; ++k) {
    dst[k][0] = (float)vv[k]->x;
    dst[k][1] = (float)vv[k]->y;
    dst[k][2] = (float)vv[k]->z;
  }
  return PT_OK;
}

void pt_scene_free(pt_scene* s) { delete s; }

int pt_scene_get_desc(const pt_scene* sc, pt_scene_desc* d) {
  if (!sc || !d) return PT_E_INVALID;
  const Scene& S = sc->s;
  memset(d, 0, sizeof(*d));
  d->n_prims = (int32_t)S.dprims.size();
  d->prims = S.dprims.data();
  d->shading = S.dshading.data();
  d->n_nodes = (int32_t)S.dnodes.size();
  d->nodes = S.dnodes.data();
  d->n_levels = (int32_t)S.level_start.size() - 1;
  d->level_start = S.level_start.data();
  d->n_bsdfs = (int32_t)S.dbsdfs.size();
  d->bsdfs = S.dbsdfs.data();
  d->light = S.light;
  d->camera = S.camera;
  d->n_lights = (int32_t)S.lights.size();
  d->lights = S.lights.empty() ? nullptr : S.lights.data();
  return PT_OK;
}

int pt_scene_level_counts(const pt_scene* sc, int32_t* counts, int32_t max_levels, int32_t* n_levels) {
  if (!sc || !n_levels) return PT_E_INVALID;
  const auto& lc = sc->s.level_counts;
  *n_levels = (int32_t)lc.size();
  for (int32_t i = 0; counts && i < max_levels && i < (int32_t)lc.size(); ++i) counts[i] = lc[i];
  return PT_OK;
}

int pt_scene_sorted_to_input(const pt_scene* sc, int32_t* out, int32_t n) {
  if (!sc || !out) return PT_E_INVALID;
  const auto& v = sc->s.sorted_to_input;
  for (int32_t i = 0; i < n && i < (int32_t)v.size(); ++i) out[i] = v[i];
  return PT_OK;
}

}  // extern "C"
