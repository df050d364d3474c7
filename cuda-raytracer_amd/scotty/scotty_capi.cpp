// C entry points over the Scotty3D surface (scotty_pt.h) on the GPU, for
// callers without C++ (ctypes tests, other host languages): the
// CMU462::PathTracer tile/worker loop with the GPU estimator, the
// progressive viewer loop of display.cpp driven by a key script, the
// Camera's generate_ray and the BVHAccel over Scotty3D primitives.
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "scotty_capi.h"
#include "scotty_pt.h"

namespace {
void put_ray(const scotty::Ray& r, double* out) {
  out[0] = r.o.x;
  out[1] = r.o.y;
  out[2] = r.o.z;
  out[3] = r.d.x;
  out[4] = r.d.y;
  out[5] = r.d.z;
}
int fail(const std::exception& e, int code, char* err, size_t errlen) {
  if (err && errlen) {
    std::strncpy(err, e.what(), errlen - 1);
    err[errlen - 1] = 0;
  }
  return code;
}
}  // namespace

extern "C" {

// PathTracer(ns_aa = spp, max_ray_depth = depth, ..., num_threads = threads):
// set_scene, set_frame_size, start_raytracing (one pt_render), the workers'
// raytrace_tile -> raytrace_pixel, then the frame (w x h RGBA, rows bottom-up).
int scotty_render(const pt_scene_desc* desc, int w, int h, int spp, int depth, uint32_t flags, int threads,
                  int device, float* out, char* err, size_t errlen) {
  if (!desc || !out || w <= 0 || h <= 0 || spp <= 0 || threads < 0) return PT_E_INVALID;
  try {
    scotty::PathTracer pt((size_t)spp, (size_t)depth, 1, 1, 1, 1, (size_t)threads, device);
    pt.set_scene(*desc);
    pt.set_frame_size((size_t)w, (size_t)h);
    pt.set_flags(flags);
    pt.start_raytracing();
    const std::vector<float>& f = pt.frame();
    std::memcpy(out, f.data(), f.size() * sizeof(float));
    return PT_OK;
  } catch (const scotty::Error& e) {
    return fail(e, e.code, err, errlen);
  } catch (const std::exception& e) {
    return fail(e, PT_E_HIP, err, errlen);
  }
}

// The same PathTracer over several GPUs of one process (pt_group): tiles dealt
// to devices[0..n), sums gathered into devices[0]; *gather_kind (optional):
// PT_GATHER_RCCL or PT_GATHER_HOST, the gather used.
int scotty_render_multi(const pt_scene_desc* desc, int w, int h, int spp, int depth, uint32_t flags, int threads,
                        const int32_t* devices, int32_t n_devices, int32_t gather, float* out, int32_t* gather_kind,
                        double* gather_ms, char* err, size_t errlen) {
  if (!desc || !out || !devices || n_devices <= 0 || w <= 0 || h <= 0 || spp <= 0 || threads < 0)
    return PT_E_INVALID;
  try {
    scotty::MultiGpuPathTracer pt(std::vector<int>(devices, devices + n_devices), (size_t)spp, (size_t)depth,
                                  (size_t)threads, gather);
    pt.set_scene(*desc);
    pt.set_frame_size((size_t)w, (size_t)h);
    pt.set_flags(flags);
    pt.start_raytracing();
    const std::vector<float>& f = pt.frame();
    std::memcpy(out, f.data(), f.size() * sizeof(float));
    if (gather_kind) *gather_kind = pt.gather_kind();
    if (gather_ms) pt_group_timing(pt.group(), gather_ms, nullptr);
    return PT_OK;
  } catch (const scotty::Error& e) {
    return fail(e, e.code, err, errlen);
  } catch (const std::exception& e) {
    return fail(e, PT_E_HIP, err, errlen);
  }
}

// The viewer: one renderPicture per character of `keys`, after
// handleKeyPress(c) unless c is '.'.  out: the last displayed frame;
// *samples: the samples accumulated in it.
int scotty_viewer(const pt_scene_desc* desc, int w, int h, int samples_per_frame, int bounces, uint32_t flags,
                  const char* keys, int device, float* out, int32_t* samples, char* err, size_t errlen) {
  if (!desc || !out || !keys || w <= 0 || h <= 0 || samples_per_frame <= 0) return PT_E_INVALID;
  try {
    scotty::CudaRenderer r(device);
    r.allocOutputImage(w, h);
    r.loadScene(*desc);
    r.setup();
    scotty::Viewer v(r, samples_per_frame, bounces, flags);
    const scotty::Image* img = nullptr;
    for (const char* k = keys; *k; ++k) {
      if (*k != '.') v.handleKeyPress(*k);
      img = v.renderPicture();
    }
    if (img) std::memcpy(out, img->data.data(), img->data.size() * sizeof(float));
    if (samples) pt_samples(r.device().get(), samples);
    return PT_OK;
  } catch (const scotty::Error& e) {
    return fail(e, e.code, err, errlen);
  } catch (const std::exception& e) {
    return fail(e, PT_E_HIP, err, errlen);
  }
}

int scotty_generate_rays(const pt_camera* cam, int32_t n, const double* xy, double* rays) {
  if (!cam || n < 0 || (n > 0 && (!xy || !rays))) return PT_E_INVALID;
  const scotty::Camera c(*cam);
  for (int32_t i = 0; i < n; ++i) put_ray(c.generate_ray(xy[2 * i], xy[2 * i + 1]), rays + 6 * (size_t)i);
  return PT_OK;
}

int scotty_camera_place(const double info[4], int32_t w, int32_t h, const double target[3], double phi, double theta,
                        double r, double min_r, double max_r, pt_camera* out, int32_t n, const double* xy,
                        double* rays, double* fov_out) {
  if (!info || !target || w <= 0 || h <= 0 || n < 0 || (n > 0 && (!xy || !rays))) return PT_E_INVALID;
  scotty::Camera c;
  scotty::CameraInfo ci;
  ci.hFov = info[0];
  ci.vFov = info[1];
  ci.nClip = info[2];
  ci.fClip = info[3];
  c.configure(ci, (size_t)w, (size_t)h);
  c.place(scotty::Vector3D(target[0], target[1], target[2]), phi, theta, r, min_r, max_r);
  if (out) *out = c.params();
  for (int32_t i = 0; i < n; ++i) put_ray(c.generate_ray(xy[2 * i], xy[2 * i + 1]), rays + 6 * (size_t)i);
  if (fov_out) {
    fov_out[0] = c.h_fov();
    fov_out[1] = c.v_fov();
  }
  return PT_OK;
}

}  // extern "C"

// The BVHAccel entry points own the Scotty3D objects the accelerator points to.
struct scotty_bvh {
  scotty::DiffuseBSDF mesh_bsdf{scotty::Spectrum(0.5f, 0.5f, 0.5f)};
  scotty::MirrorBSDF sphere_bsdf{scotty::Spectrum(1.0f, 1.0f, 1.0f)};
  std::unique_ptr<scotty::Mesh> mesh;
  std::vector<std::unique_ptr<scotty::SphereObject>> spheres;
  std::vector<std::unique_ptr<scotty::Primitive>> prims;  // triangles, then spheres
  std::unordered_map<const scotty::Primitive*, int32_t> index;
  std::unique_ptr<scotty::BVHAccel> bvh;
};

extern "C" {

int scotty_bvh_create(const double* positions, const double* normals, int32_t n_verts, const int32_t* indices,
                      int32_t n_tris, const double* spheres, int32_t n_spheres, int32_t max_leaf, int32_t device,
                      scotty_bvh** out, char* err, size_t errlen) {
  if (!out || n_verts < 0 || n_tris < 0 || n_spheres < 0 || max_leaf <= 0 || (n_tris && (!positions || !normals || !indices)) ||
      (n_spheres && !spheres))
    return PT_E_INVALID;
  *out = nullptr;
  try {
    auto b = std::make_unique<scotty_bvh>();
    std::vector<scotty::Vector3D> P((size_t)n_verts), N((size_t)n_verts);
    for (int32_t i = 0; i < n_verts; ++i) {
      P[(size_t)i] = scotty::Vector3D(positions[3 * i], positions[3 * i + 1], positions[3 * i + 2]);
      N[(size_t)i] = scotty::Vector3D(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]);
    }
    std::vector<size_t> idx((size_t)n_tris * 3);
    for (size_t i = 0; i < idx.size(); ++i) {
      if (indices[i] < 0 || indices[i] >= n_verts) return PT_E_INVALID;
      idx[i] = (size_t)indices[i];
    }
    b->mesh = std::make_unique<scotty::Mesh>(std::move(P), std::move(N), std::move(idx), &b->mesh_bsdf);
    std::vector<scotty::Primitive*> list = b->mesh->get_primitives();  // Mesh::get_primitives
    for (int32_t i = 0; i < n_spheres; ++i) {
      const double* s = spheres + 4 * (size_t)i;
      b->spheres.push_back(
          std::make_unique<scotty::SphereObject>(scotty::Vector3D(s[0], s[1], s[2]), s[3], &b->sphere_bsdf));
      for (scotty::Primitive* p : b->spheres.back()->get_primitives()) list.push_back(p);
    }
    for (size_t i = 0; i < list.size(); ++i) {
      b->prims.emplace_back(list[i]);
      b->index[list[i]] = (int32_t)i;
    }
    b->bvh = std::make_unique<scotty::BVHAccel>(list, (size_t)max_leaf, device);
    *out = b.release();
    return PT_OK;
  } catch (const scotty::Error& e) {
    return fail(e, e.code, err, errlen);
  } catch (const std::exception& e) {
    return fail(e, PT_E_HIP, err, errlen);
  }
}

static scotty::Ray get_ray(const double* r) {
  scotty::Ray ray(scotty::Vector3D(r[0], r[1], r[2]), scotty::Vector3D(r[3], r[4], r[5]));
  ray.min_t = r[6];
  ray.max_t = r[7];
  return ray;
}

int scotty_bvh_intersect(scotty_bvh* b, const double* rays, int32_t n, int32_t single, int32_t* hit, double* t,
                         int32_t* prim, double* normal) {
  if (!b || n < 0 || (n > 0 && (!rays || !hit || !t || !prim || !normal))) return PT_E_INVALID;
  try {
    std::vector<scotty::Intersection> is((size_t)n);
    std::vector<char> h((size_t)n, 0);
    if (single) {
      for (int32_t i = 0; i < n; ++i) h[(size_t)i] = b->bvh->intersect(get_ray(rays + 8 * (size_t)i), &is[(size_t)i]);
    } else {
      std::vector<scotty::Ray> rv;
      for (int32_t i = 0; i < n; ++i) rv.push_back(get_ray(rays + 8 * (size_t)i));
      is = b->bvh->intersect(rv);
      for (int32_t i = 0; i < n; ++i) h[(size_t)i] = is[(size_t)i].primitive != nullptr;
    }
    for (int32_t i = 0; i < n; ++i) {
      hit[i] = h[(size_t)i];
      t[i] = h[(size_t)i] ? is[(size_t)i].t : INFINITY;
      prim[i] = h[(size_t)i] ? b->index.at(is[(size_t)i].primitive) : -1;
      normal[3 * i] = is[(size_t)i].n.x;
      normal[3 * i + 1] = is[(size_t)i].n.y;
      normal[3 * i + 2] = is[(size_t)i].n.z;
    }
    return PT_OK;
  } catch (const scotty::Error& e) {
    return e.code;
  } catch (const std::exception&) {
    return PT_E_HIP;
  }
}

int scotty_bvh_occluded(scotty_bvh* b, const double* rays, int32_t n, int32_t* hit) {
  if (!b || n < 0 || (n > 0 && (!rays || !hit))) return PT_E_INVALID;
  try {
    for (int32_t i = 0; i < n; ++i) hit[i] = b->bvh->intersect(get_ray(rays + 8 * (size_t)i)) ? 1 : 0;
    return PT_OK;
  } catch (const scotty::Error& e) {
    return e.code;
  } catch (const std::exception&) {
    return PT_E_HIP;
  }
}

void scotty_bvh_destroy(scotty_bvh* b) { delete b; }

}  // extern "C"
