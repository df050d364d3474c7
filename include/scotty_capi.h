/* scotty_capi.h -- C entry points of the Scotty3D surface on the GPU
 * (cuda-raytracer_amd/scotty/scotty_capi.cpp -> lib/libscotty_gpu.so, linked
 * against libptcore.so).  For callers without C++; C++ callers use
 * cuda-raytracer_amd/scotty/scotty_pt.h directly.
 *
 *   CMU462::PathTracer::start_raytracing / raytrace_tile / raytrace_pixel /
 *     worker_thread      src/pathtracer.cpp:183-213, 499-558   scotty_render
 *   the GLUT viewer loop: handleKeyPress + renderPicture (display.cpp:99-190)
 *     over CudaRenderer::renderAccumulate / setViewpoint
 *     (src/cudaRenderer.cu:1845-1870, 2419-2457)              scotty_viewer
 *   CMU462::Camera::configure / place / generate_ray
 *     (src/camera.h:26-81, camera.cpp:15-117)      scotty_camera_place, scotty_generate_rays
 *   StaticScene::BVHAccel(primitives, max_leaf_size), intersect(ray[, isect])
 *     (src/bvh.h:111-149, static_scene/triangle.cpp:119-209)
 *                                  scotty_bvh_create / _intersect / _occluded / _destroy
 *
 * Frames are width x height RGBA float, rows bottom-up (pt_api.h layout).
 * Return 0 or a negative PT_E* code; err (optional) receives the message. */
#ifndef SCOTTY_CAPI_H
#define SCOTTY_CAPI_H

#include <stddef.h>
#include <stdint.h>

#include "pt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* PathTracer(ns_aa = spp, max_ray_depth = depth, ..., num_threads = threads
 * (0 = hardware_concurrency)) on device `device`: set_scene(desc),
 * set_frame_size(w, h), start_raytracing (one pt_render on the GPU, then the
 * 32x32-tile workers' raytrace_pixel reads), the frame into out[w*h*4]. */
int scotty_render(const pt_scene_desc* desc, int w, int h, int spp, int depth, uint32_t flags, int threads,
                  int device, float* out, char* err, size_t errlen);

/* The same PathTracer over n_devices GPUs of one process (pt_group_*,
 * pt_api.h): the tiles are dealt to devices[i] round-robin, each device
 * renders on its own host thread, the sums are gathered into devices[0]
 * (gather: PT_GATHER_AUTO / _RCCL / _HOST).  *gather_kind (optional): the
 * gather used; *gather_ms (optional): its wall time. */
int scotty_render_multi(const pt_scene_desc* desc, int w, int h, int spp, int depth, uint32_t flags, int threads,
                        const int32_t* devices, int32_t n_devices, int32_t gather, float* out, int32_t* gather_kind,
                        double* gather_ms, char* err, size_t errlen);

/* The viewer: one renderPicture (samples_per_frame more samples, progressive)
 * per character of `keys`, after handleKeyPress(c) unless c is '.'
 * (w/a/s/d move the camera by 0.01 and restart the accumulation, p pauses).
 * out[w*h*4]: the last displayed frame (median-filtered below 32 samples);
 * *samples: the samples accumulated in it. */
int scotty_viewer(const pt_scene_desc* desc, int w, int h, int samples_per_frame, int bounces, uint32_t flags,
                  const char* keys, int device, float* out, int32_t* samples, char* err, size_t errlen);

/* ---- CMU462::Camera::generate_ray (camera.h:71-81) ------------------------
 * scotty::Camera over a pt_camera (the kernels' camera model, cu:80-86):
 * generate_ray(x, y) for n normalised sensor points xy[2n] ((0.5, 0.5) the
 * centre, y up); rays[6n] = origin.xyz, unit direction.xyz (double). */
int scotty_generate_rays(const pt_camera* cam, int32_t n, const double* xy, double* rays);
/* The Scotty3D framing: Camera::configure({hfov, vfov, nclip, fclip} in
 * degrees, w, h) (camera.cpp:15-33) then place(target, phi, theta, r, min_r,
 * max_r) (camera.cpp:35-46, 86-108).  *out: the camera as a pt_camera (for
 * pt_set_camera); then generate_ray for n points as above (rays may be NULL
 * when n == 0); fov_out (optional): the fitted {hFov, vFov} in degrees. */
int scotty_camera_place(const double info[4], int32_t w, int32_t h, const double target[3], double phi, double theta,
                        double r, double min_r, double max_r, pt_camera* out, int32_t n, const double* xy,
                        double* rays, double* fov_out);

/* ---- StaticScene::BVHAccel(primitives, max_leaf_size) + intersect --------------
 * (bvh.h:111-149) over Scotty3D primitives: the Triangles of one Mesh
 * (positions[3 n_verts], vertex normals[3 n_verts], indices[3 n_tris]; a
 * DiffuseBSDF) followed by n_spheres Spheres (spheres[4 n]: centre, radius), on
 * GPU `device`.  scotty_bvh_intersect answers intersect(ray, isect) for n rays
 * (rays[8n] = o.xyz, d.xyz, min_t, max_t, double): hit[i] 0/1, and for a hit
 * t[i], prim[i] (index into the primitive list: triangles, then spheres) and
 * normal[3i] (Intersection::n).  single != 0 calls the one-ray form per ray,
 * else one batch (the same results). */
typedef struct scotty_bvh scotty_bvh;
int scotty_bvh_create(const double* positions, const double* normals, int32_t n_verts, const int32_t* indices,
                      int32_t n_tris, const double* spheres, int32_t n_spheres, int32_t max_leaf, int32_t device,
                      scotty_bvh** out, char* err, size_t errlen);
int scotty_bvh_intersect(scotty_bvh* b, const double* rays, int32_t n, int32_t single, int32_t* hit, double* t,
                         int32_t* prim, double* normal);
/* bool intersect(const Ray&) (bvh.h:134): any hit in [min_t, max_t] */
int scotty_bvh_occluded(scotty_bvh* b, const double* rays, int32_t n, int32_t* hit);
void scotty_bvh_destroy(scotty_bvh* b);

#ifdef __cplusplus
}
#endif

#endif /* SCOTTY_CAPI_H */
