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

/* The viewer: one renderPicture (samples_per_frame more samples, progressive)
 * per character of `keys`, after handleKeyPress(c) unless c is '.'
 * (w/a/s/d move the camera by 0.01 and restart the accumulation, p pauses).
 * out[w*h*4]: the last displayed frame (median-filtered below 32 samples);
 * *samples: the samples accumulated in it. */
int scotty_viewer(const pt_scene_desc* desc, int w, int h, int samples_per_frame, int bounces, uint32_t flags,
                  const char* keys, int device, float* out, int32_t* samples, char* err, size_t errlen);

#ifdef __cplusplus
}
#endif

#endif /* SCOTTY_CAPI_H */
