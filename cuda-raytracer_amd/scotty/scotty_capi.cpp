// C entry points over the Scotty3D surface (scotty_pt.h) on the GPU, for
// callers without C++ (ctypes tests, other host languages): the
// CMU462::PathTracer tile/worker loop with the GPU estimator, and the
// progressive viewer loop of display.cpp driven by a key script.
#include <cstring>
#include <string>

#include "scotty_capi.h"
#include "scotty_pt.h"

namespace {
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

}  // extern "C"
