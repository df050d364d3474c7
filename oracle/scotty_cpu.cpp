// scotty_cpu.cpp -- CPU ORACLE run through the Scotty3D PathTracer surface
// (test infrastructure only: the CPU baseline of bench.py and the config-1
// golden images; the product never links it).
//
// BASELINE config 1 / SURVEY §8(d): the reference CPU path tracer's structure
// -- PathTracer::start_raytracing's work queue of 32x32 tiles and
// numWorkerThreads = std::thread::hardware_concurrency() workers calling
// raytrace_tile -> raytrace_pixel (src/pathtracer.cpp:183-213, 499-558) -- is
// scotty::PathTracerT from the product's header (cuda-raytracer_amd/scotty/
// scotty_pt.h); the per-pixel estimator here is the oracle's restated path
// (ptoracle.c pto_pixel), because the shipped pathtracer.cpp is a stub that
// renders black.
#include <atomic>
#include <chrono>
#include <cstdint>

#include "../cuda-raytracer_amd/scotty/scotty_pt.h"

extern "C" float* pto_bw_table(const pt_scene_desc* S);
extern "C" void pto_free(void* p);
extern "C" void pto_pixel_bw(const pt_scene_desc* S, const float* bw, int W, int H, int spp, int max_bounces,
                             uint32_t seed, uint32_t flags, int sample_offset, uint32_t g, float* out4, uint64_t* rays);

namespace {

struct OracleEstimator {
  const pt_scene_desc* S = nullptr;
  float* bw = nullptr;  // the scene's triangle rows (pto_bw_table), built in begin()
  ~OracleEstimator() { pto_free(bw); }
  uint32_t seed = 15618;
  int W = 0, H = 0, spp = 1, depth = 8;
  uint32_t flags = 0;
  // the tiles to render (bench samples a subset of the frame): tile t renders
  // iff t % stride == 0; others are left 0
  size_t stride = 1;
  std::atomic<uint64_t> rays{0};
  void begin(size_t w, size_t h, size_t s, size_t d, uint32_t f) {
    W = (int)w;
    H = (int)h;
    spp = (int)s;
    depth = (int)d;
    flags = f;
    rays = 0;
    pto_free(bw);
    bw = pto_bw_table(S);
  }
  void pixel(size_t x, size_t y, float rgba[4]) {
    const size_t ntx = ((size_t)W + 31) / 32;
    if (((y / 32) * ntx + x / 32) % stride != 0) {
      rgba[0] = rgba[1] = rgba[2] = rgba[3] = 0.0f;
      return;
    }
    uint64_t n = 0;
    pto_pixel_bw(S, bw, W, H, spp, depth, seed, flags, 0, (uint32_t)(y * (size_t)W + x), rgba, &n);
    rays += n;
  }
};

}  // namespace

// Render W x H at spp samples through the Scotty3D surface on `threads`
// workers (0 = std::thread::hardware_concurrency()), into rgba (W*H*4 floats,
// rows bottom-up).  Only tiles t with t % tile_stride == 0 are rendered (1 =
// the whole frame).  Returns the rays cast; *seconds = wall time of
// start_raytracing .. is_done; *threads_used = the worker count.
extern "C" uint64_t pto_scotty_render(const pt_scene_desc* S, int W, int H, int spp, int max_bounces, uint32_t seed,
                                      uint32_t flags, int threads, int tile_stride, float* rgba, double* seconds,
                                      int* threads_used) {
  OracleEstimator est;
  est.S = S;
  est.seed = seed;
  est.stride = tile_stride > 0 ? (size_t)tile_stride : 1;
  scotty::PathTracerT<OracleEstimator> pt(est, (size_t)spp, (size_t)max_bounces, 1, 1, 1, 1,
                                          threads > 0 ? (size_t)threads : 0);
  pt.set_frame_size((size_t)W, (size_t)H);
  pt.set_flags(flags);
  const auto t0 = std::chrono::steady_clock::now();
  pt.start_raytracing();
  pt.is_done();
  const auto t1 = std::chrono::steady_clock::now();
  if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
  if (threads_used) *threads_used = (int)pt.num_worker_threads();
  const std::vector<float>& f = pt.frame();
  std::copy(f.begin(), f.end(), rgba);
  return est.rays.load();
}
