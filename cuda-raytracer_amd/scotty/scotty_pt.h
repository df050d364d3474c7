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
};

// CMU462::Ray subset (src/ray.h): origin, direction, [min_t, max_t]
struct Ray {
  Vector3D o, d;
  double min_t = 0.0, max_t = INFINITY;
  Ray() = default;
  Ray(const Vector3D& o_, const Vector3D& d_, double maxt = INFINITY) : o(o_), d(d_), max_t(maxt) {}
};

// CMU462::Intersection subset (src/intersection.h)
struct Intersection {
  double t = INFINITY;
  int primitive = -1;  // index into the BVH-sorted primitive array
  Vector3D n;          // geometric normal facing the ray
  int bsdf = -1;
};

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
  ~Scene() {
    if (s_) pt_scene_free(s_);
  }
  Scene(const Scene&) = delete;
  Scene& operator=(const Scene&) = delete;
  const pt_scene_desc& desc() const { return d_; }

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

// The reference GPU camera (cu:80-86, cu:1590-1607, cu:338-354): fixed
// 53.13 degree field of view; (x, y) are normalised screen coordinates in [0,1].
class Camera {
 public:
  Camera() = default;
  explicit Camera(const pt_camera& c) : c_(c) {}
  const pt_camera& params() const { return c_; }
  Ray generate_ray(double x, double y) const {
    double kx = x - 0.5, ky = -(y - 0.5), kz = 1.0;
    double len = std::sqrt(kx * kx + ky * ky + kz * kz);
    kx /= len;
    ky /= len;
    kz /= len;
    Vector3D d(kx * c_.left[0] + ky * c_.up[0] + kz * c_.look_at[0],
               kx * c_.left[1] + ky * c_.up[1] + kz * c_.look_at[1],
               kx * c_.left[2] + ky * c_.up[2] + kz * c_.look_at[2]);
    double dl = std::sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
    return Ray(Vector3D(c_.origin[0], c_.origin[1], c_.origin[2]), Vector3D(d.x / dl, d.y / dl, d.z / dl));
  }

 private:
  pt_camera c_{};
};

// BVHAccel over the GPU breadth-first traversal.  Single rays work, but the
// path is built for batches: intersect(std::vector<Ray>) is the fast form.
class BVHAccel {
 public:
  BVHAccel(Device& dev, const Scene& scene, size_t max_leaf_size = 32) : dev_(dev), d_(scene.desc()) {
    if (max_leaf_size != 32) throw Error(PT_E_UNSUPPORTED, "BVHAccel: max_leaf_size must be 32 (bvh.h:111)");
    dev_.check(pt_load_scene(dev_.get(), &d_), "pt_load_scene");
  }
  std::vector<Intersection> intersect(const std::vector<Ray>& rays) const {
    std::vector<float> r(rays.size() * 8);
    for (size_t i = 0; i < rays.size(); ++i) {
      float* p = &r[i * 8];
      p[0] = (float)rays[i].o.x;
      p[1] = (float)rays[i].o.y;
      p[2] = (float)rays[i].o.z;
      p[3] = (float)rays[i].max_t;
      p[4] = (float)rays[i].d.x;
      p[5] = (float)rays[i].d.y;
      p[6] = (float)rays[i].d.z;
      p[7] = 0.f;
    }
    std::vector<uint64_t> h(rays.size());
    dev_.check(pt_intersect(dev_.get(), r.data(), (int32_t)rays.size(), h.data()), "pt_intersect");
    std::vector<Intersection> out(rays.size());
    for (size_t i = 0; i < rays.size(); ++i) {
      if (h[i] == PT_HIT_NONE) continue;
      uint32_t tb = (uint32_t)(h[i] >> 32);
      float t;
      memcpy(&t, &tb, 4);
      Intersection& is = out[i];
      is.t = t;
      is.primitive = (int)(uint32_t)h[i];
      const float* q = d_.prims[is.primitive].q;
      uint32_t meta;
      memcpy(&meta, &q[3], 4);
      is.bsdf = (int)(meta & 0x0FFFFFFFu);
      Vector3D n;
      if ((meta >> 28) == PT_PRIM_SPHERE) {
        n = Vector3D(rays[i].o.x + t * rays[i].d.x - q[0], rays[i].o.y + t * rays[i].d.y - q[1],
                     rays[i].o.z + t * rays[i].d.z - q[2]);
      } else {
        n = Vector3D(q[12], q[13], q[14]);
      }
      double nl = std::sqrt(n.x * n.x + n.y * n.y + n.z * n.z);
      double s = (n.x * rays[i].d.x + n.y * rays[i].d.y + n.z * rays[i].d.z) < 0 ? 1.0 / nl : -1.0 / nl;
      is.n = Vector3D(n.x * s, n.y * s, n.z * s);
    }
    return out;
  }
  bool intersect(const Ray& r, Intersection* isect) const {
    Intersection i = intersect(std::vector<Ray>{r})[0];
    if (i.primitive < 0 || i.t < r.min_t) return false;
    if (isect) *isect = i;
    return true;
  }
  bool intersect(const Ray& r) const { return intersect(r, nullptr); }

 private:
  Device& dev_;
  pt_scene_desc d_;
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

// ---- the progressive viewer (display.cpp:99-190 without the GLUT window) -----
// Each displayed frame is renderPicture(): unless paused, one more
// renderAccumulate of samples_per_frame samples on top of the accumulation
// (sample indices continue: sample_offset), then the display image (median
// filtered below 32 accumulated samples, cu:1539-1569).  handleKeyPress moves
// the camera like the reference's w/a/s/d keys (origin += (0, 0, -+0.01) /
// (-+0.01, 0, 0) in double, then setViewpoint: the accumulation restarts), p
// toggles pause, + resumes.  A GUI would call these from its event loop; the
// headless loop drives them from a key script (ptrender --viewer).
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
    if (!paused_) r_.render(spf_, bounces_, flags_);
    if (paused_) update_ = false;
    ++frames_;
    return r_.getImage();
  }
  bool paused() const { return paused_; }
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
