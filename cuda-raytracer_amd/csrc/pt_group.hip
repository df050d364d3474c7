// pt_group: one frame rendered by several GPUs of one process, gathered into
// member 0's device frame (pt_api.h "one frame over several
// GPUs").  The members are ordinary contexts (pt_create per device) driven
// through the public C ABI -- pt_render with rank = i, nranks = n on one host
// thread per member -- so the tile sharding is exactly the Python bench's
// (ptdist.py) and the gathered frame equals one context's whole frame bit for
// bit.  The gather moves each member's accumulation sums (pt_owned_pixels'
// device pointer: float4 per owned pixel in slot order, no staging copy) to
// member 0 with one grouped RCCL send/receive round over xGMI, then one kernel
// on member 0 scatters them to their row-major positions as sums / spp
// (k_frame's arithmetic, post.hip).  RCCL is loaded with dlopen at
// pt_group_create, so libptcore does not depend on it; a device listed twice
// (RCCL takes one rank per GPU) or a missing librccl selects the host-staged
// copy instead.  The reference has no multi-GPU path (cu:1874-1897).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "pt_api.h"

namespace {

constexpr int TPB = 256;

// frame[idx[q]] = (sum.xyz / ns, 1): the assembly k_frame does for one context
__global__ __launch_bounds__(TPB) void k_group_frame(const float4* __restrict__ sums,
                                                     const uint32_t* __restrict__ idx, uint32_t n, float ns,
                                                     float4* __restrict__ frame) {
  const uint32_t q = blockIdx.x * TPB + threadIdx.x;
  if (q >= n) return;
  const float4 a = sums[q];
  frame[idx[q]] = make_float4(a.x / ns, a.y / ns, a.z / ns, 1.0f);
}

// the RCCL entry points the gather uses, resolved from librccl at run time
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;

  bool load(std::string* why) {
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) {
      *why = std::string("librccl not loadable: ") + dlerror();
      return false;
    }
    bool ok = sym(CommInitAll, "ncclCommInitAll") && sym(CommDestroy, "ncclCommDestroy") &&
              sym(GroupStart, "ncclGroupStart") && sym(GroupEnd, "ncclGroupEnd") && sym(Send, "ncclSend") &&
              sym(Recv, "ncclRecv") && sym(GetErrorString, "ncclGetErrorString");
    if (!ok) *why = "librccl lacks a needed entry point";
    return ok;
  }
  template <class F>
  bool sym(F& f, const char* name) {
    f = reinterpret_cast<F>(dlsym(h, name));
    return f != nullptr;
  }
  ~Rccl() {
    if (h) dlclose(h);
  }
};

}  // namespace

struct pt_group {
  std::vector<int32_t> dev;
  std::vector<pt_ctx*> m;
  int32_t kind = PT_GATHER_HOST;
  Rccl rccl;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;  // one per member: its send (member 0: receives + assembly)
  // member 0's buffers: received sums, their pixel indices, the frame
  float4* d_recv = nullptr;
  uint32_t* d_idx = nullptr;
  float4* d_frame = nullptr;
  size_t cap = 0;
  std::vector<int32_t> counts, offs;  // owned pixels per member, prefix offsets
  int32_t lw = 0, lh = 0, ltile = 0;  // the layout the index buffer holds
  std::vector<float> stage;           // host-staged gather
  int32_t fb_w = 0, fb_h = 0;
  double gather_ms = 0, render_ms = 0;
  std::string err;
};

static int gfail(pt_group* g, int code, const std::string& msg) {
  if (g) g->err = msg;
  return code;
}

#define GHIP(g, x)                                                                         \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return gfail(g, PT_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define GNCCL(g, x)                                                                           \
  do {                                                                                        \
    ncclResult_t r_ = (x);                                                                    \
    if (r_ != ncclSuccess) return gfail(g, PT_E_HIP, std::string(#x) + ": " + g->rccl.GetErrorString(r_)); \
  } while (0)

extern "C" {

int pt_group_create(pt_group** out, const int32_t* devices, int32_t n, int32_t gather) {
  if (!out || !devices || n <= 0 || gather < PT_GATHER_AUTO || gather > PT_GATHER_HOST) return PT_E_INVALID;
  *out = nullptr;
  auto g = new pt_group();
  g->dev.assign(devices, devices + n);
  for (int32_t i = 0; i < n; ++i) {
    pt_ctx* c = nullptr;
    int rc = pt_create(&c, devices[i]);
    if (rc) {
      for (pt_ctx* x : g->m) pt_destroy(x);
      delete g;
      return rc;
    }
    g->m.push_back(c);
  }
  std::vector<int32_t> sorted = g->dev;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  std::string why = "a device is listed twice (RCCL takes one rank per GPU)";
  if (gather != PT_GATHER_HOST && distinct && g->rccl.load(&why)) {
    g->comms.resize(n);
    std::vector<int> d(g->dev.begin(), g->dev.end());
    ncclResult_t r = g->rccl.CommInitAll(g->comms.data(), n, d.data());
    if (r == ncclSuccess) {
      g->kind = PT_GATHER_RCCL;
    } else {
      why = std::string("ncclCommInitAll: ") + g->rccl.GetErrorString(r);
      g->comms.clear();
    }
  }
  if (gather == PT_GATHER_RCCL && g->kind != PT_GATHER_RCCL) {
    pt_group_destroy(g);
    return PT_E_UNSUPPORTED;
  }
  g->streams.resize(n, nullptr);
  for (int32_t i = 0; i < n; ++i) {
    if (hipSetDevice(g->dev[i]) != hipSuccess ||
        hipStreamCreateWithFlags(&g->streams[i], hipStreamNonBlocking) != hipSuccess) {
      pt_group_destroy(g);
      return PT_E_HIP;
    }
  }
  if (g->kind != PT_GATHER_RCCL) g->err = "host-staged gather: " + why;
  *out = g;
  return PT_OK;
}

void pt_group_destroy(pt_group* g) {
  if (!g) return;
  for (ncclComm_t c : g->comms)
    if (c) g->rccl.CommDestroy(c);
  for (size_t i = 0; i < g->streams.size(); ++i)
    if (g->streams[i]) {
      hipSetDevice(g->dev[i]);
      hipStreamDestroy(g->streams[i]);
    }
  if (!g->dev.empty()) {
    hipSetDevice(g->dev[0]);
    hipFree(g->d_recv);
    hipFree(g->d_idx);
    hipFree(g->d_frame);
  }
  for (pt_ctx* c : g->m) pt_destroy(c);
  delete g;
}

const char* pt_group_last_error(const pt_group* g) { return g ? g->err.c_str() : "null group"; }

int pt_group_gather_kind(const pt_group* g, int32_t* kind) {
  if (!g || !kind) return PT_E_INVALID;
  *kind = g->kind;
  return PT_OK;
}

int pt_group_size(const pt_group* g, int32_t* n) {
  if (!g || !n) return PT_E_INVALID;
  *n = (int32_t)g->m.size();
  return PT_OK;
}

pt_ctx* pt_group_member(pt_group* g, int32_t i) {
  return (g && i >= 0 && (size_t)i < g->m.size()) ? g->m[i] : nullptr;
}

static int each(pt_group* g, const char* what, int (*f)(pt_ctx*, const void*), const void* arg) {
  if (!g) return PT_E_INVALID;
  for (size_t i = 0; i < g->m.size(); ++i) {
    int rc = f(g->m[i], arg);
    if (rc) return gfail(g, rc, std::string(what) + " on member " + std::to_string(i) + ": " + pt_last_error(g->m[i]));
  }
  return PT_OK;
}

int pt_group_load_scene(pt_group* g, const pt_scene_desc* s) {
  if (!s) return PT_E_INVALID;
  return each(g, "pt_load_scene", [](pt_ctx* c, const void* a) { return pt_load_scene(c, (const pt_scene_desc*)a); },
              s);
}

int pt_group_set_camera(pt_group* g, const pt_camera* cam) {
  if (!cam) return PT_E_INVALID;
  return each(g, "pt_set_camera", [](pt_ctx* c, const void* a) { return pt_set_camera(c, (const pt_camera*)a); },
              cam);
}

int pt_group_clear(pt_group* g) {
  return each(g, "pt_clear", [](pt_ctx* c, const void*) { return pt_clear(c); }, nullptr);
}

// (re)build member 0's pixel index of the gathered rows for this frame shape
static int layout(pt_group* g, int32_t w, int32_t h, int32_t tile) {
  const size_t n = g->m.size();
  g->counts.assign(n, 0);
  g->offs.assign(n + 1, 0);
  for (size_t i = 0; i < n; ++i) {
    int rc = pt_owned_pixels(g->m[i], &g->counts[i], nullptr, 0, nullptr);
    if (rc) return gfail(g, rc, "pt_owned_pixels");
    g->offs[i + 1] = g->offs[i] + g->counts[i];
  }
  const size_t total = (size_t)g->offs[n];
  if (total != (size_t)w * h) return gfail(g, PT_E_INVALID, "members' owned pixels do not tile the frame");
  if (w == g->lw && h == g->lh && tile == g->ltile) return PT_OK;
  std::vector<int32_t> idx(total);
  for (size_t i = 0; i < n; ++i) {
    int32_t k = 0;
    int rc = pt_owned_pixels(g->m[i], &k, idx.data() + g->offs[i], (size_t)g->counts[i], nullptr);
    if (rc) return gfail(g, rc, "pt_owned_pixels");
  }
  GHIP(g, hipSetDevice(g->dev[0]));
  if (total > g->cap) {
    hipFree(g->d_recv);
    hipFree(g->d_idx);
    hipFree(g->d_frame);
    g->d_recv = g->d_frame = nullptr;
    g->d_idx = nullptr;
    g->cap = 0;
    GHIP(g, hipMalloc(&g->d_recv, total * sizeof(float4)));
    GHIP(g, hipMalloc(&g->d_idx, total * sizeof(uint32_t)));
    GHIP(g, hipMalloc(&g->d_frame, total * sizeof(float4)));
    g->cap = total;
  }
  GHIP(g, hipMemcpy(g->d_idx, idx.data(), total * sizeof(uint32_t), hipMemcpyHostToDevice));
  g->lw = w;
  g->lh = h;
  g->ltile = tile;
  return PT_OK;
}

int pt_group_render(pt_group* g, const pt_render_params* params) {
  if (!g || !params || params->width <= 0 || params->height <= 0) return PT_E_INVALID;
  const auto t0 = std::chrono::steady_clock::now();
  const int32_t n = (int32_t)g->m.size();
  std::vector<int> rc(n, PT_OK);
  {
    std::vector<std::thread> th;
    for (int32_t i = 0; i < n; ++i)
      th.emplace_back([&, i] {
        pt_render_params p = *params;
        p.rank = i;
        p.nranks = n;
        rc[i] = pt_render(g->m[i], &p);
      });
    for (auto& t : th) t.join();
  }
  for (int32_t i = 0; i < n; ++i)
    if (rc[i]) return gfail(g, rc[i], "pt_render on member " + std::to_string(i) + ": " + pt_last_error(g->m[i]));
  const auto t1 = std::chrono::steady_clock::now();
  const int32_t tile = params->tile_size > 0 ? params->tile_size : 32;
  int r = layout(g, params->width, params->height, tile);
  if (r) return r;
  int32_t spp = 0;
  for (int32_t i = 0; i < n; ++i) {
    int32_t s = 0;
    pt_samples(g->m[i], &s);
    if (i == 0) spp = s;
    else if (s != spp) return gfail(g, PT_E_INVALID, "members hold different sample counts");
  }
  std::vector<void*> sums(n, nullptr);
  for (int32_t i = 0; i < n; ++i) {
    int32_t k = 0;
    if ((r = pt_owned_pixels(g->m[i], &k, nullptr, 0, &sums[i]))) return gfail(g, r, "pt_owned_pixels");
  }
  if (g->kind == PT_GATHER_RCCL) {
    // one grouped round: every member sends its sums (from its accumulation
    // buffer, which pt_render left complete) to member 0, which receives each
    // into its slice
    // (a failing Send / Recv still closes the group before the error returns:
    // an open group would swallow the next render's calls)
    GNCCL(g, g->rccl.GroupStart());
    ncclResult_t gr = ncclSuccess;
    const char* what = "ncclSend";
    for (int32_t i = 0; i < n && gr == ncclSuccess; ++i)
      if (g->counts[i]) gr = g->rccl.Send(sums[i], 4 * (size_t)g->counts[i], ncclFloat32, 0, g->comms[i], g->streams[i]);
    if (gr == ncclSuccess) what = "ncclRecv";
    for (int32_t i = 0; i < n && gr == ncclSuccess; ++i)
      if (g->counts[i])
        gr = g->rccl.Recv(g->d_recv + g->offs[i], 4 * (size_t)g->counts[i], ncclFloat32, i, g->comms[0], g->streams[0]);
    const ncclResult_t er = g->rccl.GroupEnd();
    if (gr != ncclSuccess) return gfail(g, PT_E_HIP, std::string(what) + ": " + g->rccl.GetErrorString(gr));
    if (er != ncclSuccess) return gfail(g, PT_E_HIP, std::string("ncclGroupEnd: ") + g->rccl.GetErrorString(er));
    for (int32_t i = 1; i < n; ++i) {
      GHIP(g, hipSetDevice(g->dev[i]));
      GHIP(g, hipStreamSynchronize(g->streams[i]));
    }
  } else {
    const size_t total = (size_t)g->offs[n];
    g->stage.resize(total * 4);
    for (int32_t i = 0; i < n; ++i) {
      if (!g->counts[i]) continue;
      GHIP(g, hipSetDevice(g->dev[i]));
      GHIP(g, hipMemcpyAsync(g->stage.data() + 4 * (size_t)g->offs[i], sums[i], 16 * (size_t)g->counts[i],
                             hipMemcpyDeviceToHost, g->streams[i]));
      GHIP(g, hipStreamSynchronize(g->streams[i]));
    }
    GHIP(g, hipSetDevice(g->dev[0]));
    GHIP(g, hipMemcpyAsync(g->d_recv, g->stage.data(), total * sizeof(float4), hipMemcpyHostToDevice, g->streams[0]));
  }
  GHIP(g, hipSetDevice(g->dev[0]));
  const uint32_t total = (uint32_t)g->offs[n];
  hipLaunchKernelGGL(k_group_frame, dim3((total + TPB - 1) / TPB), dim3(TPB), 0, g->streams[0],
                     (const float4*)g->d_recv, (const uint32_t*)g->d_idx, total, (float)(spp > 0 ? spp : 1),
                     g->d_frame);
  GHIP(g, hipGetLastError());
  GHIP(g, hipStreamSynchronize(g->streams[0]));
  g->fb_w = params->width;
  g->fb_h = params->height;
  const auto t2 = std::chrono::steady_clock::now();
  g->gather_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
  g->render_ms = std::chrono::duration<double, std::milli>(t2 - t0).count();
  return PT_OK;
}

int pt_group_get_image(pt_group* g, float* rgba, size_t n_floats) {
  if (!g || !rgba) return PT_E_INVALID;
  const size_t npx = (size_t)g->fb_w * g->fb_h;
  if (npx == 0) return gfail(g, PT_E_INVALID, "pt_group_get_image before pt_group_render");
  if (npx * 4 > n_floats) return gfail(g, PT_E_INVALID, "image buffer too small");
  GHIP(g, hipSetDevice(g->dev[0]));
  GHIP(g, hipMemcpy(rgba, g->d_frame, npx * sizeof(float4), hipMemcpyDeviceToHost));
  return PT_OK;
}

int pt_group_timing(const pt_group* g, double* gather_ms, double* render_ms) {
  if (!g) return PT_E_INVALID;
  if (gather_ms) *gather_ms = g->gather_ms;
  if (render_ms) *render_ms = g->render_ms;
  return PT_OK;
}

}  // extern "C"
