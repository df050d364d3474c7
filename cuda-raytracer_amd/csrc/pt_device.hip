// pt_ctx: device context, memory layout and pass orchestration behind pt_api.h.
//
// Replaces CudaRenderer::setup / render / renderFrame / rayIntersect /
// processLevel (src/cudaRenderer.cu:1872-2564) with a wavefront schedule that
// never synchronises with the host inside a batch:
//
//   batch b (N = npix * spp_b paths):
//     k_camera                                 (pass 0 rays: camera)
//     for pass = 0 .. max_bounces + 1:
//       trace(slots):  memset(cnt) ; k_trace_root ; { k_scan_level ; k_trace_level } per level
//       k_shade                                (resolve shadows, shade, emit rays of next pass)
//     k_accum
//
// Ray slots: [0, N) extension rays, [N, 2N) shadow rays of the same paths, so a
// pass traces both at once (the reference traces them in separate passes,
// cu:2499-2533).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kernels/trace.hip"
#include "kernels/shade.hip"
#include "kernels/post.hip"

// k_shade_push lives in pt_shade.hip (its own compile flags)
hipError_t pt_launch_shade_push(int nsh, bool refa, bool xl, unsigned grid, hipStream_t stream, hipEvent_t e0,
                                hipEvent_t e1, const void* S);

using namespace pt;

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

}  // namespace

struct pt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;

  // scene
  bool have_scene = false;
  int n_prims = 0, n_nodes = 0, n_levels = 0;
  std::vector<int32_t> level_start;
  int max_level_nodes = 0;
  bool root_leaf = true;
  bool skip_l1 = false;  // root pass pushes straight into the level-2 queues
  bool two_level = true; // two-level traversal (trace_levels; PT_TWO_LEVEL=0: one level per pass)
  bool leaf_kernel = true;  // k_trace_leaves for the leaf-only levels (PT_LEAF_KERNEL=0: k_trace_level)
  bool real_kernel = true;  // k_trace_real for the real levels of two-level mode (PT_REAL_KERNEL=0: k_trace_level)
  std::vector<char> level_has_leaf;          // levels with a leaf the traversal can reach
  std::vector<std::pair<int, int>> detached;  // (parent, slot) of leaves tested inline by the root pass
  RootTable rt{};        // root pass: inline leaves and queue targets (build_root_table)
  std::vector<pt_node> nodes_host;
  pt_light light{};
  pt_camera camera{};
  // The stored BVH boxes carry a guard band G = 2^-14 M (scene_internal.h
  // box_guard) that keeps the fp32 slab test conservative for ray origins
  // with |coordinates| up to ~180 M (M: the scene's largest coordinate
  // magnitude); camera and query-ray origins beyond origin_bound = 64 M
  // (beyond Scotty3D's farthest camera, ~52 x the scene's half-extent) are
  // refused (PT_E_UNSUPPORTED) rather than risking a culled grazing hit.
  double origin_bound = INFINITY;
  pt_node* d_nodes = nullptr;
  float4* d_prims = nullptr;
  float4* d_prims_ref = nullptr;  // PT_FLAG_REF_ARITH records (ref_prim_records)
  bool has_sphere = false, has_glass = false;
  bool refa = false;              // the current render / intersect runs PT_FLAG_REF_ARITH
  bool tmin = false;              // the current pt_intersect has rays with t_min > 0 (d_tmin)
  float* d_tmin = nullptr;        // their t_min per ray slot
  size_t tmin_cap = 0;
  float4* d_shade = nullptr;  // hit-shading records (SHADE_REC float4 per primitive)
  BsdfRec* d_bsdfs = nullptr;
  pt_light* d_lights = nullptr;  // pt_scene_desc.lights (n_lights > 1)
  uint32_t n_lights = 0;
  float* d_cbox = nullptr;  // single-leaf scenes: boxes of the leaf's primitive pairs, 8 floats each
  float* d_rcbox = nullptr;   // root pass: the inline primitives' clusters (RootTable::cbox, root_clusters)
  float4* d_rcmem = nullptr;  // their member records (RootTable::cmem)
  float4* d_rcmem_ref = nullptr;  // ... as PT_FLAG_REF_ARITH records (RootTable::cmem_ref)
  uint32_t* d_rcinfo = nullptr;  // their member ranges and primitive ids (RootTable::cinfo)
  int nclus = 0;
  uint32_t sph_clmask = 0;  // the single-leaf clusters that hold a sphere (bit c: cluster c)

  // wavefront buffers (sized for N paths = 2N ray slots)
  uint32_t cap_paths = 0;  // paths the buffers hold
  uint32_t cap_spp = 0;    // ray slots per path they hold (2, or 3 under the reference schedule)
  size_t qfactor = 4;      // ray entries per ray slot and parity half (doubles on overflow)
  size_t cap_qfactor = 0;
  float4* d_ray = nullptr;  // 2N ray records (trace.h), RSTRIDE float4 each
  float4 *d_ps0 = nullptr, *d_ps1 = nullptr, *d_ps2 = nullptr, *d_ps3 = nullptr;
  // the second buffer set of the tail compaction (ShadeArgs::compact), and
  // the record buffer the traversal currently reads (null: d_ray)
  float4* d_ray_b = nullptr;
  float4 *d_ps0_b = nullptr, *d_ps1_b = nullptr, *d_ps2_b = nullptr, *d_ps3_b = nullptr;
  uint32_t b_paths = 0, b_spp = 0;  // shape of the second set (allocated at a chunk's first compaction)
  float4* ray_cur = nullptr;
  uint32_t* d_compact = nullptr;  // MAX_COMPACTIONS slot counters
  bool compaction = true;         // PT_COMPACT=0: off
  int compact_pct = 65;           // compact when live slots <= this % of the layout (PT_COMPACT=pct)
  int compact_first = 70;         // the same for the chunk's first compaction (PT_COMPACT_FIRST=pct)
  uint32_t* d_q = nullptr;   // ray-id queues (QREGIONS regions): the root's targets and the levels above entry_level
  size_t qcap = 0;           // ids per region
  int entry_level = 0;       // first level whose queues hold ray entries (build_root_table)
  uint32_t shadow_base = 0xFFFFFFFFu;  // ray slots >= it are shadow rays (pt_render sets N; pt_intersect none)
  float4* d_qe = nullptr;    // ray-entry queues of the levels below the root's targets
  size_t qecap = 0;          // entries per region
  uint32_t* d_cnt = nullptr;
  uint32_t* d_qoff = nullptr;
  uint32_t* d_iprefix = nullptr;
  uint32_t* d_nitems = nullptr;  // one per level
  uint32_t* d_icnt = nullptr;
  uint32_t* d_scan_aux = nullptr;  // multi-workgroup scan: partials + per-node target counts
  int scan_multi_min = 0;          // levels with more nodes use k_scan_count + k_scan_alloc
  int dfs_level = 1 << 20;         // the DFS cut: this real level's rays finish their subtrees depth-first
  unsigned long long* d_rcount = nullptr;  // valid root rays: RCOUNT_SLOTS counters, one 128-B line each
  // the ray and statistics counters as a wavefront chunk started: restored
  // when the chunk is re-run after a queue overflow (its abandoned passes
  // counted rays and visits)
  unsigned long long* d_rcount_bak = nullptr;
  unsigned long long* d_stats_bak = nullptr;
  unsigned long long* d_stats = nullptr;
  uint32_t* d_err = nullptr;
  uint32_t* d_work = nullptr;  // k_path_leaf path-region counters (128 B apart)
  float4* d_res = nullptr;     // per-path radiance of a chunk
  size_t res_cap = 0;
  bool async_pending = false;  // frames queued with PT_FLAG_ASYNC (or a synchronous one's work) not yet waited for
  // Pipelined single-leaf frames (PT_FLAG_ASYNC): a launch's per-path results
  // are summed by the leading workgroups of the next launch (k_path_leaf,
  // ShadeArgs::acc_*) or by flush_sums; acc_on: such sums are pending (job
  // acc_job).  The results alternate between two slots (d_res, d_res_b; res_k
  // the next one), pt_clear between two accumulation buffers while sums or
  // images are pending on the current one, and an image requested before its
  // sums are made (pt_get_image_async) waits in img_job until they are.
  struct AccJob {
    const float4* res;
    float4* dst;
    uint32_t npix, spp;
  } acc_job{};
  bool acc_on = false;
  float4* d_res_b = nullptr;
  size_t res_cap_b = 0;
  int res_k = 0;
  float4* d_accum_b = nullptr;
  struct ImgJob {
    const float4* acc;
    float* rgba;
    float ns;
  } img_job[2]{};
  int n_img = 0;
  int acc_blocks = 64;  // k_path_leaf's leading sum workgroups (env PT_ACC_BLOCKS; a multiple of 8)
  uint4* d_wstate = nullptr;   // per shade workgroup {block next, block end, live slots, shaded vertices}
  uint32_t* d_pool = nullptr;  // POOLS path-block dispensers, CSTRIDE apart
  size_t wstate_cap = 0;
  uint32_t* d_live = nullptr;  // live slots after a pass group (k_live_sum)
  uint32_t* h_poll = nullptr;  // pinned: {live, err} x 2 poll slots
  hipEvent_t ev_poll[2] = {};
  int path_grid[4] = {0, 0, 0, 0};  // resident workgroups of k_path_leaf<1|2, refa>
  int path_regions = 8;             // k_path_leaf path regions / counters (PT_PATH_REGIONS)
  uint32_t path_chunk = 0;  // k_path_leaf's grab size (0: path_chunk_for; env PT_PATH_CHUNK)
  uint32_t chunk_paths = 1u << 28;  // paths per chunk (PT_CHUNK_PATHS; tests force multi-chunk frames)

  // framebuffer
  int fb_w = 0, fb_h = 0, fb_tile = 0, fb_rank = 0, fb_nranks = 0;
  std::vector<uint32_t> pix_of;  // owned pixel slot -> global pixel
  uint32_t* d_pix_of = nullptr;
  // camera-ray culling (cull_pixels): the owned pixels whose camera rays may
  // reach the scene (global pixel index, owned slot), valid for cull_cam and
  // the current framebuffer / scene; the others' camera rays provably miss
  // the root box: radiance 0, counted as cast (host_rays)
  bool cull = true;  // PT_CULL=0: trace every camera ray
  bool cull_valid = false;
  pt_camera cull_cam{};
  std::vector<uint32_t> act_pix, act_slot;
  uint32_t* d_act_pix = nullptr;
  uint32_t* d_act_slot = nullptr;
  uint64_t host_rays = 0;
  float4* d_accum = nullptr;
  float4* d_frame = nullptr;  // row-major frame staged for pt_get_image (k_frame)
  size_t frame_cap = 0;
  // pt_get_image_async: two alternating staged frames, their copies to the
  // host on copy_stream (ev_fr: staged on `stream`, ev_cp: copy done)
  hipStream_t copy_stream = nullptr;
  float4* d_frame_a[2] = {nullptr, nullptr};
  size_t frame_cap_a[2] = {0, 0};
  hipEvent_t ev_fr[2] = {}, ev_cp[2] = {};
  bool cp_queued[2] = {false, false};
  int fidx = 0;
  int32_t samples = 0;

  pt_stats stats{};
  hipEvent_t ev[8] = {};

  // kernel timing with a pool of events, read back once per render
  enum { K_CAM, K_ROOT, K_SCAN, K_LEVEL, K_SHADE, K_ACCUM, K_PATH };
  struct Mark {
    int cls, level;
    size_t e0, e1;
  };
  template <typename K, typename... Args>
  void launch(int cls, int level, K kernel, dim3 grid, dim3 block, Args... args) {
    if (timing) {
      auto e = pair(cls, level);
      hipExtLaunchKernelGGL(kernel, grid, block, 0, stream, e.first, e.second, 0, args...);
    } else {
      hipLaunchKernelGGL(kernel, grid, block, 0, stream, args...);
    }
    if (dbg_sync) sync_check(cls, level, grid.x);
  }
  // PT_DEBUG_SYNC (environment, read at pt_create; a debugging aid): every
  // kernel launch is waited for and a failure reported on stderr with the
  // kernel class, level and grid -- the first kernel that faults, not the
  // next synchronising call
  bool dbg_sync = false;
  void sync_check(int cls, int level, unsigned grid) {
    const hipError_t e = hipStreamSynchronize(stream);
    if (e != hipSuccess)
      fprintf(stderr, "PT_DEBUG_SYNC: kernel class %d level %d grid %u: %s\n", cls, level, grid, hipGetErrorString(e));
  }
  bool timing = false;
  std::vector<hipEvent_t> evpool;
  size_t evn = 0;
  std::vector<Mark> marks;
  // two pool events for one kernel launch; they are handed to
  // hipExtLaunchKernelGGL, which timestamps the dispatch packet itself (no
  // extra barrier packets in the stream)
  std::pair<hipEvent_t, hipEvent_t> pair(int cls, int level) {
    while (evn + 2 > evpool.size()) {
      hipEvent_t e;
      hipEventCreate(&e);
      evpool.push_back(e);
    }
    marks.push_back(Mark{cls, level, evn, evn + 1});
    evn += 2;
    return {evpool[evn - 2], evpool[evn - 1]};
  }
};

#define HIPCHK(ctx, call)                                                                 \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) {                                                               \
      (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                    \
      return PT_E_HIP;                                                                    \
    }                                                                                     \
  } while (0)

static int fail(pt_ctx* ctx, int code, const std::string& m) {
  if (ctx) ctx->err = m;
  return code;
}

// Wait for the frames queued since the last wait (PT_FLAG_ASYNC, and a
// synchronous single-leaf frame's own work) and report their failure: the
// kernel-argument check of k_path_leaf sets ERR_KERNARG in d_err (sticky
// across queued frames: reset only when nothing is pending).
static int flush_sums(pt_ctx* c);
static int serve_images(pt_ctx* c);

// Zero `bytes` (a multiple of 4) on the context's stream (post.hip k_zero_u32:
// not hipMemsetAsync, which waits behind an image copy on the copy stream).
static hipError_t zero_async(pt_ctx* c, void* p, size_t bytes) {
  const uint32_t n = (uint32_t)(bytes / 4);
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_zero_u32, dim3((n + TPB - 1) / TPB), dim3(TPB), 0, c->stream, (uint32_t*)p, n);
  return hipGetLastError();
}
static hipError_t copy_async(pt_ctx* c, void* dst, const void* src, size_t bytes) {
  const uint32_t n = (uint32_t)(bytes / 4);
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_copy_u32, dim3((n + TPB - 1) / TPB), dim3(TPB), 0, c->stream, (const uint32_t*)src,
                     (uint32_t*)dst, n);
  return hipGetLastError();
}
static int drain(pt_ctx* c) {
  if (!c->async_pending) return PT_OK;
  if (int rc = flush_sums(c)) return rc;
  c->async_pending = false;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  uint32_t e = 0;
  HIPCHK(c, hipMemcpy(&e, c->d_err, 4, hipMemcpyDeviceToHost));
  if (e & ERR_KERNARG) return fail(c, PT_E_HIP, "k_path_leaf: ShadeArgs is not the kernel's first argument (light_of<true>)");
  return PT_OK;
}

template <class T>
static int dalloc(pt_ctx* ctx, T** p, size_t count) {
  if (*p) {
    hipFree(*p);
    *p = nullptr;
  }
  if (count == 0) count = 1;
  HIPCHK(ctx, hipMalloc((void**)p, count * sizeof(T)));
  return PT_OK;
}

static void free_all(pt_ctx* c) {
  void* ptrs[] = {c->d_nodes, c->d_prims,  c->d_prims_ref, c->d_shade, c->d_bsdfs,   c->d_lights, c->d_cbox, c->d_rcbox, c->d_rcmem, c->d_rcmem_ref, c->d_rcinfo, c->d_ray,
                  c->d_ps0,    c->d_ps1,     c->d_ps2,     c->d_ps3,     c->d_q,   c->d_qe,   c->d_cnt,
                  c->d_qoff,  c->d_iprefix, c->d_nitems, c->d_icnt, c->d_scan_aux, c->d_rcount, c->d_stats,  c->d_err, c->d_work, c->d_res, c->d_res_b, c->d_accum_b, c->d_wstate, c->d_live, c->d_pool,
                  c->d_pix_of, c->d_accum, c->d_frame, c->d_frame_a[0], c->d_frame_a[1], c->d_tmin, c->d_ray_b, c->d_ps0_b, c->d_ps1_b, c->d_ps2_b,
                  c->d_ps3_b, c->d_compact, c->d_act_pix, c->d_act_slot, c->d_rcount_bak, c->d_stats_bak};
  for (void* p : ptrs)
    if (p) hipFree(p);
}

// Buffers for N paths (spp ray slots each).  Queue halves hold qfactor ids
// per slot: 24 covers the measured scenes (peak_queue_entries); a level that
// would overflow is abandoned on the device, the batch is re-run with twice
// the factor (pathological overlap, e.g. random triangle soups).
// Paths in flight per batch.  Large batches amortise the per-level launches
// (deep levels hold few rays per pass); queue offsets are u32, so both parity
// halves (2 x qfactor x slots ids) must stay below 2^32.
// 36 Mi slots: a power-of-two pool (32 Mi) puts the extension and shadow ray
// records of a path, and its state arrays, a power of two apart and runs 7 %
// slower on CBbunny (HBM channel aliasing); 28-42 Mi all measure within 1.5 %.
static constexpr uint32_t DEFAULT_BATCH_PATHS = 36u << 20;
static constexpr int MAX_COMPACTIONS = 8;  // tail compactions per chunk (slot counters, pt_ctx::d_compact)
// per compaction: CREGIONS slot counters, then the compacted layout's extent
static constexpr uint32_t CBLK = 2 * CREGIONS;
// k_live_sum's output: work left, unclaimed paths, the compaction regions' bounds
static constexpr uint32_t LIVE_WORDS = 2 + CREGIONS;
// paths per chunk: pt_ctx::chunk_paths (per-path radiance buffer: 12 B each);
// POLL_GROUP passes are queued between two reads of the finished-path count
static constexpr int POLL_GROUP = 4;
// ray-id queues hold ID_FACTOR x qfactor ids per ray slot and region (the
// entry queues qfactor entries of 32 B).  Queues live in QREGIONS rotating
// regions: the scan of level l allocates its targets' queues (levels l + 1 and,
// two-level, l + 2) in region l % 3, the root pass in region 0; region l % 3 is
// next written by the scan of level l + 3, after the last reader (level l + 2).
static constexpr size_t ID_FACTOR = 4;
static constexpr size_t QREGIONS = 3;
// Ray entries below the root targets' level measured -3 % on CBbunny and
// +1.5-4 % on the dragon proxy trees (the leaf-heavy levels are bound by the
// leaf loop and the closest-hit atomics, not by the ray gathers): off by default.
static constexpr int ENTRY_LEVEL_DEFAULT = 0;  // (env PT_ENTRY_LEVEL)
static constexpr int SCAN_MULTI_MIN_DEFAULT = 512;  // (env PT_SCAN_MULTI_MIN)
// k_path_leaf's grab size for a launch of M paths over `blocks` resident
// workgroups: a launch's tail is about one chunk's time, and more grabs cost
// counter atomics (DESIGN.md §4 "path grabs"): 512 paths for a whole frame
// (>= 256 paths per resident lane), 256 down to 128 per lane, 128 below (one
// rank's 1/8 share of a 1024^2 x 256 spp frame: 64 per lane)
static uint32_t path_chunk_for(uint32_t M, uint32_t blocks) {
  const uint64_t lanes = (uint64_t)std::max<uint32_t>(1, blocks) * TPB;
  return (uint64_t)M >= 256 * lanes ? 512u : (uint64_t)M >= 96 * lanes ? 256u : 128u;
}

static uint32_t max_batch_paths(const pt_ctx* c, uint32_t slots_per_path) {
  // u32 entry offsets: both halves of the entry queues, and the root's id
  // queues (<= 16 targets x every ray, see root_per_lane)
  const uint64_t a = (1ull << 32) / (QREGIONS * ID_FACTOR * c->qfactor * slots_per_path);
  // every region is as large as the root targets' allocation (root_per_lane:
  // ~nt x every ray slot of the lane, plus the per-workgroup rounding)
  const uint64_t b = (1ull << 32) / (QREGIONS * (uint64_t)(std::max(1, c->rt.nt) + 1) * slots_per_path);
  return (uint32_t)std::min<uint64_t>(std::min(a, b), 0xFFFFFFFFull) & ~4095u;
}

// Per-lane capacity of each root target queue for N paths with spp ray slots
// per path: the root kernel (pt_intersect) pushes <= TILE rays per workgroup
// and lane = item & 7; the fused producers (k_camera_push / k_shade_push)
// push <= spp * TPB rays per workgroup with lane = workgroup & 7.
static size_t root_per_lane(size_t N, size_t spp) {
  const size_t items = (N * spp + TILE - 1) / TILE;
  const size_t blocks = (N + TPB - 1) / TPB;
  return std::max((items + NLANE - 1) / NLANE * TILE, (blocks + NLANE - 1) / NLANE * TPB * spp);
}

// The caller runs N paths of spp slots and must be able to rely on that: the
// buffers always hold at least N x spp.  They keep the larger of the old and
// the requested shape when that fits the u32 queue offsets at the current
// queue factor, else exactly the request (after a queue overflow doubled the
// factor, or a reference-schedule render left 3 slots per path).
static int ensure_paths(pt_ctx* c, uint32_t N, uint32_t spp) {
  if (N <= c->cap_paths && spp <= c->cap_spp && c->qfactor == c->cap_qfactor) return PT_OK;
  if (N > max_batch_paths(c, spp)) return fail(c, PT_E_UNSUPPORTED, "batch too large for u32 queue offsets");
  uint32_t aN = std::max(N, c->cap_paths), aspp = std::max(spp, c->cap_spp);
  if (aN > max_batch_paths(c, aspp)) {
    aN = N;
    aspp = spp;
  }
  N = aN;
  spp = aspp;
  const size_t slots = (size_t)spp * N;
  int rc;
  if ((rc = dalloc(c, &c->d_ray, slots * RSTRIDE))) return rc;
  if ((rc = dalloc(c, &c->d_ps0, N))) return rc;
  if ((rc = dalloc(c, &c->d_ps1, N))) return rc;
  if ((rc = dalloc(c, &c->d_ps2, N))) return rc;
  if (spp > 2 && (rc = dalloc(c, &c->d_ps3, N))) return rc;
  // the tail compaction's second set follows lazily (ensure_compact_set):
  // pt_intersect and single-leaf scenes never compact
  if (c->b_paths) {
    for (float4** p : {&c->d_ray_b, &c->d_ps0_b, &c->d_ps1_b, &c->d_ps2_b, &c->d_ps3_b})
      if (*p) {
        hipFree(*p);
        *p = nullptr;
      }
    c->b_paths = c->b_spp = 0;
  }
  // every root target needs root_per_lane ids per lane (see
  // set_root_child_offsets); the levels below get ray entries: a level needs at
  // most 4x the visits of the level above (the scan's allocation), which
  // qfactor entries per ray slot cover for the scenes measured
  // (peak_queue_entries; an overflowing level re-runs the chunk with 2x)
  const size_t root_need = (size_t)NLANE * std::max(1, c->rt.nt) * root_per_lane(N, spp);
  // a single-leaf tree queues nothing (k_path_leaf / the root pass only)
  c->qcap = c->root_leaf ? NLANE * 64 : std::max(root_need, ID_FACTOR * c->qfactor * slots);
  c->qcap = (c->qcap + NLANE * 64 - 1) / (NLANE * 64) * (NLANE * 64);
  const bool entries = !c->root_leaf && c->entry_level < c->n_levels;
  c->qecap = entries ? c->qfactor * slots : NLANE * 64;
  c->qecap = (c->qecap + NLANE * 64 - 1) / (NLANE * 64) * (NLANE * 64);
  if (QREGIONS * c->qcap >= (1ull << 32) || QREGIONS * c->qecap >= (1ull << 32))
    return fail(c, PT_E_UNSUPPORTED, "batch too large for u32 queue offsets");
  if ((rc = dalloc(c, &c->d_q, QREGIONS * c->qcap))) return rc;
  if ((rc = dalloc(c, &c->d_qe, QREGIONS * c->qecap * QESTRIDE))) return rc;
  c->cap_paths = N;
  c->cap_spp = spp;
  c->cap_qfactor = c->qfactor;
  return PT_OK;
}

// The tail compaction's second slot-buffer set (ray records + path state
// again), in the shape of the first: allocated at the first compaction a
// render decides on.
static int ensure_compact_set(pt_ctx* c) {
  if (c->b_paths == c->cap_paths && c->b_spp == c->cap_spp) return PT_OK;
  const size_t N = c->cap_paths, slots = (size_t)c->cap_spp * N;
  int rc;
  c->b_paths = c->b_spp = 0;
  if ((rc = dalloc(c, &c->d_ray_b, slots * RSTRIDE))) return rc;
  if ((rc = dalloc(c, &c->d_ps0_b, N))) return rc;
  if ((rc = dalloc(c, &c->d_ps1_b, N))) return rc;
  if ((rc = dalloc(c, &c->d_ps2_b, N))) return rc;
  if (c->cap_spp > 2 && (rc = dalloc(c, &c->d_ps3_b, N))) return rc;
  c->b_paths = c->cap_paths;
  c->b_spp = c->cap_spp;
  return PT_OK;
}

// The root pass's table.  Small leaves among the root's children (and, when
// level 1 is skipped, grandchildren) are tested inline by the ray producers,
// up to PT_INLINE_MAX primitives in all (default 32; 0 disables).  Level 1 is
// skipped when every other child of the root is interior (PT_NO_SKIP_L1=1
// disables it): the producers then test the grandchild boxes directly (boxes
// are conservative for their subtrees, so no ray is lost).
template <int W>
static void box_row(float (&b)[6][W], int i, const pt_node& parent, int k) {
  b[0][i] = parent.bmin_x[k];
  b[1][i] = parent.bmax_x[k];
  b[2][i] = parent.bmin_y[k];
  b[3][i] = parent.bmax_y[k];
  b[4][i] = parent.bmin_z[k];
  b[5][i] = parent.bmax_z[k];
}

// Primitive boxes and guard-banded cluster boxes (the candidate loops of
// k_path_leaf and root_pass).
static void prim_box(const pt_prim& p, double* lo, double* hi, bool& sph) {
  const float* q = p.q;
  uint32_t meta;
  memcpy(&meta, &q[3], 4);
  sph = (meta >> 28) == PT_PRIM_SPHERE;
  for (int k = 0; k < 3; ++k) {
    lo[k] = sph ? (double)q[k] - q[4] : std::min({(double)q[k], (double)q[4 + k], (double)q[8 + k]});
    hi[k] = sph ? (double)q[k] + q[4] : std::max({(double)q[k], (double)q[4 + k], (double)q[8 + k]});
  }
}
static double half_area(const double* lo, const double* hi) {
  const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
  return x * y + y * z + z * x;
}
// {xmin, xmax, ymin, ymax, zmin, zmax} (box_hit's order), widened by G and
// rounded outward to fp32
static void push_guarded_box(std::vector<float>& cb, const double* lo, const double* hi, double G) {
  for (int k = 0; k < 3; ++k) {
    float fl = (float)(lo[k] - G), fh = (float)(hi[k] + G);
    if ((double)fl > lo[k] - G) fl = std::nextafter(fl, -INFINITY);
    if ((double)fh < hi[k] + G) fh = std::nextafter(fh, INFINITY);
    cb.push_back(fl);
    cb.push_back(fh);
  }
}
static float int_bits(int32_t v) {
  float f;
  memcpy(&f, &v, 4);
  return f;
}

// The root pass's candidate clusters (RootTable::nc, PT_ROOT_CLUSTER): the
// inline leaves' primitives grouped bottom-up, merging the two clusters whose
// union lowers the expected cost most, cost(C) = 1 box test + 2 n(C) A(C) / A
// (a primitive test ~ 2 box tests, entered by the rays in proportion to the
// box's surface area A(C) against the whole set's A), at most 8 members: a
// Cornell wall's two triangles become one cluster, a far light or a few small
// triangles next to each other another.  Boxes widened by G as the BVH's.
static int root_clusters(pt_ctx* c, const pt_scene_desc* s, double G) {
  RootTable& T = c->rt;
  T.nc = T.nc_shadow = 0;
  T.cbox = nullptr;
  T.cmem = T.cmem_ref = nullptr;
  T.cinfo = nullptr;
  if (c->root_leaf || T.ni == 0 || getenv("PT_NO_ROOT_CLUSTER")) return PT_OK;
  struct Cl {
    double lo[3], hi[3];
    std::vector<int> mem;
  };
  std::vector<Cl> cl;
  for (int i = 0; i < T.ni; ++i)
    for (int k = 0; k < T.icount[i]; ++k) {
      Cl x;
      bool sph;
      prim_box(s->prims[T.istart[i] + k], x.lo, x.hi, sph);
      x.mem = {T.istart[i] + k};
      cl.push_back(x);
    }
  if (cl.empty() || cl.size() > (size_t)ROOT_CL_MAX) return PT_OK;
  double alo[3] = {INFINITY, INFINITY, INFINITY}, ahi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (const Cl& x : cl)
    for (int k = 0; k < 3; ++k) {
      alo[k] = std::min(alo[k], x.lo[k]);
      ahi[k] = std::max(ahi[k], x.hi[k]);
    }
  const double A = half_area(alo, ahi);
  if (!(A > 0.0)) return PT_OK;
  auto cost = [&](const double* lo, const double* hi, size_t n) { return 1.0 + 2.0 * (double)n * half_area(lo, hi) / A; };
  for (;;) {
    double best = 0.0;
    size_t ba = 0, bb = 0;
    for (size_t a = 0; a < cl.size(); ++a)
      for (size_t b = a + 1; b < cl.size(); ++b) {
        const size_t n = cl[a].mem.size() + cl[b].mem.size();
        if (n > 8) continue;
        double lo[3], hi[3];
        for (int k = 0; k < 3; ++k) {
          lo[k] = std::min(cl[a].lo[k], cl[b].lo[k]);
          hi[k] = std::max(cl[a].hi[k], cl[b].hi[k]);
        }
        const double save = cost(cl[a].lo, cl[a].hi, cl[a].mem.size()) + cost(cl[b].lo, cl[b].hi, cl[b].mem.size()) -
                            cost(lo, hi, n);
        if (save > best) {
          best = save;
          ba = a;
          bb = b;
        }
      }
    if (best <= 0.0) break;
    for (int k = 0; k < 3; ++k) {
      cl[ba].lo[k] = std::min(cl[ba].lo[k], cl[bb].lo[k]);
      cl[ba].hi[k] = std::max(cl[ba].hi[k], cl[bb].hi[k]);
    }
    cl[ba].mem.insert(cl[ba].mem.end(), cl[bb].mem.begin(), cl[bb].mem.end());
    cl.erase(cl.begin() + (long)bb);
  }
  std::vector<float> cb;
  std::vector<uint32_t> info(2 * ROOT_CL_MAX, 0u);
  uint32_t nm = 0;
  for (size_t k = 0; k < cl.size(); ++k) {
    push_guarded_box(cb, cl[k].lo, cl[k].hi, G);
    cb.push_back(0.0f);
    cb.push_back(0.0f);
    info[k] = nm | (uint32_t)cl[k].mem.size() << 16;
    for (int p : cl[k].mem) info[ROOT_CL_MAX + nm++] = (uint32_t)p;
  }
  int rc;
  if ((rc = dalloc(c, &c->d_rcbox, cb.size()))) return rc;
  if ((rc = dalloc(c, &c->d_rcmem, 4 * ROOT_CL_MAX))) return rc;
  if ((rc = dalloc(c, &c->d_rcinfo, 2 * ROOT_CL_MAX))) return rc;
  if ((rc = dalloc(c, &c->d_rcmem_ref, 6 * ROOT_CL_MAX))) return rc;
  HIPCHK(c, hipMemset(c->d_rcmem_ref, 0, 6 * ROOT_CL_MAX * sizeof(float4)));
  HIPCHK(c, hipMemcpy(c->d_rcbox, cb.data(), cb.size() * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_rcinfo, info.data(), info.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemset(c->d_rcmem, 0, 4 * ROOT_CL_MAX * sizeof(float4)));
  for (uint32_t m = 0; m < nm; ++m) {
    HIPCHK(c, hipMemcpy(c->d_rcmem + 4 * m, c->d_prims + (size_t)4 * info[ROOT_CL_MAX + m], 4 * sizeof(float4),
                        hipMemcpyDeviceToDevice));
    HIPCHK(c, hipMemcpy(c->d_rcmem_ref + 6 * m, c->d_prims_ref + (size_t)6 * info[ROOT_CL_MAX + m],
                        6 * sizeof(float4), hipMemcpyDeviceToDevice));
  }
  T.nc = (int)cl.size();
  T.nc_shadow = getenv("PT_NO_ROOT_CLUSTER_SHADOW") ? 0 : T.nc;
  T.cbox = c->d_rcbox;
  T.cmem = c->d_rcmem;
  T.cmem_ref = c->d_rcmem_ref;
  T.cinfo = c->d_rcinfo;
  return PT_OK;
}

static void build_root_table(pt_ctx* c) {
  RootTable& T = c->rt;
  memset(&T, 0, sizeof(T));
  c->skip_l1 = false;
  c->detached.clear();  // (before the early return: a single-leaf scene keeps none of the last scene's)
  if (c->root_leaf) return;
  const char* e = getenv("PT_INLINE_MAX");
  int budget = e ? atoi(e) : 32;
  const std::vector<pt_node>& nd = c->nodes_host;
  auto try_inline = [&](int parent, int k) {
    const pt_node& leaf = nd[nd[parent].child[k]];
    if (leaf.prim_count <= 0 || leaf.prim_count > budget || T.ni >= MAX_INLINE_LEAVES) return false;
    T.ibox[T.ni] = parent * 4 + k;
    box_row(T.ib, T.ni, nd[parent], k);
    T.istart[T.ni] = leaf.prim_start;
    T.icount[T.ni] = leaf.prim_count;
    T.ni++;
    budget -= leaf.prim_count;
    return true;
  };
  auto add_target = [&](int parent, int k) {
    T.tbox[T.nt] = parent * 4 + k;
    box_row(T.tb, T.nt, nd[parent], k);
    T.tnode[T.nt] = nd[parent].child[k];
    T.nt++;
  };
  std::vector<int> rest;  // root slots neither empty nor inline
  for (int k = 0; k < 4; ++k)
    if (nd[0].child[k] >= 0 && !try_inline(0, k)) rest.push_back(k);
  bool skip = c->n_levels >= 3 && !getenv("PT_NO_SKIP_L1") && !rest.empty();
  for (int k : rest)
    if (nd[nd[0].child[k]].prim_count > 0) skip = false;
  for (int k : rest) {
    if (!skip) {
      add_target(0, k);
      continue;
    }
    const int ch = nd[0].child[k];
    for (int g = 0; g < 4; ++g)
      if (nd[ch].child[g] >= 0 && !try_inline(ch, g)) add_target(ch, g);
  }
  c->skip_l1 = skip;
  // Hot small leaves one level deeper (children of the root's targets): a
  // leaf of <= 4 primitives whose box has >= PT_INLINE_SA (default 5 %) of
  // the root's surface area is tested inline too (CBbunny: a 2-triangle leaf
  // entered by 21 % of all rays, 10.8 ms per frame as a queued level) and
  // detached from its parent in the device's copy of the tree, so the
  // traversal never queues it (c->detached)
  if (skip) {
    auto sa = [](const pt_node& n, int k) {
      const double dx = n.bmax_x[k] - n.bmin_x[k], dy = n.bmax_y[k] - n.bmin_y[k], dz = n.bmax_z[k] - n.bmin_z[k];
      return 2.0 * (dx * dy + dy * dz + dz * dx);
    };
    double rsa = 0;
    for (int k = 0; k < 4; ++k)
      if (nd[0].child[k] >= 0) rsa += sa(nd[0], k);
    const char* se = getenv("PT_INLINE_SA");
    const double min_ratio = se ? atof(se) : 0.05;
    std::vector<std::pair<double, std::pair<int, int>>> cand;  // (area ratio, (parent, slot))
    for (int t = 0; t < T.nt; ++t) {
      const int par = T.tnode[t];
      for (int k = 0; k < 4; ++k) {
        const int ch = nd[par].child[k];
        if (ch < 0 || nd[ch].prim_count <= 0 || nd[ch].prim_count > 4 || rsa <= 0) continue;
        const double r = sa(nd[par], k) / rsa;
        if (r >= min_ratio) cand.push_back({r, {par, k}});
      }
    }
    std::sort(cand.begin(), cand.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    for (const auto& cd : cand)
      if (try_inline(cd.second.first, cd.second.second)) c->detached.push_back(cd.second);
  }
  // two-level traversal (default; PT_TWO_LEVEL=0 restores one level per pass)
  const char* tl = getenv("PT_TWO_LEVEL");
  c->two_level = !(tl && atoi(tl) == 0);
  const char* lk = getenv("PT_LEAF_KERNEL");
  c->leaf_kernel = !(lk && atoi(lk) == 0);
  const char* rk = getenv("PT_REAL_KERNEL");
  c->real_kernel = !(rk && atoi(rk) == 0);
  // ray entries from PT_ENTRY_LEVEL levels below the root's targets on (0: ids
  // only; the two-level push writes ids)
  const char* el = getenv("PT_ENTRY_LEVEL");
  const int eoff = el ? atoi(el) : ENTRY_LEVEL_DEFAULT;
  c->entry_level = (eoff > 0 && !c->two_level) ? (skip ? 2 : 1) + eoff : 1 << 20;
  // levels wider than this scan with many workgroups (PT_SCAN_MULTI_MIN nodes)
  const char* sm = getenv("PT_SCAN_MULTI_MIN");
  c->scan_multi_min = sm ? atoi(sm) : SCAN_MULTI_MIN_DEFAULT;
  // depth-first below the k-th real level (PT_DFS_LEVEL=k, 0 = the root
  // targets' level; negative: off), when its per-lane stack fits the deepest
  // subtree (3 entries per level below the cut)
  const char* dl = getenv("PT_DFS_LEVEL");
  const int dk = dl ? atoi(dl) : -1;
  c->dfs_level = 1 << 20;
  if (dk >= 0 && !c->root_leaf) {
    const int l0 = skip ? 2 : 1;
    const int ls = l0 + (c->two_level ? 2 : 1) * dk;
    if (ls < c->n_levels && 3 * (c->n_levels - 1 - ls) + 1 <= DFS_STACK) c->dfs_level = ls;
  }
}

// Queue offsets of the root's targets: each gets root_per_lane ids in every
// lane of the id queue.
static int set_root_child_offsets(pt_ctx* c) {
  if (c->root_leaf) return PT_OK;
  const size_t per_lane = root_per_lane(c->cap_paths, c->cap_spp);
  const size_t lanecap = c->qcap / NLANE;
  const pt_node& root = c->nodes_host[0];
  // targets: nodes of level 1 or, when level 1 is skipped, of level 2
  std::vector<int> targets(c->rt.tnode, c->rt.tnode + c->rt.nt);
  if (targets.size() * per_lane > lanecap) return fail(c, PT_E_OVERFLOW, "root queue capacity");
  const size_t half = 0;  // region 0 (the root pass's allocation)
  // ordered on the context's (non-blocking) stream behind any work in flight
  std::vector<uint32_t> off(targets.size() * NLANE);
  for (size_t jj = 0; jj < targets.size(); ++jj)
    for (int s = 0; s < NLANE; ++s) off[jj * NLANE + s] = (uint32_t)(half + (size_t)s * lanecap + jj * per_lane);
  for (size_t jj = 0; jj < targets.size(); ++jj)
    HIPCHK(c, hipMemcpyAsync(c->d_qoff + (size_t)targets[jj] * NLANE, &off[jj * NLANE], NLANE * 4,
                             hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PT_OK;
}

static TraceArgs trace_args(pt_ctx* c) {
  TraceArgs A;
  A.nodes = c->d_nodes;
  A.prims = c->refa ? c->d_prims_ref : c->d_prims;
  A.ray = c->ray_cur ? c->ray_cur : c->d_ray;
  A.cnt = c->d_cnt;
  A.qoff = c->d_qoff;
  A.q = c->d_q;
  A.qe = c->d_qe;
  A.shadow_base = c->shadow_base;
  A.tmin = c->tmin ? c->d_tmin : nullptr;
  A.dbg_nslots = (uint32_t)std::min<size_t>((size_t)c->cap_paths * c->cap_spp, 0xFFFFFFFFu);
  A.dbg_nnodes = (uint32_t)c->n_nodes;
  A.dbg_qids = (uint64_t)QREGIONS * c->qcap;
  A.dbg_nprims = (uint32_t)c->n_prims;
  return A;
}

// The per-level part of a traversal pass: { k_scan_level ; k_trace_level } for
// every level below the root's targets (the root pass itself is k_trace_root
// or fused into k_camera_push / k_shade_push).
static int trace_levels(pt_ctx* c) {
  TraceArgs A = trace_args(c);
  // Two-level traversal: the root targets' level l0 and every second level
  // below it are "real" -- their interior nodes push rays straight to their
  // leaf children and to their grandchildren; interior nodes of the levels in
  // between are never queued, so those levels run only for their leaves (and
  // not at all when they have none).  One ray gather, one queue round trip and
  // one scan per two BVH levels.
  const int l0 = c->skip_l1 ? 2 : 1;  // the root targets' level: its queues hold ids
  for (int l = l0; l < c->n_levels; ++l) {
    const bool real = !c->two_level || ((l - l0) & 1) == 0;
    if (!real && !c->level_has_leaf[l]) continue;
    const bool dfs = l == c->dfs_level;
    LevelArgs L;
    // the DFS level allocates no targets (real = 0) and runs wave items
    L.real = real && !dfs;
    L.two_level = (c->two_level && real) || dfs;
    L.first = c->level_start[l];
    L.nl = c->level_start[l + 1] - c->level_start[l];
    L.maxln = c->max_level_nodes;
    L.iprefix = c->d_iprefix;
    L.iprefix_w = c->d_iprefix;
    L.icnt = c->d_icnt;
    L.icnt_w = c->d_icnt;
    L.nitems = c->d_nitems + l;
    L.nitems_w = c->d_nitems + l;
    L.mode = c->d_nitems + c->n_levels + l;
    L.mode_w = c->d_nitems + c->n_levels + l;
    // levels above entry_level take ray ids, the others ray entries
    L.ids = l < c->entry_level;
    L.out_ids = l + 1 < c->entry_level;
    const size_t lanecap = (L.out_ids ? c->qcap : c->qecap) / NLANE;
    const uint32_t out_base = (uint32_t)((size_t)(l % QREGIONS) * (L.out_ids ? c->qcap : c->qecap));
    const int G = (L.nl + SCAN_WG - 1) / SCAN_WG;
    if (L.nl > c->scan_multi_min && G <= SCAN_MAXG) {
      c->launch(pt_ctx::K_SCAN, l, k_scan_count, dim3(G), dim3(SCAN_WG), A, L, c->d_scan_aux);
      c->launch(pt_ctx::K_SCAN, l, k_scan_alloc, dim3(G), dim3(SCAN_WG), A, L, (const uint32_t*)c->d_scan_aux,
                (uint32_t)lanecap, out_base, c->d_stats, l, c->d_err);
    } else {
      c->launch(pt_ctx::K_SCAN, l, k_scan_level, dim3(1), dim3(1024), A, L, (uint32_t)lanecap, out_base,
                c->d_stats, l, c->d_err);
    }
    // a level between two real ones holds only leaf rays: the leaf-only kernel
    // (fewer registers, more waves per SIMD); PT_LEAF_KERNEL=0 disables it
    // (a real level's leaf items stay in the shared kernel: running them in a
    // second, leaf-only launch that skips the other items measured -3 to -5 %)
    const bool leaves = !real && c->leaf_kernel;
    // (a real level of the two-level traversal: wave items only, k_trace_real)
    const bool wave_only = L.two_level && c->real_kernel;
    auto kl = c->tmin ? (c->refa ? (leaves ? k_trace_leaves<true, true> : wave_only ? k_trace_real<true, true>
                                                                                   : k_trace_level<true, true>)
                                 : (leaves ? k_trace_leaves<false, true> : wave_only ? k_trace_real<false, true>
                                                                                     : k_trace_level<false, true>))
              : (c->refa ? (leaves ? k_trace_leaves<true> : wave_only ? k_trace_real<true> : k_trace_level<true>)
                         : (leaves ? k_trace_leaves<false> : wave_only ? k_trace_real<false> : k_trace_level<false>));
    if (dfs) {
      auto kd = c->tmin ? (c->refa ? k_trace_dfs<true, true> : k_trace_dfs<false, true>)
                        : (c->refa ? k_trace_dfs<true> : k_trace_dfs<false>);
      c->launch(pt_ctx::K_LEVEL, l, kd, dim3(LEVEL_GRID), dim3(TPB), A, L);
      break;  // nothing is queued below the cut
    }
    c->launch(pt_ctx::K_LEVEL, l, kl, dim3(LEVEL_GRID), dim3(TPB), A, L);
  }
  HIPCHK(c, hipGetLastError());
  c->stats.passes++;
  return PT_OK;
}

// One breadth-first traversal pass over ray slots [r0, r1) (pt_intersect).
static int trace_pass(pt_ctx* c, uint32_t r0, uint32_t r1) {
  if (r1 <= r0) return PT_OK;
  TraceArgs A = trace_args(c);
  const uint32_t items = (r1 - r0 + TILE - 1) / TILE;
  // the (node, lane) counters are zero here: each level's scan re-zeroes them
  // after taking its snapshot (pt_load_scene zeroes them once)
  auto kr = c->tmin ? (c->refa ? k_trace_root<true, true> : k_trace_root<false, true>)
                    : (c->refa ? k_trace_root<true> : k_trace_root<false>);
  c->launch(pt_ctx::K_ROOT, 0, kr, dim3(items), dim3(TPB), A, c->rt, r0, r1, c->d_rcount);
  if (c->root_leaf) {
    HIPCHK(c, hipGetLastError());
    c->stats.passes++;
    return PT_OK;
  }
  return trace_levels(c);
}

// Fold the recorded kernel intervals into the stats (after the stream is idle).
static void collect_marks(pt_ctx* c) {
  for (const auto& m : c->marks) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, c->evpool[m.e0], c->evpool[m.e1]) != hipSuccess) continue;
    switch (m.cls) {
      case pt_ctx::K_ROOT:
        c->stats.ms_root += ms;
        c->stats.root_launches++;
        c->stats.ms_trace += ms;
        break;
      case pt_ctx::K_SCAN:
        c->stats.ms_scan += ms;
        if (m.level < 16) c->stats.ms_scan_level[m.level] += ms;
        c->stats.ms_trace += ms;
        break;
      case pt_ctx::K_LEVEL:
        if (m.level < 16) {
          c->stats.ms_level[m.level] += ms;
          c->stats.level_launches[m.level]++;
        }
        c->stats.ms_trace += ms;
        break;
      case pt_ctx::K_PATH:
        c->stats.ms_path += ms;
        c->stats.path_launches++;
        break;
      case pt_ctx::K_SHADE:
        c->stats.ms_shade_push += ms;
        c->stats.shade_launches++;
        c->stats.ms_shade += ms;
        break;
      default:
        c->stats.ms_shade += ms;
        break;
    }
  }
  c->marks.clear();
  c->evn = 0;
}

static int read_device_stats(pt_ctx* c) {
  unsigned long long st[STAT_COUNT];
  uint32_t e = 0;
  unsigned long long rl[RCOUNT_SLOTS * 16];
  HIPCHK(c, hipMemcpyAsync(st, c->d_stats, sizeof(st), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(rl, c->d_rcount, sizeof(rl), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(&e, c->d_err, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  unsigned long long R = 0;
  unsigned long long nt[3] = {0, 0, 0};  // PT_FLAG_COUNT_TESTS: words 1-3 of each counter line
  for (int s = 0; s < RCOUNT_SLOTS; ++s) {
    R += rl[s * 16];
    for (int j = 0; j < 3; ++j) nt[j] += rl[s * 16 + 1 + j];
  }
  c->stats.prim_tests_tri = nt[0];
  c->stats.prim_tests_sph = nt[1];
  c->stats.cluster_box_tests = nt[2];
  c->stats.rays = R + c->host_rays;
  c->stats.culled_rays = c->host_rays;
  c->stats.visits = st[STAT_V] + R;
  st[STAT_LV0] += R;
  c->stats.peak_queue_entries = st[STAT_PEAKQ];
  c->stats.shaded = st[STAT_SHADED];
  for (int l = 0; l < 16; ++l) {
    c->stats.level_visits[l] = st[STAT_LV0 + l];
    c->stats.level_leaf_visits[l] = st[STAT_LEAF0 + l];
    c->stats.level_items[l] = st[STAT_ITEMS0 + l];
  }
  if (c->root_leaf) c->stats.level_leaf_visits[0] = st[STAT_LV0];
  c->stats.n_levels = c->n_levels;
  if (e) return fail(c, PT_E_OVERFLOW, "ray queue capacity exceeded");
  return PT_OK;
}

// PT_FLAG_REF_ARITH primitive records (trace.hip tri_test<true>): the
// operands of intersectRayTriangle computed as the reference does per call
// (cu:223-237) in the kernels' arithmetic -- N = cross(v1 - v0, v2 - v0) and
// dot(N, v0) as the FMA chains of ptmath.h -- and the edges e0 = v1 - v0,
// e1 = v2 - v1, e2 = v0 - v2 in the slots of the edge normals.  Spheres are
// copied (pt_render refuses them under PT_FLAG_REF_ARITH).
static std::vector<pt_prim> ref_prim_records(const pt_scene_desc* s) {
  std::vector<pt_prim> out(s->prims, s->prims + s->n_prims);
  for (int i = 0; i < s->n_prims; ++i) {
    float* q = out[i].q;
    uint32_t meta;
    memcpy(&meta, &q[3], 4);
    if ((meta >> 28) != PT_PRIM_TRIANGLE) continue;
    const float v0[3] = {q[0], q[1], q[2]}, v1[3] = {q[4], q[5], q[6]}, v2[3] = {q[8], q[9], q[10]};
    float e0[3], v02[3], e1[3], e2[3];
    for (int k = 0; k < 3; ++k) {
      e0[k] = v1[k] - v0[k];
      v02[k] = v2[k] - v0[k];
      e1[k] = v2[k] - v1[k];
      e2[k] = v0[k] - v2[k];
    }
    const float N[3] = {std::fma(e0[1], v02[2], -(e0[2] * v02[1])), std::fma(e0[2], v02[0], -(e0[0] * v02[2])),
                        std::fma(e0[0], v02[1], -(e0[1] * v02[0]))};
    q[7] = std::fma(N[2], v0[2], std::fma(N[1], v0[1], N[0] * v0[0]));
    q[11] = e0[0];
    q[12] = N[0];
    q[13] = N[1];
    q[14] = N[2];
    q[15] = e0[1];
    q[16] = e1[0];
    q[17] = e1[1];
    q[18] = e1[2];
    q[19] = e0[2];
    q[20] = e2[0];
    q[21] = e2[1];
    q[22] = e2[2];
    q[23] = 0.0f;
  }
  return out;
}

// The default arithmetic's records (trace.hip, 4 float4 per primitive): a
// triangle's Baldwin-Weber rows U, V, W and {meta, 0, 0, 0}.  From the fp32
// vertices A, B, C in double: e1 = B - A, e2 = C - A, n = e1 x e2 (component
// by component, in this order), and with k the axis of n's largest magnitude
// (x if |n.x| > |n.y| and |n.x| > |n.z|, else y if |n.y| > |n.z|, else z)
// the rows that map v -> (u, v, w) with w = dot(n, v - A) / n_k; each entry
// one double division, rounded once to fp32 (oracle/ptoracle.c bw_rows
// restates the same operations).  A sphere: {centre, 0}, {radius,
// radius^2, 0, 0}, 0, {meta, 0, 0, 0}.
static void bw_rows(const float* q, double r[12]) {
  const double A[3] = {q[0], q[1], q[2]}, B[3] = {q[4], q[5], q[6]}, C[3] = {q[8], q[9], q[10]};
  double e1[3], e2[3], n[3];
  for (int k = 0; k < 3; ++k) {
    e1[k] = B[k] - A[k];
    e2[k] = C[k] - A[k];
  }
  n[0] = e1[1] * e2[2] - e1[2] * e2[1];
  n[1] = e1[2] * e2[0] - e1[0] * e2[2];
  n[2] = e1[0] * e2[1] - e1[1] * e2[0];
  const double an = n[0] * A[0] + n[1] * A[1] + n[2] * A[2];
  if (std::fabs(n[0]) > std::fabs(n[1]) && std::fabs(n[0]) > std::fabs(n[2])) {
    const double x = n[0];
    const double rr[12] = {0, e2[2] / x, -e2[1] / x, (C[1] * A[2] - C[2] * A[1]) / x,
                           0, -e1[2] / x, e1[1] / x, -(B[1] * A[2] - B[2] * A[1]) / x,
                           1, n[1] / x, n[2] / x, -an / x};
    memcpy(r, rr, sizeof rr);
  } else if (std::fabs(n[1]) > std::fabs(n[2])) {
    const double y = n[1];
    const double rr[12] = {-e2[2] / y, 0, e2[0] / y, (C[2] * A[0] - C[0] * A[2]) / y,
                           e1[2] / y, 0, -e1[0] / y, -(B[2] * A[0] - B[0] * A[2]) / y,
                           n[0] / y, 1, n[2] / y, -an / y};
    memcpy(r, rr, sizeof rr);
  } else {
    const double z = n[2];
    const double rr[12] = {e2[1] / z, -e2[0] / z, 0, (C[0] * A[1] - C[1] * A[0]) / z,
                           -e1[1] / z, e1[0] / z, 0, -(B[0] * A[1] - B[1] * A[0]) / z,
                           n[0] / z, n[1] / z, 1, -an / z};
    memcpy(r, rr, sizeof rr);
  }
}
static std::vector<float4> bw_prim_records(const pt_scene_desc* s) {
  std::vector<float4> out((size_t)s->n_prims * prim_stride<false>(), make_float4(0.f, 0.f, 0.f, 0.f));
  for (int i = 0; i < s->n_prims; ++i) {
    const float* q = s->prims[i].q;
    uint32_t meta;
    memcpy(&meta, &q[3], 4);
    float4* o = &out[(size_t)i * prim_stride<false>()];
    if ((meta >> 28) == PT_PRIM_SPHERE) {
      o[0] = make_float4(q[0], q[1], q[2], 0.f);
      o[1] = make_float4(q[4], q[5], 0.f, 0.f);
    } else {
      double r[12];
      bw_rows(q, r);
      // U and V interleaved (trace.hip bw_uv)
      o[0] = make_float4((float)r[0], (float)r[4], (float)r[1], (float)r[5]);
      o[1] = make_float4((float)r[2], (float)r[6], (float)r[3], (float)r[7]);
      o[2] = make_float4((float)r[8], (float)r[9], (float)r[10], (float)r[11]);
    }
    o[3] = make_float4(q[3], 0.f, 0.f, 0.f);
  }
  return out;
}

// Camera-ray culling.  A camera ray of pixel (row, col) is
//   dir ~ kx left + ky up + look_at,  kx = (col + v) / W - 1/2,
//   ky = -((row + u) / H - 1/2),  u, v in [0, 1)          (camera_dir, cu:338-354)
// from the camera origin.  Each corner X of the root node's box (the union
// of its children's boxes, guard band included) is solved for the (kx, ky, s)
// with X - origin = s (kx left + ky up + look_at), in double; when every corner
// lies in front (s > 0), the box's projection -- the convex hull of the
// corners' (kx, ky) -- lies in their bounding rectangle.  A pixel whose whole
// footprint lies outside that rectangle, widened by 4 pixels (the device's
// fp32 directions deviate by ~1e-7 from the exact ones; a pixel is ~1e-3),
// has camera rays that miss the root box, hence every primitive: its paths
// end at the camera vertex with radiance 0, exactly what tracing them gives
// (no emission from a miss, no shadow or extension ray), so it is left out of
// the path space and its camera rays are counted as cast.  Returns false (no
// culling) for a single-leaf tree, a box that reaches behind the camera, or a
// degenerate camera basis.
static bool cull_rect(const pt_ctx* c, int W, int H, double& x0, double& x1, double& y0, double& y1) {
  if (c->root_leaf || c->nodes_host.empty()) return false;
  const pt_node& r = c->nodes_host[0];
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int k = 0; k < 4; ++k) {
    if (r.child[k] < 0) continue;
    lo[0] = std::min(lo[0], (double)r.bmin_x[k]);
    hi[0] = std::max(hi[0], (double)r.bmax_x[k]);
    lo[1] = std::min(lo[1], (double)r.bmin_y[k]);
    hi[1] = std::max(hi[1], (double)r.bmax_y[k]);
    lo[2] = std::min(lo[2], (double)r.bmin_z[k]);
    hi[2] = std::max(hi[2], (double)r.bmax_z[k]);
  }
  if (!(lo[0] <= hi[0])) return false;
  const pt_camera& cam = c->camera;
  // columns left, up, look_at; solve A y = X - origin by Cramer's rule
  const double A[3][3] = {{cam.left[0], cam.up[0], cam.look_at[0]},
                          {cam.left[1], cam.up[1], cam.look_at[1]},
                          {cam.left[2], cam.up[2], cam.look_at[2]}};
  auto det3 = [](const double m[3][3]) {
    return m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) - m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
           m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
  };
  const double D = det3(A);
  if (!(std::fabs(D) > 1e-12)) return false;
  x0 = y0 = INFINITY;
  x1 = y1 = -INFINITY;
  for (int k = 0; k < 8; ++k) {
    const double X[3] = {((k & 1) ? hi[0] : lo[0]) - cam.origin[0], ((k & 2) ? hi[1] : lo[1]) - cam.origin[1],
                         ((k & 4) ? hi[2] : lo[2]) - cam.origin[2]};
    double y[3];
    for (int j = 0; j < 3; ++j) {
      double M[3][3];
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) M[a][b] = b == j ? X[a] : A[a][b];
      y[j] = det3(M) / D;
    }
    const double s = y[2];
    if (!(s > 1e-9 * (std::fabs(X[0]) + std::fabs(X[1]) + std::fabs(X[2]) + 1e-30))) return false;
    x0 = std::min(x0, y[0] / s);
    x1 = std::max(x1, y[0] / s);
    y0 = std::min(y0, y[1] / s);
    y1 = std::max(y1, y[1] / s);
  }
  const double mx = 4.0 / W + 1e-6 * (std::fabs(x0) + std::fabs(x1)), my = 4.0 / H + 1e-6 * (std::fabs(y0) + std::fabs(y1));
  x0 -= mx;
  x1 += mx;
  y0 -= my;
  y1 += my;
  return true;
}

// The active (not culled) owned pixels for the current camera and frame
// (cached until either changes); act_slot[i] is pixel act_pix[i]'s owned slot.
static int cull_pixels(pt_ctx* c, int W, int H) {
  if (c->cull_valid && !memcmp(&c->cull_cam, &c->camera, sizeof(pt_camera))) return PT_OK;
  c->act_pix.clear();
  c->act_slot.clear();
  double x0, x1, y0, y1;
  const bool on = c->cull && cull_rect(c, W, H, x0, x1, y0, y1);
  for (size_t i = 0; i < c->pix_of.size(); ++i) {
    const uint32_t g = c->pix_of[i];
    if (on) {
      const int row = (int)(g / (uint32_t)W), col = (int)(g % (uint32_t)W);
      const double kx0 = (double)col / W - 0.5, kx1 = (double)(col + 1) / W - 0.5;
      const double ky0 = -((double)(row + 1) / H - 0.5), ky1 = -((double)row / H - 0.5);
      if (kx1 < x0 || kx0 > x1 || ky1 < y0 || ky0 > y1) continue;  // the whole footprint misses
    }
    c->act_pix.push_back(g);
    c->act_slot.push_back((uint32_t)i);
  }
  int rc;
  if ((rc = dalloc(c, &c->d_act_pix, std::max<size_t>(1, c->act_pix.size())))) return rc;
  if ((rc = dalloc(c, &c->d_act_slot, std::max<size_t>(1, c->act_slot.size())))) return rc;
  if (!c->act_pix.empty()) {
    HIPCHK(c, hipMemcpy(c->d_act_pix, c->act_pix.data(), c->act_pix.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_act_slot, c->act_slot.data(), c->act_slot.size() * 4, hipMemcpyHostToDevice));
  }
  c->cull_cam = c->camera;
  c->cull_valid = true;
  return PT_OK;
}

static void build_owned_pixels(pt_ctx* c, int W, int H, int T, int rank, int nranks) {
  c->pix_of.clear();
  const int ntx = (W + T - 1) / T, nty = (H + T - 1) / T;
  for (int t = 0; t < ntx * nty; ++t) {
    if (t % nranks != rank) continue;
    const int ty = t / ntx, tx = t % ntx;
    for (int r = ty * T; r < std::min(H, (ty + 1) * T); ++r)
      for (int col = tx * T; col < std::min(W, (tx + 1) * T); ++col) c->pix_of.push_back((uint32_t)(r * W + col));
  }
}

extern "C" {

#if PT_PATH_TIMING
// diagnostic build only: the per-wave marks of the last k_path_leaf launch
int pt_dbg_path_timing(unsigned long long* out, int nwaves) {
  if (!out || nwaves <= 0 || nwaves > (int)PT_TIMING_WAVES) return PT_E_INVALID;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_path_timing), (size_t)nwaves * 64) == hipSuccess ? PT_OK
                                                                                                 : PT_E_HIP;
}
#endif
#if PT_DBG_LINES
// diagnostic build only: the level items' record-line counts (read, then reset)
int pt_dbg_lines(unsigned long long* out8) {
  if (!out8) return PT_E_INVALID;
  if (hipDeviceSynchronize() != hipSuccess) return PT_E_HIP;
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_dbg_lines), 64) != hipSuccess) return PT_E_HIP;
  const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_lines), z, 64) == hipSuccess ? PT_OK : PT_E_HIP;
}
#endif

int pt_check_division(pt_ctx* c, const float* num, const float* den, float* q, int32_t n) {
  if (!c || !num || !den || !q || n < 0) return PT_E_INVALID;
  if (n == 0) return PT_OK;
  float* d = nullptr;
  HIPCHK(c, hipMalloc((void**)&d, (size_t)n * 12));
  int rc = PT_OK;
  if (hipMemcpy(d, num, (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d + n, den, (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess)
    rc = fail(c, PT_E_HIP, "pt_check_division: copy in");
  if (rc == PT_OK) {
    hipLaunchKernelGGL(k_check_division, dim3((n + TPB - 1) / TPB), dim3(TPB), 0, c->stream, (const float*)d,
                       (const float*)(d + n), d + 2 * (size_t)n, (uint32_t)n);
    if (hipStreamSynchronize(c->stream) != hipSuccess ||
        hipMemcpy(q, d + 2 * (size_t)n, (size_t)n * 4, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(c, PT_E_HIP, "pt_check_division: kernel");
  }
  hipFree(d);
  return rc;
}

int pt_check_fast_math(pt_ctx* c, int32_t which, uint32_t lo, uint32_t hi, uint64_t* mismatches,
                       uint32_t* first_bad) {
  if (!c || (which != 0 && which != 1) || hi < lo || !mismatches || !first_bad) return PT_E_INVALID;
  unsigned int* d = nullptr;
  HIPCHK(c, hipMalloc((void**)&d, 8));
  const unsigned int init[2] = {0u, 0xFFFFFFFFu};
  unsigned int h[2] = {0u, 0xFFFFFFFFu};
  int rc = PT_OK;
  if (hipMemcpy(d, init, 8, hipMemcpyHostToDevice) != hipSuccess) rc = fail(c, PT_E_HIP, "pt_check_fast_math: init");
  if (rc == PT_OK && hi > lo) {
    hipLaunchKernelGGL(k_check_fast_math, dim3(16384), dim3(TPB), 0, c->stream, (int)which, lo, hi, d);
    if (hipStreamSynchronize(c->stream) != hipSuccess || hipMemcpy(h, d, 8, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(c, PT_E_HIP, "pt_check_fast_math: kernel");
  }
  hipFree(d);
  *mismatches = h[0];
  *first_bad = h[1];
  return rc;
}

int pt_api_version(void) { return PT_API_VERSION; }

int pt_device_count(int* n) {
  if (!n) return PT_E_INVALID;
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    *n = 0;
    return PT_E_NODEVICE;
  }
  return PT_OK;
}

int pt_create(pt_ctx** out, int device) {
  if (!out) return PT_E_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return PT_E_NODEVICE;
  if (device < 0 || device >= n) return PT_E_INVALID;
  pt_ctx* c = new pt_ctx();
  c->device = device;
  // initial queue factor (doubles whenever a level overflows; PT_QFACTOR=1
  // exercises that path in the tests)
  if (const char* q = getenv("PT_QFACTOR")) c->qfactor = std::max(1, atoi(q));
  if (const char* q = getenv("PT_PATH_REGIONS")) c->path_regions = std::max(1, atoi(q));
  if (const char* q = getenv("PT_PATH_CHUNK")) c->path_chunk = (uint32_t)std::min(4096, std::max(64, atoi(q)));
  // paths per chunk (a frame of npix x spp paths runs in ceil(spp / (chunk / npix))
  // chunks, summed per pixel in sample order across them): tests set it small
  if (const char* q = getenv("PT_CULL")) c->cull = atoi(q) != 0;
  // (A/B: PT_ACC_BLOCKS=0 sums each pipelined launch by a k_accum of its own)
  if (const char* q = getenv("PT_ACC_BLOCKS")) c->acc_blocks = atoi(q) <= 0 ? 0 : std::max(8, std::min(4096, atoi(q) / 8 * 8));
  c->dbg_sync = getenv("PT_DEBUG_SYNC") != nullptr;
  if (const char* q = getenv("PT_CHUNK_PATHS")) c->chunk_paths = (uint32_t)std::min<long long>(1ll << 28, std::max(1ll, atoll(q)));
  // tail compaction needs the wave record order's continuing-first ranks
  if (const char* q = getenv("PT_COMPACT")) {
    c->compaction = atoi(q) != 0;
    if (atoi(q) > 1) c->compact_pct = std::min(100, atoi(q));
  }
  if (const char* q = getenv("PT_COMPACT_FIRST")) {
    c->compact_first = std::min(100, std::max(1, atoi(q)));
  }
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return PT_E_HIP;
  }
  for (auto& e : c->ev) hipEventCreate(&e);
  for (auto& e : c->ev_poll) hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (int k = 0; k < 2; ++k) {
    hipEventCreateWithFlags(&c->ev_fr[k], hipEventDisableTiming);
    hipEventCreateWithFlags(&c->ev_cp[k], hipEventDisableTiming);
  }
  if (hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) c->copy_stream = nullptr;
  if (hipMalloc((void**)&c->d_stats, STAT_COUNT * 8) != hipSuccess ||
      hipMalloc((void**)&c->d_rcount, RCOUNT_SLOTS * 16 * 8) != hipSuccess ||
      hipMalloc((void**)&c->d_rcount_bak, RCOUNT_SLOTS * 16 * 8) != hipSuccess ||
      hipMalloc((void**)&c->d_stats_bak, STAT_COUNT * 8) != hipSuccess ||
      hipMalloc((void**)&c->d_err, 4) != hipSuccess || hipMalloc((void**)&c->d_work, PATH_REGIONS_MAX * PATH_CTR_STRIDE * 4) != hipSuccess ||
      hipMalloc((void**)&c->d_live, LIVE_WORDS * 4) != hipSuccess ||
      hipMalloc((void**)&c->d_compact, MAX_COMPACTIONS * CBLK * 4) != hipSuccess ||
      hipMalloc((void**)&c->d_pool, POOLS * CSTRIDE * 4) != hipSuccess ||
      hipHostMalloc((void**)&c->h_poll, 32, hipHostMallocDefault) != hipSuccess) {
    delete c;
    return PT_E_HIP;
  }
  hipMemset(c->d_stats, 0, STAT_COUNT * 8);
  hipMemset(c->d_rcount, 0, RCOUNT_SLOTS * 16 * 8);
  hipMemset(c->d_err, 0, 4);
  // k_path_leaf runs persistent waves: one grid of exactly the resident workgroups
  {
    int ncu = 0, nb[4] = {0, 0, 0, 0};
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb[0], k_path_leaf<1, false, true>, TPB, 0);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb[1], k_path_leaf<2, false, true>, TPB, 0);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb[2], k_path_leaf<1, true, false>, TPB, 0);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb[3], k_path_leaf<2, true, false>, TPB, 0);
    for (int i = 0; i < 4; ++i) c->path_grid[i] = std::max(1, ncu * std::max(1, nb[i]));
  }
  *out = c;
  return PT_OK;
}

void pt_destroy(pt_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->copy_stream) hipStreamSynchronize(c->copy_stream);
  free_all(c);
  for (int k = 0; k < 2; ++k) {
    if (c->ev_fr[k]) hipEventDestroy(c->ev_fr[k]);
    if (c->ev_cp[k]) hipEventDestroy(c->ev_cp[k]);
  }
  if (c->copy_stream) hipStreamDestroy(c->copy_stream);
  for (auto& e : c->evpool) hipEventDestroy(e);
  for (auto& e : c->ev)
    if (e) hipEventDestroy(e);
  for (auto& e : c->ev_poll)
    if (e) hipEventDestroy(e);
  if (c->h_poll) hipHostFree(c->h_poll);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

const char* pt_last_error(const pt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pt_load_scene(pt_ctx* c, const pt_scene_desc* s) {
  if (!c || !s || s->n_prims <= 0 || s->n_nodes <= 0 || s->n_levels <= 0) return fail(c, PT_E_INVALID, "empty scene");
  hipSetDevice(c->device);
  int rc;
  if ((rc = drain(c))) return rc;
  c->n_prims = s->n_prims;
  c->n_nodes = s->n_nodes;
  c->n_levels = s->n_levels;
  c->level_start.assign(s->level_start, s->level_start + s->n_levels + 1);
  c->max_level_nodes = 0;
  for (int l = 0; l < s->n_levels; ++l)
    c->max_level_nodes = std::max(c->max_level_nodes, c->level_start[l + 1] - c->level_start[l]);
  c->nodes_host.assign(s->nodes, s->nodes + s->n_nodes);
  c->root_leaf = c->nodes_host[0].prim_count > 0;
  c->level_has_leaf.assign(s->n_levels, 0);
  for (int l = 0; l < s->n_levels; ++l)
    for (int i = std::max(0, s->level_start[l]); i < std::min(s->n_nodes, s->level_start[l + 1]); ++i)
      if (s->nodes[i].prim_count > 0) c->level_has_leaf[l] = 1;
  for (int i = 0; i < s->n_nodes; ++i) {
    const pt_node& nd = s->nodes[i];
    if (nd.prim_start < 0 || nd.prim_count < 0 || nd.prim_start + nd.prim_count > s->n_prims)
      return fail(c, PT_E_INVALID, "node primitive range out of bounds");
    for (int k = 0; k < 4; ++k)
      if (nd.child[k] >= s->n_nodes || (nd.child[k] >= 0 && nd.child[k] <= i))
        return fail(c, PT_E_INVALID, "node child out of range / not breadth-first");
  }
  c->has_sphere = c->has_glass = false;
  for (int i = 0; i < s->n_prims; ++i) {
    uint32_t meta;
    memcpy(&meta, &s->prims[i].q[3], 4);
    if ((int)(meta & 0x0FFFFFFFu) >= s->n_bsdfs) return fail(c, PT_E_INVALID, "primitive bsdf out of range");
    // (bit 27 of a device shading record's meta word is its SHADE_SMOOTH flag)
    if ((meta & 0x0FFFFFFFu) >= SHADE_SMOOTH) return fail(c, PT_E_UNSUPPORTED, "more than 2^27 bsdfs");
    if ((meta >> 28) == PT_PRIM_SPHERE) c->has_sphere = true;
  }
  for (int i = 0; i < s->n_bsdfs; ++i)
    if (s->bsdfs[i].type == PT_BSDF_GLASS || s->bsdfs[i].type == PT_BSDF_REFRACTION) c->has_glass = true;
  build_root_table(c);
  if ((rc = dalloc(c, &c->d_nodes, s->n_nodes))) return rc;
  if ((rc = dalloc(c, &c->d_prims, (size_t)s->n_prims * prim_stride<false>()))) return rc;
  if ((rc = dalloc(c, &c->d_prims_ref, (size_t)s->n_prims * 6))) return rc;
  if ((rc = dalloc(c, &c->d_shade, (size_t)s->n_prims * SHADE_REC))) return rc;
  if ((rc = dalloc(c, &c->d_bsdfs, std::max(1, s->n_bsdfs)))) return rc;
  if (s->n_lights > 1 && !s->lights) return fail(c, PT_E_INVALID, "n_lights > 1 without lights");
  if (s->n_lights > 256) return fail(c, PT_E_UNSUPPORTED, "more than 256 lights");
  if ((rc = dalloc(c, &c->d_lights, std::max(1, (int)s->n_lights)))) return rc;
  if ((rc = dalloc(c, &c->d_cnt, (size_t)s->n_nodes * NLANE * CSTRIDE))) return rc;
  if ((rc = dalloc(c, &c->d_qoff, (size_t)s->n_nodes * NLANE))) return rc;
  if ((rc = dalloc(c, &c->d_iprefix, (size_t)NLANE * (c->max_level_nodes + 1)))) return rc;
  if ((rc = dalloc(c, &c->d_icnt, (size_t)NLANE * (c->max_level_nodes + 1)))) return rc;
  if ((rc = dalloc(c, &c->d_scan_aux, (size_t)SCAN_MAXG * AGG_STRIDE + c->max_level_nodes + 1))) return rc;
  if ((rc = dalloc(c, &c->d_nitems, 2 * std::max(1, s->n_levels) + NLANE))) return rc;
  {
    // the device's tree: the inlined deep leaves detached from their parents
    std::vector<pt_node> dn(s->nodes, s->nodes + s->n_nodes);
    for (const auto& pk : c->detached)
      if (pk.first >= 0 && pk.first < s->n_nodes && pk.second >= 0 && pk.second < 4) dn[pk.first].child[pk.second] = -1;
    HIPCHK(c, hipMemcpy(c->d_nodes, dn.data(), sizeof(pt_node) * s->n_nodes, hipMemcpyHostToDevice));
    // levels with a reachable leaf (a detached leaf's level may have none left)
    c->level_has_leaf.assign(s->n_levels, 0);
    if (c->root_leaf) c->level_has_leaf[0] = 1;
    for (int l = 0; l + 1 < s->n_levels; ++l)
      for (int i = std::max(0, s->level_start[l]); i < std::min(s->n_nodes, s->level_start[l + 1]); ++i)
        for (int k = 0; k < 4; ++k) {
          const int ch = dn[i].child[k];
          if (ch >= 0 && dn[ch].prim_count > 0) c->level_has_leaf[l + 1] = 1;  // (children sit one level down)
        }
  }
  {
    const std::vector<float4> rec = bw_prim_records(s);
    HIPCHK(c, hipMemcpy(c->d_prims, rec.data(), rec.size() * sizeof(float4), hipMemcpyHostToDevice));
  }
  {
    const std::vector<pt_prim> ref = ref_prim_records(s);
    HIPCHK(c, hipMemcpy(c->d_prims_ref, ref.data(), sizeof(pt_prim) * s->n_prims, hipMemcpyHostToDevice));
  }
  {
    // shade.hip ShadeArgs::shade: triangle {n0, meta'}{A, n1.x}{B, n1.y}{C, n1.z}{n2, 0},
    // sphere {centre, meta'}; meta' = meta | SHADE_SMOOTH unless the triangle is
    // flat (identical vertex normals: its shading normal is normalize(n0), so
    // a hit on it reads the first 16 B only)
    std::vector<float4> rec((size_t)s->n_prims * SHADE_REC);
    for (int i = 0; i < s->n_prims; ++i) {
      const float* q = s->prims[i].q;
      const float *n0 = s->shading[i].n0, *n1 = s->shading[i].n1, *n2 = s->shading[i].n2;
      float4* r = &rec[(size_t)i * SHADE_REC];
      uint32_t meta;
      memcpy(&meta, &q[3], 4);
      if ((meta >> 28) == PT_PRIM_SPHERE) {
        r[0] = make_float4(q[0], q[1], q[2], q[3]);
        r[1] = r[2] = r[3] = r[4] = make_float4(0.f, 0.f, 0.f, 0.f);
        continue;
      }
      // flat: the three normals identical to the bit (not float ==, under
      // which a +0 and a -0 component match: the reference arithmetic's
      // blend then takes n2 for n0, below, and the signs of zero components
      // of its normal could differ from cu:1213-1221's; the oracle decides the
      // same way)
      const bool flat = memcmp(n0, n1, 3 * sizeof(float)) == 0 && memcmp(n1, n2, 3 * sizeof(float)) == 0;
      const uint32_t m2 = meta | (flat ? 0u : SHADE_SMOOTH);
      float mf;
      memcpy(&mf, &m2, 4);
      if (flat) {
        // a flat triangle's shading normal normalize(n0) (ptmath.h normalize:
        // n0 * (1 / sqrt(fma-chain dot)), correctly rounded fp32 here as on
        // the device), so the kernels read it instead of computing it; the
        // raw n0 stays in r[4] (= n2) for the reference arithmetic's blend
        const float dd = std::fmaf(n0[2], n0[2], std::fmaf(n0[1], n0[1], n0[0] * n0[0]));
        const float inv = 1.0f / std::sqrt(dd);
        r[0] = make_float4(n0[0] * inv, n0[1] * inv, n0[2] * inv, mf);
      } else {
        r[0] = make_float4(n0[0], n0[1], n0[2], mf);
      }
      r[1] = make_float4(q[0], q[1], q[2], n1[0]);
      r[2] = make_float4(q[4], q[5], q[6], n1[1]);
      r[3] = make_float4(q[8], q[9], q[10], n1[2]);
      r[4] = make_float4(n2[0], n2[1], n2[2], 0.0f);
    }
    HIPCHK(c, hipMemcpy(c->d_shade, rec.data(), rec.size() * sizeof(float4), hipMemcpyHostToDevice));
  }
  if (s->n_bsdfs > 0) {
    // pt_bsdf + the dielectric's 1 / ior and r0 in IEEE fp32 (BsdfRec; this
    // translation unit is built with -ffp-contract=off)
    std::vector<BsdfRec> br((size_t)s->n_bsdfs);
    for (int i = 0; i < s->n_bsdfs; ++i) {
      const pt_bsdf& b = s->bsdfs[i];
      BsdfRec& r = br[(size_t)i];
      r.type = b.type;
      for (int k = 0; k < 3; ++k) {
        r.albedo[k] = b.albedo[k];
        r.transmittance[k] = b.transmittance[k];
      }
      r.ior = b.ior;
      r.roughness = b.roughness;
      r.inv_ior = 1.0f / b.ior;
      const float q = (1.0f - b.ior) / (1.0f + b.ior);
      r.r0 = q * q;
      r.pad = 0.0f;
    }
    HIPCHK(c, hipMemcpy(c->d_bsdfs, br.data(), sizeof(BsdfRec) * br.size(), hipMemcpyHostToDevice));
  }
  HIPCHK(c, hipMemset(c->d_cnt, 0, (size_t)s->n_nodes * NLANE * CSTRIDE * 4));
  HIPCHK(c, hipMemset(c->d_qoff, 0, (size_t)s->n_nodes * NLANE * 4));
  c->light = s->light;
  c->camera = s->camera;
  c->cull_valid = false;  // (the culled pixels depend on the scene's box, not only on the camera)
  c->n_lights = s->n_lights > 1 ? (uint32_t)s->n_lights : 0u;
  if (c->n_lights)
    HIPCHK(c, hipMemcpy(c->d_lights, s->lights, sizeof(pt_light) * c->n_lights, hipMemcpyHostToDevice));
  {  // origin_bound: 64 x the largest magnitude of the scene's vertices, sphere extents, camera, light
    double m = 0.0;
    auto upd = [&](double v) { m = std::max(m, std::fabs(v)); };
    for (int i = 0; i < s->n_prims; ++i) {
      const float* q = s->prims[i].q;
      uint32_t meta;
      memcpy(&meta, &q[3], 4);
      if ((meta >> 28) == PT_PRIM_SPHERE) {
        for (int k = 0; k < 3; ++k) upd(std::fabs(q[k]) + q[4]);
      } else {
        for (int k = 0; k < 3; ++k) {
          upd(q[k]);
          upd(q[4 + k]);
          upd(q[8 + k]);
        }
      }
    }
    for (int k = 0; k < 3; ++k) {
      upd(s->camera.origin[k]);
      upd(s->light.position[k]);
      for (int l = 0; l < (int)c->n_lights; ++l) upd(s->lights[l].position[k]);
    }
    c->origin_bound = 64.0 * m;
    // single-leaf scenes: the root leaf's primitives in clusters of one, or
    // two consecutive triangles whose union box is barely larger than either
    // (a Cornell wall's two halves), each cluster's box widened by the BVH
    // boxes' guard band G = 2^-14 M (scene_internal.h box_guard) and rounded
    // outward: k_path_leaf's closest-hit loop (PT_PATH_CLUSTER) tests a lane's
    // ray only against the clusters whose box it enters.  Conservative as the
    // BVH's own leaf boxes are: a triangle-test hit lies within ~2^-18 M of its
    // triangle for origins up to 64 M.  Record: {xmin, xmax, ymin, ymax, zmin,
    // zmax} (box_hit's order), first primitive (leaf-relative), count.
    c->nclus = 0;
    c->sph_clmask = 0;
    if (c->root_leaf) {
      const pt_node& r = c->nodes_host[0];
      const double G = std::ldexp(m, -14);
      std::vector<float> cb;
      for (int i = 0; i < r.prim_count;) {
        double lo[3], hi[3], lo2[3], hi2[3];
        bool s1 = false, s2 = true;
        prim_box(s->prims[r.prim_start + i], lo, hi, s1);
        int cnt = 1;
        if (i + 1 < r.prim_count) {
          prim_box(s->prims[r.prim_start + i + 1], lo2, hi2, s2);
          double ul[3], uh[3];
          for (int k = 0; k < 3; ++k) {
            ul[k] = std::min(lo[k], lo2[k]);
            uh[k] = std::max(hi[k], hi2[k]);
          }
          if (!s1 && !s2 && half_area(ul, uh) <= 1.05 * std::max(half_area(lo, hi), half_area(lo2, hi2))) {
            cnt = 2;
            for (int k = 0; k < 3; ++k) {
              lo[k] = ul[k];
              hi[k] = uh[k];
            }
          }
        }
        if (s1 && cb.size() / 8 < 32) c->sph_clmask |= 1u << (cb.size() / 8);
        push_guarded_box(cb, lo, hi, G);
        cb.push_back(int_bits(i));
        cb.push_back(int_bits(cnt));
        i += cnt;
      }
      // record nclus: the union of the cluster boxes (PT_PATH_EXT_AABB)
      const int nc = (int)(cb.size() / 8);
      float ub[6] = {INFINITY, -INFINITY, INFINITY, -INFINITY, INFINITY, -INFINITY};
      for (int k = 0; k < nc; ++k)
        for (int a = 0; a < 3; ++a) {
          ub[2 * a] = std::min(ub[2 * a], cb[8 * k + 2 * a]);
          ub[2 * a + 1] = std::max(ub[2 * a + 1], cb[8 * k + 2 * a + 1]);
        }
      cb.insert(cb.end(), ub, ub + 6);
      cb.push_back(0.0f);
      cb.push_back(0.0f);
      int rc2;
      if ((rc2 = dalloc(c, &c->d_cbox, std::max<size_t>(8, cb.size())))) return rc2;
      HIPCHK(c, hipMemcpy(c->d_cbox, cb.data(), cb.size() * sizeof(float), hipMemcpyHostToDevice));
      c->nclus = nc;
    }
    int rc3;
    if ((rc3 = root_clusters(c, s, std::ldexp(m, -14)))) return rc3;
  }
  c->have_scene = true;
  c->cull_valid = false;
  c->cap_paths = 0;  // force re-derivation of root queue offsets
  c->cap_spp = 0;
  return PT_OK;
}

int pt_set_camera(pt_ctx* c, const pt_camera* cam) {
  if (!c || !cam) return PT_E_INVALID;
  for (int k = 0; k < 3; ++k)
    if (!(std::fabs((double)cam->origin[k]) <= c->origin_bound))
      return fail(c, PT_E_UNSUPPORTED, "pt_set_camera: origin beyond 64x the scene's extent (conservative box guard)");
  c->camera = *cam;
  c->cull_valid = false;
  return pt_clear(c);
}

int pt_clear(pt_ctx* c) {
  if (!c) return PT_E_INVALID;
  hipSetDevice(c->device);
  // (queued, not waited for: ordered after the frames before it on `stream`,
  // where their sums are made, so a pipelined next frame is not held up)
  if (c->d_accum && !c->pix_of.empty()) {
    const uint32_t n = (uint32_t)c->pix_of.size();
    // sums or an image still pending on the current buffer: the next frame
    // accumulates into the other one
    bool pending = c->acc_on && c->acc_job.dst == c->d_accum;
    for (int i = 0; i < c->n_img; ++i) pending = pending || c->img_job[i].acc == c->d_accum;
    if (pending) {
      if (!c->d_accum_b) {
        int rc;
        if ((rc = dalloc(c, &c->d_accum_b, n))) return rc;
      }
      std::swap(c->d_accum, c->d_accum_b);
    }
    hipLaunchKernelGGL(k_zero, dim3((n + TPB - 1) / TPB), dim3(TPB), 0, c->stream, c->d_accum, n);
    HIPCHK(c, hipGetLastError());
  }
  c->samples = 0;
  return PT_OK;
}

int pt_reset_stats(pt_ctx* c) {
  if (!c) return PT_E_INVALID;
  hipSetDevice(c->device);
  if (int rc = drain(c)) return rc;
  HIPCHK(c, hipMemset(c->d_stats, 0, STAT_COUNT * 8));
  HIPCHK(c, hipMemset(c->d_rcount, 0, RCOUNT_SLOTS * 16 * 8));
  memset(&c->stats, 0, sizeof(c->stats));
  c->host_rays = 0;
  return PT_OK;
}

int pt_get_stats(pt_ctx* c, pt_stats* out) {
  if (!c || !out) return PT_E_INVALID;
  hipSetDevice(c->device);
  int rc = drain(c);
  if (rc) return rc;
  rc = read_device_stats(c);
  c->stats.n_levels = c->n_levels;
  c->stats.queue_factor = (int32_t)c->qfactor;
  *out = c->stats;
  return rc == PT_E_OVERFLOW ? PT_OK : rc;
}

int pt_render(pt_ctx* c, const pt_render_params* P) {
  if (!c || !P) return PT_E_INVALID;
  c->ray_cur = nullptr;
  if (!c->have_scene) return fail(c, PT_E_NOSCENE, "no scene loaded");
  if (P->width <= 0 || P->height <= 0 || P->spp <= 0 || P->max_bounces < 0 || P->max_bounces > 250)
    return fail(c, PT_E_INVALID, "bad render parameters");
  const int nranks = P->nranks > 0 ? P->nranks : 1;
  const int rank = P->rank;
  if (rank < 0 || rank >= nranks) return fail(c, PT_E_INVALID, "bad rank");
  const int tile = P->tile_size > 0 ? P->tile_size : 32;
  if ((unsigned long long)P->width * P->height >= (1ull << 30))
    return fail(c, PT_E_UNSUPPORTED, "image larger than 2^30 pixels");
  hipSetDevice(c->device);
  int rc;
  const bool fb_change = P->width != c->fb_w || P->height != c->fb_h || tile != c->fb_tile || rank != c->fb_rank ||
                         nranks != c->fb_nranks;
  const bool cull_stale = !c->cull_valid || memcmp(&c->cull_cam, &c->camera, sizeof(pt_camera)) != 0;
  // PT_FLAG_ASYNC: single-leaf scenes, uninstrumented frames, and nothing the
  // queued frames read is re-uploaded (owned / culled pixel lists)
  const bool async = (P->flags & PT_FLAG_ASYNC) && c->root_leaf && !(P->flags & PT_FLAG_STATS) && !fb_change &&
                     !cull_stale;
  if (!async && (rc = drain(c))) return rc;
  // framebuffer / owned pixels
  if (fb_change) {
    build_owned_pixels(c, P->width, P->height, tile, rank, nranks);
    c->cull_valid = false;
    c->fb_w = P->width;
    c->fb_h = P->height;
    c->fb_tile = tile;
    c->fb_rank = rank;
    c->fb_nranks = nranks;
    if ((rc = dalloc(c, &c->d_pix_of, c->pix_of.size()))) return rc;
    if ((rc = dalloc(c, &c->d_accum, c->pix_of.size()))) return rc;
    if (c->d_accum_b) {  // (re-made at its first use, pt_clear)
      hipFree(c->d_accum_b);
      c->d_accum_b = nullptr;
    }
    if (!c->pix_of.empty())
      HIPCHK(c, hipMemcpy(c->d_pix_of, c->pix_of.data(), c->pix_of.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemset(c->d_accum, 0, std::max<size_t>(1, c->pix_of.size()) * sizeof(float4)));
    c->samples = 0;
  }
  if (c->pix_of.empty()) {
    c->samples += P->spp;
    return PT_OK;
  }
  // the owned pixels whose camera rays may reach the scene (cull_pixels); the
  // rest end at their camera vertex with radiance 0: counted, not traced
  if ((rc = cull_pixels(c, P->width, P->height))) return rc;
  c->host_rays += (uint64_t)(c->pix_of.size() - c->act_pix.size()) * (uint64_t)P->spp;
  const uint32_t npix = (uint32_t)c->act_pix.size();
  if (npix == 0) {
    c->samples += P->spp;
    return PT_OK;
  }
  // the reference schedule (cu:2499-2533) casts up to two shadow rays per vertex
  const bool ref_sched = (P->flags & PT_FLAG_REF_SCHEDULE) != 0;
  const uint32_t nsh = ref_sched ? 2u : 1u;
  c->refa = (P->flags & PT_FLAG_REF_ARITH) != 0;
  c->tmin = false;
  bool compact_mem = true;  // the tail compaction's second set could be allocated (ensure_compact_set)
  // (glass is read as the reference reads it, a mirror: shade.hip; spheres
  // the reference cannot render at all: cu:1765 casts every primitive to Triangle)
  if (c->refa && c->has_sphere)
    return fail(c, PT_E_UNSUPPORTED, "PT_FLAG_REF_ARITH: the reference renders triangles only");
  // (the reference's CUDA path takes exactly one light, read as an AreaLight, cu:1733-1751)
  // the extended light model (several lights, directional / hemisphere
  // lights): its own kernel variants, default arithmetic and one NEE sample
  // per vertex only
  const bool xl = c->n_lights > 0 || c->light.type == PT_LIGHT_DIRECTIONAL || c->light.type == PT_LIGHT_HEMISPHERE;
  if (xl && c->refa)
    return fail(c, PT_E_UNSUPPORTED, "PT_FLAG_REF_ARITH: the reference's CUDA path takes one area light (cu:1733-1751)");
  if (xl && (P->flags & PT_FLAG_REF_SCHEDULE))
    return fail(c, PT_E_UNSUPPORTED, "PT_FLAG_REF_SCHEDULE: the reference schedule samples one area light");
  const int max_bounces = ref_sched ? 2 : P->max_bounces;
  const int passes = max_bounces + 2;  // vertices per path at most
  // (d_err collects the queued frames' failures: reset when none is pending)
  if (!c->async_pending) HIPCHK(c, zero_async(c, c->d_err, 4));
  c->timing = (P->flags & PT_FLAG_STATS) != 0;
  const bool timed = c->timing;

  hipEvent_t t0 = c->ev[6], t1 = c->ev[7];
  HIPCHK(c, hipEventRecord(t0, c->stream));
  bool first = true;
  // chunks of spp_c samples of every owned pixel: M = npix * spp_c paths, each
  // path's radiance lands in res[j * npix + q] and is summed in sample order
  for (int done = 0; done < P->spp;) {
    const uint32_t spp_c = std::min<uint32_t>(std::max<uint32_t>(1, c->chunk_paths / npix), (uint32_t)(P->spp - done));
    const uint32_t M = npix * spp_c;
    // per-path results: slot res_k of two when frames are pipelined (the
    // previous launch's slot is summed while this one is written), else slot 0
    const int rk = async ? c->res_k : 0;
    float4*& res_slot = rk ? c->d_res_b : c->d_res;
    size_t& res_cap = rk ? c->res_cap_b : c->res_cap;
    if ((size_t)M > res_cap) {
      HIPCHK(c, hipStreamSynchronize(c->stream));  // (queued launches may still read it)
      if ((rc = dalloc(c, &res_slot, M))) return rc;
      res_cap = M;
    }
    float4* const res = res_slot;
    ShadeArgs S;
    S.A.dbg_nprims = (uint32_t)c->n_prims;  // (PT_DBG_BOUNDS; the wavefront branch sets all of S.A)
    S.prims = c->refa ? c->d_prims_ref : c->d_prims;
    S.shade = c->d_shade;
    S.bsdfs = c->d_bsdfs;
    S.pix_of = c->d_act_pix;
    S.light = c->light;
    S.cam = c->camera;
    S.lights = c->d_lights;
    S.n_lights = c->n_lights;
    S.cbox = c->d_cbox;
    S.nclus = c->nclus;
    S.sph_cl = c->sph_clmask;
    S.npix = npix;
    S.div_npix = udiv_make(npix);
    S.div_width = udiv_make((uint32_t)P->width);
    S.seed = P->seed;
    S.width = P->width;
    S.height = P->height;
    S.max_bounces = max_bounces;
    S.flags = P->flags;
    S.rcount = c->d_rcount;
    S.sample_base = (uint32_t)(P->sample_offset + done);
    S.res = res;
    S.M = M;
    S.acc_blocks = 0;  // (k_path_leaf's leading sum workgroups: none unless set below)
    S.acc_res = nullptr;
    S.acc_dst = nullptr;
    S.acc_slot = nullptr;
    S.acc_npix = S.acc_spp = 0;
    S.passes = passes;
    {  // record-order keys: SORT_KEYS equal primitive ranges (BVH order, so ~subtrees)
      uint32_t b = 0;
      while ((1u << b) < (uint32_t)c->n_prims) ++b;
      S.kshift = b > SORT_KEY_BITS ? b - SORT_KEY_BITS : 0u;
    }
    if (c->root_leaf) {
      // single-leaf tree: every path runs to completion in one kernel
      // (persistent waves with path regeneration, output res[P])
      const pt_node& root = c->nodes_host[0];
      S.ray = nullptr;
      S.ps0 = S.ps2 = S.ps3 = nullptr;
      S.ps1 = res;
      S.N = M;
      const uint32_t want = (M + 4 * PATH_CHUNK - 1) / (4 * PATH_CHUNK);
      const int kv = (nsh == 2 ? 1 : 0) + (c->refa ? 2 : 0);
      const uint32_t blocks = std::min<uint32_t>(want, c->path_grid[kv]);
      // (spheres: the sphere test compiled in; the reference arithmetic has none)
      const bool sph = c->has_sphere;
      auto kpath = xl ? (sph ? k_path_leaf<1, false, true, true> : k_path_leaf<1, false, false, true>)
                      : (kv == 0 ? (sph ? k_path_leaf<1, false, true> : k_path_leaf<1, false, false>)
                         : kv == 1 ? (sph ? k_path_leaf<2, false, true> : k_path_leaf<2, false, false>)
                         : kv == 2 ? k_path_leaf<1, true, false> : k_path_leaf<2, true, false>);
      // PT_FLAG_COUNT_TESTS: the counting variant (default schedule and
      // arithmetic, one light; the others count nothing)
      if ((P->flags & PT_FLAG_COUNT_TESTS) && kv == 0 && !xl)
        kpath = sph ? k_path_leaf<1, false, true, false, true> : k_path_leaf<1, false, false, false, true>;
      // path grabs (shade.hip k_path_leaf): nreg regions, chunks of 512 paths
      // for a whole frame, fewer when the launch has few paths per resident
      // lane (its tail is about one chunk's time)
      const uint32_t nreg = (uint32_t)std::max(1, std::min<int>(c->path_regions, (int)std::min<uint32_t>(blocks, PATH_REGIONS_MAX)));
      S.grab_chunk = c->path_chunk ? c->path_chunk : path_chunk_for(M, blocks);
      S.grab_nreg = nreg;
      S.grab_region = (M + nreg - 1) / nreg;
      S.grab_work = c->d_work;
      HIPCHK(c, zero_async(c, c->d_work, (size_t)nreg * PATH_CTR_STRIDE * 4));
      // pipelined: the previous launch's sums in this launch's leading workgroups
      if (async && c->acc_on && c->acc_blocks == 0)
        if ((rc = flush_sums(c))) return rc;
      if (async && c->acc_on) {
        S.acc_blocks = (uint32_t)c->acc_blocks;
        S.acc_res = c->acc_job.res;
        S.acc_dst = c->acc_job.dst;
        S.acc_slot = c->d_act_slot;
        S.acc_npix = c->acc_job.npix;
        S.acc_spp = c->acc_job.spp;
      }
      c->launch(pt_ctx::K_PATH, 0, kpath, dim3(blocks + S.acc_blocks), dim3(TPB), S, root.prim_start, root.prim_count,
                passes, c->d_rcount, c->d_err);
      HIPCHK(c, hipGetLastError());
      c->async_pending = true;
      if (async) {  // (this launch's sums: pending; the images that waited for the previous ones: queued)
        c->acc_on = true;
        c->acc_job = pt_ctx::AccJob{res, c->d_accum, npix, spp_c};
        c->res_k = rk ^ 1;
        if ((rc = serve_images(c))) return rc;
      }
      c->stats.passes += passes;
      if (first) c->stats.batch_paths = (int32_t)M;
    } else {
      // N path slots run the chunk's M paths: a slot whose path ends starts the
      // next one in the same shade kernel, so every pass traces a full pool
      // (the counters as the chunk starts, for a re-run after a queue overflow)
      HIPCHK(c, copy_async(c, c->d_rcount_bak, c->d_rcount, RCOUNT_SLOTS * 16 * 8));
      HIPCHK(c, copy_async(c, c->d_stats_bak, c->d_stats, STAT_COUNT * 8));
      const pt_stats stats0 = c->stats;
      const size_t marks0 = c->marks.size(), evn0 = c->evn;
      const uint32_t cap = max_batch_paths(c, 1 + nsh);
      uint32_t target = P->batch_paths > 0 ? (uint32_t)P->batch_paths : DEFAULT_BATCH_PATHS;
      const uint32_t N = std::min<uint32_t>(std::min<uint32_t>(target, cap), M);
      const bool realloc = N > c->cap_paths || 1 + nsh > c->cap_spp || c->qfactor != c->cap_qfactor;
      if ((rc = ensure_paths(c, N, 1 + nsh))) return rc;
      if (realloc && (rc = set_root_child_offsets(c))) return rc;
      if (first) c->stats.batch_paths = (int32_t)N;
      // (device buffers as (re)allocated by ensure_paths)
      S.N = N;
      c->shadow_base = N;  // slots >= N hold shadow rays
      // slot buffers: set a until the tail's first compaction, then the two
      // sets alternate (ShadeArgs::compact); in: what the shade kernel reads,
      // out: what it writes and the traversal then reads
      // (the second set is allocated at the first compaction: refreshed below)
      float4* RAY[2] = {c->d_ray, c->d_ray_b};
      float4* PS[4][2] = {{c->d_ps0, c->d_ps0_b}, {c->d_ps1, c->d_ps1_b}, {c->d_ps2, c->d_ps2_b},
                          {c->d_ps3, c->d_ps3_b}};
      auto bind = [&](int in, int out) {
        S.ray = RAY[in];
        S.ps0_in = PS[0][in];
        S.ps1_in = PS[1][in];
        S.ps2_in = PS[2][in];
        S.ps3_in = PS[3][in];
        S.ps0 = PS[0][out];
        S.ps1 = PS[1][out];
        S.ps2 = PS[2][out];
        S.ps3 = PS[3][out];
        c->ray_cur = RAY[out];
        S.A = trace_args(c);
      };
      int cur = 0;
      bind(0, 0);
      S.compact = nullptr;
      S.creg = nullptr;
      S.nact = nullptr;
      S.tprof = nullptr;
#if PT_SHADE_TIMING
      unsigned long long* d_tprof = nullptr;
      if (getenv("PT_SHADE_TIMING") && hipMalloc((void**)&d_tprof, 1024 * 8) == hipSuccess) {
        HIPCHK(c, hipMemset(d_tprof, 0, 1024 * 8));
        S.tprof = d_tprof;
      }
#endif
      S.T = c->rt;
      const dim3 grid((N + TPB - 1) / TPB);
      // workgroup b of the shade grid runs its slots' share of the chunk
      const uint32_t G = (N + TPB - 1) / TPB;
      uint32_t Gc = G;        // shade workgroups of the current slot layout
      uint32_t nbound = N;    // slots of the current layout that may hold paths
      int ncomp = 0;          // compactions so far in this chunk
      bool compact_next = false;  // the next group starts with a compaction pass
      if (G > c->wstate_cap) {
        if ((rc = dalloc(c, &c->d_wstate, G))) return rc;
        c->wstate_cap = G;
      }
      S.wstate = c->d_wstate;
      S.pool = c->d_pool;
      // dispensers: the first fill runs blocks 0 .. G-1 (workgroup b block b)
      const uint32_t nblocks = (M + POOL_BLOCK - 1) / POOL_BLOCK;
      {
        std::vector<uint32_t> init((size_t)POOLS * CSTRIDE, 0u);
        for (uint32_t k = 0; k < POOLS; ++k) init[(size_t)k * CSTRIDE] = G > k ? (G - k + POOLS - 1) / POOLS : 0u;
        HIPCHK(c, hipMemcpyAsync(c->d_pool, init.data(), init.size() * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));  // (init is a host temporary)
      }
      auto kcam = c->refa ? (nsh == 2 ? k_camera_push<2, true> : k_camera_push<1, true>)
                          : (nsh == 2 ? k_camera_push<2, false> : k_camera_push<1, false>);
      c->launch(pt_ctx::K_CAM, 0, kcam, grid, dim3(TPB), S);
      // passes in groups of POLL_GROUP; the host reads the finished-path count
      // of group g (pinned memory, event) while group g + 1 is already queued
      // (np passes; the tail of a chunk polls after every pass: a pass queued
      // after the last path ended still costs ~150 us of empty level and scan
      // launches)
      // dense passes (ShadeArgs::dense) while more than 2 N paths of work are
      // left at the last poll (PT_DENSE=0: never)
      const char* de = getenv("PT_DENSE");
      const bool dense_ok = !(de && atoi(de) == 0);
      S.dense = dense_ok ? 1u : 0u;
      auto enqueue_group = [&](int g, int np, uint32_t nlive) -> int {
        for (int k = 0; k < np; ++k) {
          int r = trace_levels(c);  // (the rays in c->ray_cur)
          if (r) return r;
          const bool comp = k == 0 && compact_next;
          uint32_t Gnew = Gc;
          if (comp) {
            // this pass writes the continuing paths densely into the other
            // set; the live slots are at most the last poll's count
            HIPCHK(c, zero_async(c, c->d_compact + ncomp * CBLK, CREGIONS * 4));
            S.compact = c->d_compact + ncomp * CBLK;
            S.creg = c->d_live + 2;  // (the regions' bounds from the k_live_sum just before)
            bind(cur, 1 - cur);
            Gnew = std::max(1u, (nlive + TPB - 1) / TPB);
          }
          if (c->timing) {
            const auto e = c->pair(pt_ctx::K_SHADE, 0);
            HIPCHK(c, pt_launch_shade_push(nsh, c->refa, xl, Gc, c->stream, e.first, e.second, &S));
          } else {
            HIPCHK(c, pt_launch_shade_push(nsh, c->refa, xl, Gc, c->stream, nullptr, nullptr, &S));
          }
          if (c->dbg_sync) c->sync_check(pt_ctx::K_SHADE, comp ? 1 : 0, Gc);
          if (comp) {
            hipLaunchKernelGGL(k_compact_wstate, dim3((Gc + TPB - 1) / TPB), dim3(TPB), 0, c->stream, S.wstate, Gc,
                               Gnew, timed ? c->d_stats + STAT_SHADED : (unsigned long long*)nullptr);
            hipLaunchKernelGGL(k_compact_slots, dim3(Gnew), dim3(TPB), 0, c->stream, S.ps0, S.wstate,
                               (const uint32_t*)S.compact, S.creg, c->d_compact + ncomp * CBLK + CREGIONS);
            if (c->dbg_sync) c->sync_check(100, 0, Gnew);
            HIPCHK(c, hipGetLastError());
            S.nact = c->d_compact + ncomp * CBLK + CREGIONS;
            S.compact = nullptr;
            cur = 1 - cur;
            bind(cur, cur);
            Gc = Gnew;
            nbound = nlive;
            ++ncomp;
            compact_next = false;
          }
        }
        HIPCHK(c, zero_async(c, c->d_live, LIVE_WORDS * 4));
        hipLaunchKernelGGL(k_live_sum, dim3(LIVE_SUM_BLOCKS), dim3(1024), 0, c->stream, (const uint4*)S.wstate, Gc,
                           (const uint32_t*)c->d_pool, nblocks, c->d_live, (unsigned long long*)nullptr);
        if (c->dbg_sync) c->sync_check(101, 0, Gc);
        HIPCHK(c, hipMemcpyAsync(c->h_poll + 4 * (g & 1), c->d_live, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->h_poll + 4 * (g & 1) + 2, c->d_err, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipEventRecord(c->ev_poll[g & 1], c->stream));
        return PT_OK;
      };
      // every path ends within `passes` passes of its start, and while blocks
      // remain every free slot starts a path: at most (M / N + 2) rounds of
      // `passes` passes
      const uint64_t max_passes = (uint64_t)(M / N + 2) * passes + 2 * POLL_GROUP;
      uint64_t queued = 2 * POLL_GROUP;
      bool overflow = false, finished = false;
      if ((rc = enqueue_group(0, POLL_GROUP, N)) || (rc = enqueue_group(1, POLL_GROUP, N))) return rc;
      for (int g = 0; queued <= max_passes + 2 * POLL_GROUP; ++g) {
        HIPCHK(c, hipEventSynchronize(c->ev_poll[g & 1]));
        const uint32_t nlive = c->h_poll[4 * (g & 1)], unclaimed = c->h_poll[4 * (g & 1) + 1],
                       err = c->h_poll[4 * (g & 1) + 2];
        if (err) {
          overflow = true;
          break;
        }
        if (nlive == 0) {
          finished = true;
          break;
        }
        // paths left (live slots + unstarted paths, k_live_sum) below 1/16
        // of the pool: the chunk's tail, one pass per poll
        // (once the dispensers are dry with compaction on, one pass per poll
        // too: the compaction decision is then at most two passes old)
        const int np = (uint64_t)nlive * 16 < N || (c->compaction && unclaimed == 0) ? 1 : POLL_GROUP;
        // the dispensers are dry and at most compact_first % (later compactions:
        // compact_pct %) of the current layout's slots are live or unstarted:
        // compact them (the next group's first pass; it also starts every path
        // still left in a workgroup's block).  With the per-region slot counters
        // a compaction pass costs what a plain one does, so compacting early
        // pays: 70 / 65 against 50 / 50 measured +0.5 % CBbunny, +0.9 % dragon proxy
        compact_next = c->compaction && compact_mem && unclaimed == 0 && ncomp < MAX_COMPACTIONS &&
                       (uint64_t)nlive * 100 <= (uint64_t)nbound * (ncomp ? c->compact_pct : c->compact_first);
        if (compact_next && ensure_compact_set(c) != PT_OK) {
          // no memory for the second set: this render goes on without tail
          // compaction (a speed measure only) instead of failing with earlier
          // chunks already added to the accumulation and the sample count not
          // advanced
          (void)hipGetLastError();
          compact_mem = false;
          compact_next = false;
        }
        if (compact_next) {
          RAY[1] = c->d_ray_b;
          PS[0][1] = c->d_ps0_b;
          PS[1][1] = c->d_ps1_b;
          PS[2][1] = c->d_ps2_b;
          PS[3][1] = c->d_ps3_b;
        }
        S.dense = dense_ok && ((uint64_t)nlive > 2ull * N || (ncomp > 0 && (uint64_t)nlive * 2 > nbound)) ? 1u : 0u;
        if ((rc = enqueue_group(g + 2, np, nlive))) return rc;
        queued += (uint64_t)np;
      }
      if (overflow) {
        // a level overflowed its queue (the pass was abandoned): re-run the
        // chunk with twice the queue factor (nothing has been accumulated yet)
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (max_batch_paths(c, 1 + nsh) / 2 < 4096)
          return fail(c, PT_E_OVERFLOW, "ray queue capacity exceeded (u32 queue offsets)");
        c->qfactor *= 2;
        HIPCHK(c, zero_async(c, c->d_err, 4));
        // The passes queued behind the overflowing one ran on: their shade
        // kernels pushed rays into the root targets' queues that no level
        // consumed, so the (node, lane) counters are not all zero -- a re-run
        // would read that many stale ids from its reallocated queues (a
        // memory fault).  Zero them, and take back the abandoned passes' ray
        // and visit counts.
        HIPCHK(c, zero_async(c, c->d_cnt, (size_t)c->n_nodes * NLANE * CSTRIDE * 4));
        HIPCHK(c, copy_async(c, c->d_rcount, c->d_rcount_bak, RCOUNT_SLOTS * 16 * 8));
        HIPCHK(c, copy_async(c, c->d_stats, c->d_stats_bak, STAT_COUNT * 8));
        c->stats = stats0;
        c->marks.resize(marks0);
        c->evn = evn0;
        continue;
      }
      if (!finished) return fail(c, PT_E_HIP, "paths did not finish within the pass bound");
#if PT_SHADE_TIMING
      if (d_tprof) {
        unsigned long long h[1024], a[16] = {};
        HIPCHK(c, hipMemcpy(h, d_tprof, sizeof(h), hipMemcpyDeviceToHost));
        for (int i = 0; i < 1024; ++i) a[i % 16] += h[i];
        const double n = a[0] ? (double)a[0] : 1.0;
        fprintf(stderr,
                "PT_SHADE_TIMING workgroup-passes %llu  cycles per workgroup-pass: wstate %.0f  shade %.0f  claim %.0f  "
                "camera %.0f  root %.0f  (live slots per workgroup-pass %.1f); root: inline leaves + records %.0f  "
                "target tests + counts %.0f  reservations %.0f  pushes %.0f  tail %.0f  (first ray's inline leaves "
                "%.0f)\n",
                a[0], a[1] / n, a[2] / n, a[3] / n, a[4] / n, a[5] / n, a[6] / n, a[7] / n, a[8] / n, a[9] / n,
                a[10] / n, a[11] / n, a[12] / n);
        hipFree(d_tprof);
      }
#endif
      c->ray_cur = nullptr;
      if (timed)  // shaded vertices of the chunk (stats only)
        hipLaunchKernelGGL(k_live_sum, dim3(LIVE_SUM_BLOCKS), dim3(1024), 0, c->stream, (const uint4*)S.wstate, Gc,
                           (const uint32_t*)c->d_pool, nblocks, c->d_live, c->d_stats + STAT_SHADED);
    }
    if (!async) {  // (pipelined: the sums are pending, see above)
      c->launch(pt_ctx::K_ACCUM, 0, k_accum, dim3((npix + TPB - 1) / TPB), dim3(TPB), (const float4*)res,
                c->d_accum, (const uint32_t*)c->d_act_slot, npix, spp_c);
      HIPCHK(c, hipGetLastError());
    }
    done += (int)spp_c;
    first = false;
    c->stats.batches++;
  }
  HIPCHK(c, hipEventRecord(t1, c->stream));
  if (async) {  // (queued: pt_sync and the other waiting calls report its failure)
    c->samples += P->spp;
    return PT_OK;
  }
  HIPCHK(c, hipEventSynchronize(t1));
  if ((rc = drain(c))) {
    c->timing = false;
    return rc;
  }
  float total = 0;
  hipEventElapsedTime(&total, t0, t1);
  c->stats.ms_total = total;
  if (timed) collect_marks(c);
  c->timing = false;
  c->samples += P->spp;
  return PT_OK;
}

int pt_samples(pt_ctx* c, int32_t* spp) {
  if (!c || !spp) return PT_E_INVALID;
  *spp = c->samples;
  return PT_OK;
}

// The frame is assembled on the device (k_frame: sums / spp at their row-major
// positions) and copied to the host in one transfer (full PCIe rate when the
// caller's buffer is pinned).
int pt_get_image(pt_ctx* c, float* rgba, size_t n_floats) {
  if (!c || !rgba) return PT_E_INVALID;
  const size_t npx = (size_t)c->fb_w * c->fb_h;
  if (npx * 4 > n_floats) return fail(c, PT_E_INVALID, "image buffer too small");
  if (npx == 0) return PT_OK;
  hipSetDevice(c->device);
  int rc;
  if ((rc = drain(c))) return rc;
  if (npx > c->frame_cap) {
    if ((rc = dalloc(c, &c->d_frame, npx))) return rc;
    c->frame_cap = npx;
  }
  const uint32_t npix = (uint32_t)c->pix_of.size();
  if (npix < npx) HIPCHK(c, zero_async(c, c->d_frame, npx * sizeof(float4)));
  const float ns = (float)(c->samples > 0 ? c->samples : 1);
  if (npix)
    hipLaunchKernelGGL(k_frame, dim3((npix + TPB - 1) / TPB), dim3(TPB), 0, c->stream, (const float4*)c->d_accum,
                       (const uint32_t*)c->d_pix_of, npix, ns, c->d_frame);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(rgba, c->d_frame, npx * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PT_OK;
}

// The frame of accumulation buffer `acc` (sums / ns) assembled into staged
// frame fidx on `stream` and copied to rgba on copy_stream.
static int queue_image(pt_ctx* c, const float4* acc, float* rgba, float ns) {
  const size_t npx = (size_t)c->fb_w * c->fb_h;
  int rc;
  const int k = c->fidx;
  if (npx > c->frame_cap_a[k]) {
    if (c->cp_queued[k]) HIPCHK(c, hipEventSynchronize(c->ev_cp[k]));
    if ((rc = dalloc(c, &c->d_frame_a[k], npx))) return rc;
    c->frame_cap_a[k] = npx;
  }
  // the staged frame k is rewritten only after its last copy has read it
  if (c->cp_queued[k]) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_cp[k], 0));
  const uint32_t npix = (uint32_t)c->pix_of.size();
  if (npix < npx)
    hipLaunchKernelGGL(k_zero, dim3((uint32_t)((npx + TPB - 1) / TPB)), dim3(TPB), 0, c->stream, c->d_frame_a[k],
                       (uint32_t)npx);
  if (npix)
    hipLaunchKernelGGL(k_frame, dim3((npix + TPB - 1) / TPB), dim3(TPB), 0, c->stream, acc,
                       (const uint32_t*)c->d_pix_of, npix, ns, c->d_frame_a[k]);
  HIPCHK(c, hipGetLastError());
  // (pt_clear / pt_render on `stream` after this point cannot change the
  // staged frame: the copy reads d_frame_a[k], not the accumulation)
  HIPCHK(c, hipEventRecord(c->ev_fr[k], c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->copy_stream, c->ev_fr[k], 0));
  HIPCHK(c, hipMemcpyAsync(rgba, c->d_frame_a[k], npx * sizeof(float4), hipMemcpyDeviceToHost, c->copy_stream));
  HIPCHK(c, hipEventRecord(c->ev_cp[k], c->copy_stream));
  c->cp_queued[k] = true;
  c->fidx = k ^ 1;
  return PT_OK;
}

static int serve_images(pt_ctx* c) {
  for (int i = 0; i < c->n_img; ++i)
    if (int rc = queue_image(c, c->img_job[i].acc, c->img_job[i].rgba, c->img_job[i].ns)) return rc;
  c->n_img = 0;
  return PT_OK;
}

// The pending sums of the last pipelined launch as a k_accum of their own
// (no launch follows to carry them), then the images waiting for them.
static int flush_sums(pt_ctx* c) {
  if (c->acc_on) {
    const pt_ctx::AccJob& j = c->acc_job;
    hipLaunchKernelGGL(k_accum, dim3((j.npix + TPB - 1) / TPB), dim3(TPB), 0, c->stream, j.res, j.dst,
                       (const uint32_t*)c->d_act_slot, j.npix, j.spp);
    HIPCHK(c, hipGetLastError());
    c->acc_on = false;
  }
  return serve_images(c);
}

int pt_get_image_async(pt_ctx* c, float* rgba, size_t n_floats) {
  if (!c || !rgba) return PT_E_INVALID;
  if (!c->copy_stream) return fail(c, PT_E_HIP, "pt_get_image_async: no copy stream");
  const size_t npx = (size_t)c->fb_w * c->fb_h;
  if (npx * 4 > n_floats) return fail(c, PT_E_INVALID, "image buffer too small");
  if (npx == 0) return PT_OK;
  hipSetDevice(c->device);
  const float ns = (float)(c->samples > 0 ? c->samples : 1);
  if (c->acc_on && c->acc_job.dst == c->d_accum) {
    // its sums are pending (pipelined frames): the frame is assembled after
    // the launch that makes them (two requests at most; a third flushes them)
    if (c->n_img == 2)
      if (int rc = flush_sums(c)) return rc;
    if (c->acc_on) {
      c->img_job[c->n_img++] = pt_ctx::ImgJob{c->d_accum, rgba, ns};
      return PT_OK;
    }
  }
  return queue_image(c, c->d_accum, rgba, ns);
}

int pt_wait_image(pt_ctx* c) {
  if (!c) return PT_E_INVALID;
  hipSetDevice(c->device);
  // (the frames the copies come from, their pending sums and images queued
  // first: their failure)
  if (int rc = drain(c)) return rc;
  for (int k = 0; k < 2; ++k)
    if (c->cp_queued[k]) HIPCHK(c, hipEventSynchronize(c->ev_cp[k]));
  return PT_OK;
}

int pt_sync(pt_ctx* c) {
  if (!c) return PT_E_INVALID;
  hipSetDevice(c->device);
  return drain(c);
}

int pt_copy_owned_sums(pt_ctx* c, void* dst, size_t n_bytes, int32_t dst_on_device) {
  if (!c || (!dst && n_bytes)) return PT_E_INVALID;
  const size_t need = c->pix_of.size() * sizeof(float4);
  if (n_bytes < need) return fail(c, PT_E_INVALID, "pt_copy_owned_sums: buffer too small");
  if (need == 0) return PT_OK;
  hipSetDevice(c->device);
  if (int rc = drain(c)) return rc;
  HIPCHK(c, hipMemcpyAsync(dst, c->d_accum, need, dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PT_OK;
}

int pt_median_filter(pt_ctx* c, const float* rgba_in, float* rgba_out, int32_t width, int32_t height) {
  if (!c || !rgba_in || !rgba_out || width <= 0 || height <= 0) return PT_E_INVALID;
  hipSetDevice(c->device);
  const size_t n = (size_t)width * height;
  float4 *d_in = nullptr, *d_out = nullptr;
  HIPCHK(c, hipMalloc((void**)&d_in, n * sizeof(float4)));
  if (hipMalloc((void**)&d_out, n * sizeof(float4)) != hipSuccess) {
    hipFree(d_in);
    return fail(c, PT_E_HIP, "pt_median_filter: out of device memory");
  }
  int rc = PT_OK;
  if (hipMemcpyAsync(d_in, rgba_in, n * sizeof(float4), hipMemcpyHostToDevice, c->stream) != hipSuccess)
    rc = fail(c, PT_E_HIP, "pt_median_filter: copy in");
  if (!rc) {
    hipLaunchKernelGGL(k_median3, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, c->stream, d_in, d_out, width,
                       height);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(rgba_out, d_out, n * sizeof(float4), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      rc = fail(c, PT_E_HIP, "pt_median_filter: kernel / copy out");
  }
  hipFree(d_in);
  hipFree(d_out);
  return rc;
}

int pt_get_display_image(pt_ctx* c, float* rgba, size_t n_floats) {
  if (!c || !rgba) return PT_E_INVALID;
  if (c->fb_nranks != 1) return fail(c, PT_E_INVALID, "display image needs the whole frame (nranks == 1)");
  int rc = pt_get_image(c, rgba, n_floats);
  if (rc) return rc;
  if (c->samples < PT_POST_PROCESS_THRESHOLD) rc = pt_median_filter(c, rgba, rgba, c->fb_w, c->fb_h);
  return rc;
}

int pt_owned_pixels(pt_ctx* c, int32_t* n_pixels, int32_t* pixel_index, size_t max_idx, void** device_sums) {
  if (!c || !n_pixels) return PT_E_INVALID;
  *n_pixels = (int32_t)c->pix_of.size();
  if (pixel_index)
    for (size_t i = 0; i < c->pix_of.size() && i < max_idx; ++i) pixel_index[i] = (int32_t)c->pix_of[i];
  if (device_sums) {  // (complete sums: the caller reads them on streams of its own)
    hipSetDevice(c->device);
    if (int rc = drain(c)) return rc;
    *device_sums = c->d_accum;
  }
  return PT_OK;
}

int pt_intersect(pt_ctx* c, const float* rays, int32_t n, uint64_t* hits) { return pt_intersect_ex(c, rays, n, hits, 0); }

int pt_intersect_ex(pt_ctx* c, const float* rays, int32_t n, uint64_t* hits, uint32_t flags) {
  if (c) c->ray_cur = nullptr;  // (a failed render may have left the compaction's second set bound)
  if (!c || (!rays && n > 0) || (!hits && n > 0) || n < 0) return PT_E_INVALID;
  if (!c->have_scene) return fail(c, PT_E_NOSCENE, "no scene loaded");
  hipSetDevice(c->device);
  if (int rc = drain(c)) return rc;
  c->refa = (flags & PT_FLAG_REF_ARITH) != 0;
  if (c->refa && c->has_sphere)
    return fail(c, PT_E_UNSUPPORTED, "PT_FLAG_REF_ARITH: the reference intersects triangles only");
  if (n == 0) return PT_OK;
  hipSetDevice(c->device);
  int rc;
  c->shadow_base = 0xFFFFFFFFu;  // every ray wants its closest hit
  // t_min (the rays' 8th float, Ray::min_t): hits with t < t_min do not count.
  // Clamped at 0 (no hit has t < 0); a batch without any t_min > 0 runs the
  // render kernels' traversal unchanged
  std::vector<float> tmin;
  for (int32_t i = 0; i < n; ++i) {
    const float* r = rays + (size_t)8 * i;
    if (!(std::fabs((double)r[0]) <= c->origin_bound && std::fabs((double)r[1]) <= c->origin_bound &&
          std::fabs((double)r[2]) <= c->origin_bound))
      return fail(c, PT_E_UNSUPPORTED, "pt_intersect: ray origin beyond 64x the scene's extent (conservative box guard)");
    const float t = r[7];
    if (t != t) return fail(c, PT_E_INVALID, "pt_intersect: t_min is NaN");
    if (c->has_sphere) {  // the sphere test assumes a unit direction (trace.hip sphere_test)
      const double l2 = (double)r[4] * r[4] + (double)r[5] * r[5] + (double)r[6] * r[6];
      if (!(std::fabs(l2 - 1.0) <= 1e-5))
        return fail(c, PT_E_INVALID, "pt_intersect: a scene with spheres needs unit ray directions");
    }
    if (t > 0.0f) {
      if (tmin.empty()) tmin.assign((size_t)n, 0.0f);
      tmin[i] = t;
    }
  }
  c->tmin = !tmin.empty();
  if (c->tmin) {
    if ((size_t)n > c->tmin_cap) {
      if ((rc = dalloc(c, &c->d_tmin, (size_t)n))) return rc;
      c->tmin_cap = (size_t)n;
    }
    HIPCHK(c, hipMemcpy(c->d_tmin, tmin.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  }
  const uint32_t N = ((uint32_t)n + 1) / 2;
  const bool realloc = N > c->cap_paths || 2 > c->cap_spp || c->qfactor != c->cap_qfactor;
  if ((rc = ensure_paths(c, N, 2))) return rc;
  if (realloc && (rc = set_root_child_offsets(c))) return rc;
  float4* d_in = nullptr;
  HIPCHK(c, hipMalloc((void**)&d_in, (size_t)n * 32));  // rays in, then hit keys out
  // (the counters before the first try: a retry after a queue overflow counts its rays once)
  HIPCHK(c, copy_async(c, c->d_rcount_bak, c->d_rcount, RCOUNT_SLOTS * 16 * 8));
  HIPCHK(c, copy_async(c, c->d_stats_bak, c->d_stats, STAT_COUNT * 8));
  for (;;) {
    HIPCHK(c, hipMemcpyAsync(d_in, rays, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, zero_async(c, c->d_err, 4));
    hipLaunchKernelGGL(k_load_rays, dim3((n + TPB - 1) / TPB), dim3(TPB), 0, c->stream, d_in, c->d_ray,
                       (uint32_t)n);
    hipEventRecord(c->ev[6], c->stream);
    rc = trace_pass(c, 0, (uint32_t)n);
    hipEventRecord(c->ev[7], c->stream);
    if (rc) {
      hipFree(d_in);
      return rc;
    }
    uint32_t e = 0;  // (the context's stream is non-blocking: read the flag on it)
    if (hipMemcpyAsync(&e, c->d_err, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
      hipFree(d_in);
      return fail(c, PT_E_HIP, "pt_intersect: error flag");
    }
    if (!e) break;
    // a level overflowed its queue: twice the queue factor, trace again
    // (while the doubled factor's u32 queue offsets still hold N paths)
    if (max_batch_paths(c, 2) / 2 < N) {
      hipFree(d_in);
      return fail(c, PT_E_OVERFLOW, "ray queue capacity exceeded");
    }
    c->qfactor *= 2;
    if ((rc = ensure_paths(c, N, 2)) || (rc = set_root_child_offsets(c))) {
      hipFree(d_in);
      return rc;
    }
    HIPCHK(c, copy_async(c, c->d_rcount, c->d_rcount_bak, RCOUNT_SLOTS * 16 * 8));
    HIPCHK(c, copy_async(c, c->d_stats, c->d_stats_bak, STAT_COUNT * 8));
  }
  hipLaunchKernelGGL(k_store_hits, dim3((n + TPB - 1) / TPB), dim3(TPB), 0, c->stream, c->d_ray,
                     (unsigned long long*)d_in, (uint32_t)n);
  HIPCHK(c, hipMemcpyAsync(hits, d_in, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  float ms = 0;
  hipEventElapsedTime(&ms, c->ev[6], c->ev[7]);
  c->stats.ms_total = ms;
  hipFree(d_in);
  return PT_OK;
}

}  // extern "C"
