/*
 * pt_api.h -- C ABI of the MI355X (gfx950) breadth-first wide-BVH path tracer.
 *
 * This is the drop-in boundary for the hot path of saipraveenb25/cuda-raytracer
 * ("CUDA-SCOTTY").  Every entry point replaces one member of the reference's
 * `cutracer::CudaRenderer` class (src/cudaRenderer.h:173-272) or one piece of the
 * Scotty3D CPU surface the north star keeps (src/pathtracer.h:51-257,
 * src/camera.h:81, src/bvh.h:111-149).  The signatures carry only plain C types
 * and pointers; no HIP, torch or C++ types cross the boundary.
 *
 *   reference member / function                        replaced by
 *   -------------------------------------------------  -------------------------
 *   CudaRenderer::CudaRenderer()        cu:1496         pt_create
 *   CudaRenderer::~CudaRenderer()       cu:1510         pt_destroy
 *   CudaRenderer::loadScene(path)       cu:1679-1842    pt_scene_load_dae + pt_load_scene
 *     (COLLADA parse, BVHAccel build, compactedTree, compress, flatten)
 *   CudaRenderer::setup()               cu:1872-2113    pt_load_scene (device upload)
 *   CudaRenderer::allocOutputImage(w,h) cu:2119         pt_render_params.width/height
 *   CudaRenderer::render()/renderAccumulate()/renderFrame()
 *                                       cu:2411-2564    pt_render
 *   CudaRenderer::getImage()            cu:1539-1570    pt_get_image
 *   CudaRenderer::setViewpoint(o,look)  cu:1845-1870    pt_set_camera (+ pt_clear)
 *   CudaRenderer::clearImage()          cu:2131         pt_clear
 *   rayIntersect() + kernelMergeIntersections
 *                                       cu:2304-2331,515 pt_intersect (closest hit)
 *   BVHAccel::intersect(ray, isect)     bvh.cpp:422     pt_intersect (one ray)
 *   lapTimer per-kernel timing          cu:2366-2376    pt_get_stats
 *
 * Conventions
 *  - Every call returns 0 (PT_OK) or a negative PT_E* code; the message of the
 *    last failure on a context is available from pt_last_error().  Nothing in
 *    this library calls exit() (the reference exits on every failure, §5).
 *  - pt_scene_* objects are host-side and own their arrays.  pt_load_scene copies
 *    the arrays to the device; the caller keeps ownership of the pt_scene.
 *  - One pt_ctx per GPU.  Calls on one ctx must be serialised by the caller;
 *    distinct contexts may be used from distinct threads / processes.
 *  - Images are float4 RGBA, row-major, rows counted bottom-up; pixel (row r,
 *    col c) is element r*width + c.  For square images this is the same memory
 *    order as the reference's x*H + y indexing (cu:327, 705-718).
 */
#ifndef PT_API_H
#define PT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: pt_bsdf grew `roughness` (36 B), pt_stats `culled_rays` (round 4);
 * PT_FLAG_EXACT_LIGHT_PDF and the light.cpp pdf as the default (round 5).
 * 3: pt_group_* (several GPUs of one process, RCCL gather; round 5).
 * 4: pt_scene_desc.n_lights / lights, PT_LIGHT_DIRECTIONAL / _HEMISPHERE.
 * 5: PT_FLAG_COUNT_TESTS and pt_stats.prim_tests_tri / _sph, cluster_box_tests;
 *    pt_get_image_async / pt_wait_image (round 6).
 * 6: PT_FLAG_ASYNC and pt_sync (pipelined single-leaf frames, round 6).
 * A client checks pt_api_version() == PT_API_VERSION before passing structs. */
#define PT_API_VERSION 6
int pt_api_version(void);

/* ---- error codes ---------------------------------------------------------- */
#define PT_OK 0
#define PT_E_INVALID (-1)     /* bad argument                                 */
#define PT_E_IO (-2)          /* file not found / parse error                 */
#define PT_E_NOSCENE (-3)     /* render/intersect before pt_load_scene        */
#define PT_E_HIP (-4)         /* HIP runtime error (message has details)      */
#define PT_E_OVERFLOW (-5)    /* ray queue capacity exceeded during a pass     */
#define PT_E_UNSUPPORTED (-6) /* scene feature not supported                  */
#define PT_E_NODEVICE (-7)    /* no GPU visible / HIP kernels not loaded       */

/* ---- device record formats (also the flattened scene format) -------------- */

/* Primitive kinds (bits 28..31 of pt_prim.meta; bits 0..27 = bsdf index). */
#define PT_PRIM_TRIANGLE 0u
#define PT_PRIM_SPHERE 1u

/* One intersectable primitive, 96 bytes = 6 x float4, in BVH-sorted order
 * (the order of BVHAccel::getSortedPrimitives(), bvh.cpp:384): the flattened
 * scene's record (the device keeps its own forms of it: pt_load_scene derives
 * the Baldwin-Weber rows the default test evaluates and the literal operands
 * of PT_FLAG_REF_ARITH from the vertices).  Triangles store the
 * operands of the reference triangle test (cu:217-270):
 *   q0 = v0.xyz, meta        q1 = v1.xyz, dN = dot(N, v0)
 *   q2 = v2.xyz, m0.x        q3 = N.xyz (= cross(v1-v0, v2-v0)), m0.y
 *   q4 = m1.xyz, m0.z        q5 = m2.xyz, 0
 * with edge normals m_k = cross(N, e_k) for e0 = v1-v0, e1 = v2-v1, e2 = v0-v2:
 * the reference's edge test dot(N, cross(e_k, P - v_k)) < 0 is evaluated as
 * dot(m_k, P - v_k) < 0 (the same quantity; it differs only in fp32 rounding).
 * All derived values are fp32 computed from the fp32 vertices.  Spheres:
 * q0 = centre.xyz, meta; q1.x = radius, q1.y = radius^2; rest 0.            */
typedef struct pt_prim {
  float q[24];
} pt_prim;

/* Shading data of a primitive (same index as pt_prim): the three vertex
 * normals of a triangle (CuTriangle.n0..n2, cudaRenderer.h:118-120). */
typedef struct pt_prim_shading {
  float n0[4];
  float n1[4];
  float n2[4];
} pt_prim_shading;

/* One 4-wide BVH node, 128 bytes (one cache line of the MI355X L2).  Children
 * are stored as SoA boxes.  child[i] < 0 marks an empty outlet (the reference's
 * (uint64_t)-1, bvh.cpp:267).  prim_count > 0 marks a leaf (range != 0,
 * cu:862).  Nodes are stored level-major (breadth-first), so the nodes of BVH
 * level l are the contiguous id range [level_start[l], level_start[l+1]). */
typedef struct pt_node {
  float bmin_x[4], bmax_x[4];
  float bmin_y[4], bmax_y[4];
  float bmin_z[4], bmax_z[4];
  int32_t child[4];
  int32_t prim_start;
  int32_t prim_count;
  int32_t level;
  int32_t ref_id; /* DFS pre-order id of BVHSubTree::compress (bvh.cpp:234) */
} pt_node;

/* BSDF kinds */
#define PT_BSDF_DIFFUSE 0
#define PT_BSDF_MIRROR 1
#define PT_BSDF_GLASS 2
#define PT_BSDF_EMISSION 3
#define PT_BSDF_REFRACTION 4 /* RefractionBSDF (bsdf.h:167-185): glass without reflectance */

/* 36 bytes; CuBSDF (cudaRenderer.h:135-140) extended with glass and emission.
 * roughness: the COLLADA <roughness> of glass / refraction (collada.cpp:910-933).
 * The kernels' default arithmetic does not model it (a smooth dielectric);
 * PT_FLAG_REF_ARITH reads a glass BSDF as the reference's CUDA path does: a
 * MirrorBSDF reinterpret_cast over the GlassBSDF object (cu:1713-1719), whose
 * reflectance is then (roughness, reflectance.r, reflectance.g) (bsdf.h:138-139
 * against bsdf.h:206-210), and (roughness, transmittance.r, transmittance.g)
 * over a RefractionBSDF (bsdf.h:180-182). */
typedef struct pt_bsdf {
  int32_t type;
  float albedo[3];        /* diffuse albedo / mirror+glass reflectance / emitted radiance */
  float transmittance[3]; /* glass, refraction */
  float ior;              /* glass, refraction */
  float roughness;        /* glass, refraction (PT_FLAG_REF_ARITH only) */
} pt_bsdf;

/* Light kinds */
#define PT_LIGHT_NONE 0
#define PT_LIGHT_AREA 1
#define PT_LIGHT_POINT 2
/* Scotty3D's infinite lights (the CPU path tracer's; static_scene/light.cpp:
 * 12-45), from COLLADA <directional> and <ambient> lights:
 *   DIRECTIONAL: `direction` = the unit direction TOWARD the light
 *     (DirectionalLight::dirToLight), pdf 1, shadow rays of infinite length;
 *   HEMISPHERE: InfiniteHemisphereLight -- radiance from every direction of
 *     the upper (+y) hemisphere, sampled uniformly (pdf 1 / 2 pi). */
#define PT_LIGHT_DIRECTIONAL 3
#define PT_LIGHT_HEMISPHERE 4

/* CuEmitter (cudaRenderer.h:126-133) + kind. */
typedef struct pt_light {
  int32_t type;
  float radiance[3];
  float position[3];
  float direction[3];
  float dim_x[3];
  float dim_y[3];
  float area;
  float pad[2];
} pt_light;

/* Camera in the reference GPU model (cu:80-86, set up at cu:1590-1607): fixed
 * 53.13 degree field of view, direction = k.x*left + k.y*up + k.z*lookAt. */
typedef struct pt_camera {
  float origin[3];
  float look_at[3];
  float left[3];
  float up[3];
} pt_camera;

/* Flattened scene handed to the device (what CudaRenderer::loadScene builds).
 * Lights: the reference's CUDA path takes exactly one (cu:1734-1737) --
 * `light`.  A scene with several (the Scotty3D CPU path tracer sums over
 * scene->lights, pathtracer.cpp:441-476) lists them all in lights[0 ..
 * n_lights) with light == lights[0]; each next-event sample then picks one
 * uniformly (the low byte of its first Philox word, weighted by the exact
 * inverse of its selection probability), which has the sum's expectation.
 * n_lights 0 or 1: `light` alone (lights may be NULL). */
typedef struct pt_scene_desc {
  int32_t n_prims;
  const pt_prim* prims;
  const pt_prim_shading* shading;
  int32_t n_nodes;
  const pt_node* nodes;
  int32_t n_levels;
  const int32_t* level_start; /* n_levels + 1 entries */
  int32_t n_bsdfs;
  const pt_bsdf* bsdfs;
  pt_light light;
  pt_camera camera;
  int32_t n_lights;
  const pt_light* lights;
} pt_scene_desc;

/* ---- host-side scene loading (input adapter, runs on the CPU) -------------- */
typedef struct pt_scene pt_scene; /* opaque, owns its arrays */

/* Parse a COLLADA file (the CMU462 subset used by media/pathtracer), build the
 * reference BVH (bvh.cpp:48-365, max leaf 32), compact it to the 4-wide tree
 * (bvh.cpp:275-337) and flatten it.  On failure *out is NULL and errbuf (if not
 * NULL) receives a message. */
int pt_scene_load_dae(const char* path, pt_scene** out, char* errbuf, size_t errbuf_len);
/* Build a scene from a plain triangle soup (tests, synthetic scenes).  All
 * triangles use bsdf 0; positions are n_tris*9 floats. */
int pt_scene_from_triangles(const float* positions, int32_t n_tris, const pt_bsdf* bsdf0,
                            const pt_light* light, const pt_camera* camera, pt_scene** out);
/* General flattened input (the scene-flattening step of SURVEY §8(f) row 2
 * for callers that already hold meshes, e.g. the Scotty3D loader or a
 * synthetic workload): a triangle soup with optional vertex normals and
 * per-triangle bsdf ids, optional spheres, a bsdf table, one light and a
 * camera.  Built with the same reference BVH (max leaf 32) as .dae scenes. */
typedef struct pt_mesh_desc {
  int32_t n_tris;
  const float* positions;   /* n_tris * 9: v0, v1, v2                        */
  const float* normals;     /* n_tris * 9 vertex normals, or NULL (face normal) */
  const int32_t* tri_bsdf;  /* n_tris bsdf ids, or NULL (all 0)              */
  int32_t n_spheres;
  const float* spheres;     /* n_spheres * 4: centre, radius                 */
  const int32_t* sphere_bsdf; /* n_spheres bsdf ids, or NULL (all 0)          */
  int32_t n_bsdfs;
  const pt_bsdf* bsdfs;     /* n_bsdfs >= 1                                   */
  const pt_light* light;    /* NULL: no light                                 */
  const pt_camera* camera;  /* NULL: default                                  */
} pt_mesh_desc;
int pt_scene_from_mesh(const pt_mesh_desc* mesh, pt_scene** out);
/* The same with the reference builder's leaf size (BVHAccel(primitives,
 * max_leaf_size), bvh.h:111; 0 = 32, the reference default). */
int pt_scene_from_mesh_ex(const pt_mesh_desc* mesh, int32_t max_leaf, pt_scene** out);
/* The same input built on GPU `device`: a binary BVH
 * on the device collapsed to the 4-wide, level-major layout (wide leaves hold
 * <= max_leaf primitives; the reference's host SAH build, bvh.cpp:48-337, is
 * pt_scene_from_mesh).  *build_ms (optional) receives the build's wall time.
 * pt_scene_build_gpu uses PT_GPU_BVH_SAH (round 6; PLOC before). */
#define PT_GPU_BVH_PLOC 0 /* agglomerative clustering in Morton order (PLOC) */
#define PT_GPU_BVH_LBVH 1 /* Karras radix tree over Morton codes            */
#define PT_GPU_BVH_SAH 2  /* top-down binned SAH, the reference's 12-plane
                             split rule (bvh.cpp:48-230), level-synchronous */
int pt_scene_build_gpu(const pt_mesh_desc* mesh, int32_t device, int32_t max_leaf, pt_scene** out,
                       double* build_ms);
int pt_scene_build_gpu_ex(const pt_mesh_desc* mesh, int32_t device, int32_t max_leaf, int32_t builder,
                          pt_scene** out, double* build_ms);
/* The Scotty3D framing of a COLLADA scene's camera (SURVEY §8(a) parity
 * decision vii, camera=scotty): Application::load places the camera at the
 * scene bbox centroid + 3 x half the bbox diagonal along the COLLADA view
 * direction, looking back at the centroid (application.cpp:395-408,
 * camera.cpp:35-46, 86-108); Camera::configure fits hFov/vFov to width/height
 * (camera.cpp:15-33); generate_ray(x, y) is the documented pinhole mapping
 * (camera.h:71-81).  The result is a pt_camera for pt_set_camera (the kernels'
 * camera model spans the same rays).  PT_E_UNSUPPORTED without COLLADA optics. */
int pt_scene_camera_scotty(const pt_scene* s, int32_t width, int32_t height, pt_camera* out);
void pt_scene_free(pt_scene* s);
/* Borrowed view of the flattened arrays (valid until pt_scene_free). */
int pt_scene_get_desc(const pt_scene* s, pt_scene_desc* out);
/* Reference-layout statistics of the compacted tree: number of wide nodes,
 * leaves and per-level node counts (the reference's levelCounts). */
int pt_scene_level_counts(const pt_scene* s, int32_t* counts, int32_t max_levels,
                          int32_t* n_levels);
/* Primitive permutation: sorted_to_input[i] = index of sorted prim i in the
 * scene's input order (triangles in mesh order, then spheres). */
int pt_scene_sorted_to_input(const pt_scene* s, int32_t* out, int32_t n);

/* ---- device context --------------------------------------------------------- */
typedef struct pt_ctx pt_ctx;

int pt_create(pt_ctx** out, int device);
void pt_destroy(pt_ctx* ctx);
const char* pt_last_error(const pt_ctx* ctx);
int pt_device_count(int* n);

int pt_load_scene(pt_ctx* ctx, const pt_scene_desc* scene);
/* PT_E_UNSUPPORTED when the origin lies beyond 64 x the scene's largest
 * coordinate magnitude M (vertices, sphere extents, the scene's camera and
 * light): the stored boxes' guard band keeps the fp32 box test conservative
 * for origins within ~180 M.  pt_intersect applies the same bound to its
 * ray origins. */
int pt_set_camera(pt_ctx* ctx, const pt_camera* camera);

/* Render parameters. */
#define PT_FLAG_COSINE_DIFFUSE 0x1u /* cosine-weighted diffuse sampling instead of
                                       the reference's uniform hemisphere (cu:619) */
#define PT_FLAG_NO_EMISSION 0x2u    /* do not count emissive surfaces (REAL_TIME,
                                       cudaRenderer.h:76, cu:1242-1246)        */
#define PT_FLAG_STATS 0x4u          /* collect R/V counters and per-pass timing  */
/* Reference-quirk modes (SURVEY §8(a) parity decisions; default off, the CPU
 * oracle implements each the same way):                                     */
#define PT_FLAG_REF_DROP_ON_MISS 0x8u /* (i) a path whose extension ray misses
                                         contributes 0 (cu:679-698)          */
#define PT_FLAG_REF_GUIDE 0x10u       /* (ii) the reference's local frame,
                                         cu:572-574 (NaN for n = (0,-1,0))   */
#define PT_FLAG_REF_SCHEDULE 0x20u    /* (vi) renderFrame's schedule, cu:2499-2533:
                                         2 bounces, NEE samples 2, 2, 1 at
                                         vertices 1, 2, 3 weighted 0.5, 0.5, 1;
                                         max_bounces is ignored              */
#define PT_FLAG_REF_ARITH 0x40u       /* the reference kernels' literal fp32
                                         arithmetic instead of the build's:
                                         the edge test dot(N, cross(e_k, P-v_k))
                                         (cu:251-267), the unnormalised camera
                                         direction (cu:354), NEE with the
                                         unnormalised two-sided cosine, |n.w| and
                                         BSDF_DIFFUSE_MULTIPLIER 0.3183 (cu:416-446,
                                         272), shadow rays unoccluded when
                                         t > maxT - 1e-3 in double (cu:1279), the
                                         barycentric normal without the
                                         flat-triangle shortcut (cu:1213-1224),
                                         unnormalised diffuse / local-frame
                                         mirror directions (cu:631-650), an
                                         emission BSDF read as diffuse with
                                         albedo = radiance (cu:1705-1711).
                                         Triangles with diffuse / mirror /
                                         emission BSDFs only (PT_E_UNSUPPORTED
                                         for spheres and glass)              */
/* The default NEE toward an area light uses the reference's light pdf,
 * AreaLight::sample_L (light.cpp:81-92, also cu:422-430): pdf = sqDist /
 * (area * |dot(d, direction)|) with d the UNnormalised vector to the light
 * sample, i.e. the solid-angle pdf times the distance.  The reference's own
 * renders (media/pathtracer/reference_results) follow it (tests/
 * test_gpu_reference_renders.py).  This flag takes the normalised cosine,
 * the unbiased estimator of the irradiance, instead.                         */
#define PT_FLAG_EXACT_LIGHT_PDF 0x80u
/* Count the primitive tests the single-leaf path kernel executes (the
 * candidate clusters skip most of the leaf: DESIGN.md §4) into
 * pt_stats.prim_tests_tri / prim_tests_sph / cluster_box_tests.  A counting
 * build of the kernel runs instead of the timed one (slower: its time is not
 * the kernel's); results are unchanged.  The wavefront kernels and the
 * reference-arithmetic, guided and extended-light path variants count nothing. */
#define PT_FLAG_COUNT_TESTS 0x100u
/* Queue the frame and return (round 6; no reference counterpart: renderFrame,
 * cu:2499-2533, returns when the frame is done).  Single-leaf scenes only
 * (the wavefront renderer polls the device between passes and stays
 * synchronous; PT_FLAG_STATS renders too): the path kernel of a frame runs
 * on a stream of its own and writes one of two per-path result buffers, so
 * the next frame's path kernel starts while the previous frame's results are
 * summed into the accumulation buffer (same sums, same order, same bits).
 * pt_clear and pt_get_image_async queue behind it without waiting; every
 * other call on the context (pt_sync, pt_wait_image, pt_get_image,
 * pt_get_stats, pt_load_scene, a synchronous pt_render, ...) first waits for
 * the queued frames and reports a failure of theirs.  pt_stats.ms_total is
 * not measured for an asynchronous frame. */
#define PT_FLAG_ASYNC 0x200u

typedef struct pt_render_params {
  int32_t width, height;
  int32_t spp;         /* samples per pixel rendered by this call             */
  int32_t max_bounces; /* indirect (BSDF-sampled) rays per path; vertices = +1 */
  uint32_t seed;       /* Philox key; reference seed 15618 (samplers.cu_inl:8) */
  int32_t sample_offset; /* index of the first sample (progressive rendering) */
  int32_t batch_paths; /* wavefront path pool: path slots in flight (each slot
                          runs path after path); 0 = auto (36 Mi)            */
  int32_t tile_size;   /* framebuffer tile edge for sharding (0 = 32)          */
  int32_t rank, nranks; /* this context renders tiles t with t % nranks == rank */
  uint32_t flags;
} pt_render_params;

/* Render params->spp samples per owned pixel and ADD them to the context's
 * accumulation buffer (progressive, like renderAccumulate, cu:2419-2457).
 * Blocks until the GPU work is complete (unless PT_FLAG_ASYNC). */
int pt_render(pt_ctx* ctx, const pt_render_params* params);
/* Wait for every frame queued with PT_FLAG_ASYNC; PT_OK or its failure. */
int pt_sync(pt_ctx* ctx);
/* Zero the accumulation buffer and sample count (kernelClearAccumulate, cu:744).
 * Queued on the context's stream (ordered after the frames before it). */
int pt_clear(pt_ctx* ctx);
/* Copy the current image (accumulated radiance / samples) of the whole frame,
 * width*height*4 floats.  Pixels this rank does not own are 0. */
int pt_get_image(pt_ctx* ctx, float* rgba, size_t n_floats);
/* pt_get_image without the wait (round 6): the frame is assembled on the
 * device by the same kernel, and its copy into `rgba` (host memory, ideally
 * pinned) is queued on a copy stream of the context; the call returns at
 * once, and a following pt_clear / pt_render overlaps the copy (it reads a
 * staged frame of its own; two alternate).  `rgba` holds the frame after
 * pt_wait_image, which waits for every queued copy.  No reference
 * counterpart: getImage (cu:1539-1570) is synchronous. */
int pt_get_image_async(pt_ctx* ctx, float* rgba, size_t n_floats);
int pt_wait_image(pt_ctx* ctx);
/* Owned-pixel view for the multi-GPU gather: *n_pixels owned pixels, their
 * global indices (row*width+col, host array filled if not NULL) and a device
 * pointer to their float4 radiance sums (not divided by spp). */
int pt_owned_pixels(pt_ctx* ctx, int32_t* n_pixels, int32_t* pixel_index, size_t max_idx,
                    void** device_sums);
/* Copy the owned pixels' float4 radiance sums (slot order of pt_owned_pixels,
 * not divided by spp) into dst: device memory of this context's GPU
 * (dst_on_device != 0, e.g. a torch tensor handed to the RCCL gather) or host
 * memory.  n_bytes >= 16 * owned pixels.  Synchronous. */
int pt_copy_owned_sums(pt_ctx* ctx, void* dst, size_t n_bytes, int32_t dst_on_device);
/* Samples per pixel accumulated so far. */
int pt_samples(pt_ctx* ctx, int32_t* spp);

/* ---- one frame over several GPUs of one process -------------
 * For C/C++ callers (the Scotty3D surface, scotty::PathTracer with a device
 * list): a group of contexts, member i on devices[i], renders the frame's
 * tiles t with t % n == i (pt_render_params.rank / nranks are set per member,
 * the caller's are ignored), each member on its own host thread; the members'
 * owned-pixel sums are then gathered into member 0's device frame.  The
 * gather is RCCL point-to-point over xGMI (ncclCommInitAll over the members'
 * devices, one ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd round into
 * member 0, librccl loaded at pt_group_create) when the devices are distinct
 * and RCCL loads; otherwise (a device listed twice -- RCCL takes one rank per
 * GPU -- or no librccl) a host-staged copy.  The reference has no multi-GPU
 * path (cu:1874-1897 only enumerates devices); the Python bench gathers the
 * same sums over torch.distributed (ptdist.py).  PT_GATHER_* select the
 * gather; pt_group_gather_kind reports the one in use. */
typedef struct pt_group pt_group;
#define PT_GATHER_AUTO 0 /* RCCL when the devices are distinct and librccl loads */
#define PT_GATHER_RCCL 1 /* RCCL or PT_E_UNSUPPORTED                             */
#define PT_GATHER_HOST 2 /* host-staged copies                                   */
int pt_group_create(pt_group** out, const int32_t* devices, int32_t n, int32_t gather);
void pt_group_destroy(pt_group* g);
const char* pt_group_last_error(const pt_group* g);
int pt_group_gather_kind(const pt_group* g, int32_t* kind); /* PT_GATHER_RCCL / _HOST */
int pt_group_size(const pt_group* g, int32_t* n);
pt_ctx* pt_group_member(pt_group* g, int32_t i); /* borrowed; NULL if out of range */
int pt_group_load_scene(pt_group* g, const pt_scene_desc* scene);
int pt_group_set_camera(pt_group* g, const pt_camera* camera);
int pt_group_clear(pt_group* g);
/* Every member renders its tiles (and adds them to its accumulation), then
 * the sums are gathered into member 0's frame: sums / accumulated samples,
 * alpha 1, as pt_get_image of one context rendering the whole frame. */
int pt_group_render(pt_group* g, const pt_render_params* params);
/* The gathered frame, width*height*4 floats (host copy from member 0). */
int pt_group_get_image(pt_group* g, float* rgba, size_t n_floats);
/* Wall time (ms) of the last pt_group_render's gather (send + receive +
 * assembly on member 0), and of the whole call. */
int pt_group_timing(const pt_group* g, double* gather_ms, double* render_ms);

/* ---- post-process and output --------------------------
 * 3x3 median filter of a width*height float RGBA frame on the device
 * (kernelMedianFilter, cu:773-842): per channel the 4th largest of the 3x3
 * neighbourhood, out-of-frame neighbours count as 1.0, alpha = 1.  In place
 * is allowed (rgba_out == rgba_in). */
int pt_median_filter(pt_ctx* ctx, const float* rgba_in, float* rgba_out, int32_t width, int32_t height);
/* The frame CudaRenderer::getImage shows (cu:1539-1569): the median-filtered
 * image while fewer than PT_POST_PROCESS_THRESHOLD samples are accumulated
 * (cudaRenderer.h:70), the accumulated image afterwards.  Whole-frame
 * contexts only (nranks == 1); ranks > 1 filter the gathered frame with
 * pt_median_filter. */
#define PT_POST_PROCESS_THRESHOLD 32
int pt_get_display_image(pt_ctx* ctx, float* rgba, size_t n_floats);
/* Scotty3D HDRImageBuffer::toColor (image.h:168-185): pow(c * sqrt(2^level),
 * 1/gamma) per channel, clamped to [0,1] and scaled to 8 bits as
 * ImageBuffer::update_pixel does (image.h:49-58); alpha 255.  Host function. */
int pt_tonemap(const float* rgba, int32_t width, int32_t height, float gamma, float level, uint8_t* rgba8);
/* Writers for frames in this ABI's layout (bottom-up rows): PNG (8-bit RGBA,
 * stored deflate blocks, written top row first) and PFM (float RGB, whose
 * scanlines run bottom-up like the frame). */
int pt_write_png(const char* path, const uint8_t* rgba8, int32_t width, int32_t height);
int pt_write_pfm(const char* path, const float* rgba, int32_t width, int32_t height);

/* Closest-hit query through the breadth-first traversal.  rays: n records of
 * 8 floats (o.xyz, tmax, d.xyz, tmin): a hit counts when tmin <= t <= tmax,
 * both ends inclusive (Ray::min_t / max_t as Triangle::intersect tests them,
 * triangle.cpp:189; a tmin <= 0 means 0, a NaN tmin is PT_E_INVALID).  hits:
 * n records of (uint64) ((float bits of t) << 32 | sorted prim index), the
 * closest such hit (ties to the lowest index), or PT_HIT_NONE.  Directions may
 * have any length for triangle-only scenes (t is the parametric t); a scene
 * with spheres needs unit directions (|d|^2 within 1e-5 of 1, else
 * PT_E_INVALID) -- scotty::BVHAccel::intersect normalises for its callers. */
#define PT_HIT_NONE 0xFFFFFFFFFFFFFFFFull
int pt_intersect(pt_ctx* ctx, const float* rays, int32_t n, uint64_t* hits);
/* The same with render flags: PT_FLAG_REF_ARITH selects the reference's
 * literal triangle test (cu:217-270); other flags are ignored. */
int pt_intersect_ex(pt_ctx* ctx, const float* rays, int32_t n, uint64_t* hits, uint32_t flags);

typedef struct pt_stats {
  uint64_t rays;      /* R: valid rays entering the root, summed over passes */
  uint64_t visits;    /* V: (ray, node) visits including the root          */
  uint64_t passes;    /* traversal passes                                  */
  uint64_t batches;
  double ms_total;    /* GPU time of the last pt_render / pt_intersect     */
  /* per-kernel GPU time, summed over the renders since pt_reset_stats;
   * collected only when PT_FLAG_STATS is set (HIP events, no host sync)    */
  double ms_trace;    /* root + scan + level kernels                        */
  double ms_shade;    /* camera + shade + accumulate kernels                */
  double ms_root;     /* k_trace_root (+ its ray-count reduction)           */
  double ms_scan;     /* k_scan_level                                       */
  double ms_level[16];       /* k_trace_level per BVH level                 */
  uint64_t level_launches[16];
  uint64_t level_visits[16]; /* V per level (level 0 = R)                   */
  uint64_t level_leaf_visits[16]; /* of which at leaf nodes                 */
  uint64_t level_items[16];  /* work items (<= 1024 rays of one node lane)  */
  uint64_t root_launches;
  uint64_t peak_queue_entries;
  int32_t n_levels;
  int32_t batch_paths;
  double ms_path;     /* k_path_leaf: whole paths of single-leaf scenes     */
  uint64_t path_launches;
  uint64_t shaded;        /* path vertices shaded by k_shade_push             */
  double ms_shade_push;   /* k_shade_push alone (part of ms_shade)            */
  uint64_t shade_launches;
  int32_t queue_factor;   /* current queue factor (grows when a level overflows) */
  int32_t pad_;
  double ms_scan_level[16]; /* k_scan_level per BVH level (part of ms_scan)  */
  uint64_t culled_rays;     /* camera rays of pixels whose whole footprint
                               provably misses the scene's root box: resolved
                               by pt_render's pixel test (radiance 0, no
                               further ray) and counted in `rays` as cast */
  /* PT_FLAG_COUNT_TESTS (single-leaf path kernel): primitive tests executed
   * -- a triangle candidate counts once whether or not its division-free
   * pre-test rejects it -- and cluster box tests (one per cluster per ray) */
  uint64_t prim_tests_tri;
  uint64_t prim_tests_sph;
  uint64_t cluster_box_tests;
} pt_stats;
int pt_get_stats(pt_ctx* ctx, pt_stats* out);
int pt_reset_stats(pt_ctx* ctx);

/* Self-check of the triangle test's division on the device (no reference
 * counterpart): q[i] = num[i] / den[i] as the Baldwin-Weber test computes it
 * (trace.hip div_rn), for n host pairs.  Tests compare it with IEEE
 * division. */
int pt_check_division(pt_ctx* ctx, const float* num, const float* den, float* q, int32_t n);

/* Self-check of the shading code's fast square root and reciprocal (no
 * reference counterpart): every fp32 bit pattern x in [lo, hi) through
 * sqrt_rn (which = 0) or rcp_rn (which = 1; ptmath.h), compared on the device
 * with the IEEE sqrtf(x) / 1.0f / x; *mismatches = how many differ,
 * *first_bad = the smallest such pattern (0xFFFFFFFF: none). */
int pt_check_fast_math(pt_ctx* ctx, int32_t which, uint32_t lo, uint32_t hi, uint64_t* mismatches,
                       uint32_t* first_bad);

#ifdef __cplusplus
}
#define PT_STATIC_ASSERT static_assert
#else
#define PT_STATIC_ASSERT _Static_assert
#endif
/* the record layouts of PT_API_VERSION 2 */
PT_STATIC_ASSERT(sizeof(pt_prim) == 96, "pt_prim layout");
PT_STATIC_ASSERT(sizeof(pt_node) == 128, "pt_node layout");
PT_STATIC_ASSERT(sizeof(pt_bsdf) == 36, "pt_bsdf layout");
PT_STATIC_ASSERT(sizeof(pt_light) == 76, "pt_light layout");
PT_STATIC_ASSERT(sizeof(pt_camera) == 48, "pt_camera layout");
PT_STATIC_ASSERT(sizeof(pt_scene_desc) == 208, "pt_scene_desc layout");
PT_STATIC_ASSERT(sizeof(pt_render_params) == 44, "pt_render_params layout");
PT_STATIC_ASSERT(sizeof(pt_stats) == 944, "pt_stats layout");
#undef PT_STATIC_ASSERT
#endif /* PT_API_H */
