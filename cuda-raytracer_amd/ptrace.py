"""ctypes binding of include/pt_api.h (the C-ABI boundary of the MI355X path tracer).

Python is plumbing here (tests, bench, torch.distributed gather); the product
is libptcore.so: the C++ scene adapter and the gfx950 HIP kernels.  Importing
this module never falls back to anything else: if the library is missing the
import raises.

Reference surface mirrored (src/cudaRenderer.h:173-272):
    CudaRenderer.loadScene(path)   -> Scene.load_dae(path) + Context.load_scene(scene)
    CudaRenderer.render()          -> Context.render(...)
    CudaRenderer.getImage()        -> Context.get_image()
    CudaRenderer.setViewpoint(...) -> Context.set_camera(...)
    CudaRenderer.clearImage()      -> Context.clear()
    BVHAccel::intersect(ray, isect)-> Context.intersect(rays)
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("PTCORE_LIB", HERE / "lib" / "libptcore.so"))

PT_OK = 0
PT_E_INVALID, PT_E_IO, PT_E_NOSCENE, PT_E_HIP, PT_E_OVERFLOW, PT_E_UNSUPPORTED, PT_E_NODEVICE = (
    -1, -2, -3, -4, -5, -6, -7)
PT_HIT_NONE = 0xFFFFFFFFFFFFFFFF
PT_FLAG_COSINE_DIFFUSE = 0x1
PT_FLAG_NO_EMISSION = 0x2
PT_FLAG_STATS = 0x4
PT_FLAG_REF_DROP_ON_MISS = 0x8   # reference quirk (i)
PT_FLAG_REF_GUIDE = 0x10         # reference quirk (ii)
PT_FLAG_REF_SCHEDULE = 0x20      # reference quirk (vi): 2 bounces, NEE 2/2/1 weighted 0.5/0.5/1
PT_FLAG_REF_ARITH = 0x40         # the reference kernels' literal arithmetic (pt_api.h)
PT_FLAG_EXACT_LIGHT_PDF = 0x80   # area-light NEE with the normalised cosine (default: light.cpp:81-92)
PT_FLAG_COUNT_TESTS = 0x100     # count the single-leaf path kernel's executed primitive tests (pt_stats)
PT_FLAG_ASYNC = 0x200           # queue a single-leaf frame and return (pt_sync / the waiting calls report it)
PT_API_VERSION = 6
PT_BSDF_DIFFUSE, PT_BSDF_MIRROR, PT_BSDF_GLASS, PT_BSDF_EMISSION, PT_BSDF_REFRACTION = 0, 1, 2, 3, 4
PT_LIGHT_NONE, PT_LIGHT_AREA, PT_LIGHT_POINT, PT_LIGHT_DIRECTIONAL, PT_LIGHT_HEMISPHERE = 0, 1, 2, 3, 4
PT_PRIM_TRIANGLE, PT_PRIM_SPHERE = 0, 1
PT_GPU_BVH_PLOC, PT_GPU_BVH_LBVH, PT_GPU_BVH_SAH = 0, 1, 2
PT_POST_PROCESS_THRESHOLD = 32


class pt_prim(C.Structure):
    _fields_ = [("q", C.c_float * 24)]


class pt_prim_shading(C.Structure):
    _fields_ = [("n0", C.c_float * 4), ("n1", C.c_float * 4), ("n2", C.c_float * 4)]


class pt_node(C.Structure):
    _fields_ = [("bmin_x", C.c_float * 4), ("bmax_x", C.c_float * 4),
                ("bmin_y", C.c_float * 4), ("bmax_y", C.c_float * 4),
                ("bmin_z", C.c_float * 4), ("bmax_z", C.c_float * 4),
                ("child", C.c_int32 * 4), ("prim_start", C.c_int32), ("prim_count", C.c_int32),
                ("level", C.c_int32), ("ref_id", C.c_int32)]


class pt_bsdf(C.Structure):
    _fields_ = [("type", C.c_int32), ("albedo", C.c_float * 3),
                ("transmittance", C.c_float * 3), ("ior", C.c_float), ("roughness", C.c_float)]


class pt_light(C.Structure):
    _fields_ = [("type", C.c_int32), ("radiance", C.c_float * 3), ("position", C.c_float * 3),
                ("direction", C.c_float * 3), ("dim_x", C.c_float * 3), ("dim_y", C.c_float * 3),
                ("area", C.c_float), ("pad", C.c_float * 2)]


class pt_camera(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("look_at", C.c_float * 3),
                ("left", C.c_float * 3), ("up", C.c_float * 3)]


class pt_scene_desc(C.Structure):
    _fields_ = [("n_prims", C.c_int32), ("prims", C.POINTER(pt_prim)),
                ("shading", C.POINTER(pt_prim_shading)),
                ("n_nodes", C.c_int32), ("nodes", C.POINTER(pt_node)),
                ("n_levels", C.c_int32), ("level_start", C.POINTER(C.c_int32)),
                ("n_bsdfs", C.c_int32), ("bsdfs", C.POINTER(pt_bsdf)),
                ("light", pt_light), ("camera", pt_camera),
                ("n_lights", C.c_int32), ("lights", C.POINTER(pt_light))]


class pt_render_params(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32),
                ("max_bounces", C.c_int32), ("seed", C.c_uint32), ("sample_offset", C.c_int32),
                ("batch_paths", C.c_int32), ("tile_size", C.c_int32), ("rank", C.c_int32),
                ("nranks", C.c_int32), ("flags", C.c_uint32)]


class pt_stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("visits", C.c_uint64), ("passes", C.c_uint64),
                ("batches", C.c_uint64), ("ms_total", C.c_double), ("ms_trace", C.c_double),
                ("ms_shade", C.c_double), ("ms_root", C.c_double), ("ms_scan", C.c_double),
                ("ms_level", C.c_double * 16), ("level_launches", C.c_uint64 * 16),
                ("level_visits", C.c_uint64 * 16), ("level_leaf_visits", C.c_uint64 * 16),
                ("level_items", C.c_uint64 * 16), ("root_launches", C.c_uint64),
                ("peak_queue_entries", C.c_uint64), ("n_levels", C.c_int32), ("batch_paths", C.c_int32),
                ("ms_path", C.c_double), ("path_launches", C.c_uint64),
                ("shaded", C.c_uint64), ("ms_shade_push", C.c_double), ("shade_launches", C.c_uint64),
                ("queue_factor", C.c_int32), ("pad_", C.c_int32),
                ("ms_scan_level", C.c_double * 16), ("culled_rays", C.c_uint64),
                ("prim_tests_tri", C.c_uint64), ("prim_tests_sph", C.c_uint64), ("cluster_box_tests", C.c_uint64)]


class pt_mesh_desc(C.Structure):
    _fields_ = [("n_tris", C.c_int32), ("positions", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
                ("tri_bsdf", C.POINTER(C.c_int32)), ("n_spheres", C.c_int32), ("spheres", C.POINTER(C.c_float)),
                ("sphere_bsdf", C.POINTER(C.c_int32)), ("n_bsdfs", C.c_int32), ("bsdfs", C.POINTER(pt_bsdf)),
                ("light", C.POINTER(pt_light)), ("camera", C.POINTER(pt_camera))]


# every symbol include/pt_api.h declares (tests check the library exports them)
API_SYMBOLS = [
    "pt_api_version", "pt_scene_load_dae", "pt_scene_from_triangles", "pt_scene_from_mesh", "pt_scene_from_mesh_ex", "pt_scene_build_gpu", "pt_scene_build_gpu_ex", "pt_scene_camera_scotty", "pt_scene_free", "pt_scene_get_desc",
    "pt_scene_level_counts", "pt_scene_sorted_to_input", "pt_create", "pt_destroy",
    "pt_last_error", "pt_device_count", "pt_load_scene", "pt_set_camera", "pt_render",
    "pt_clear", "pt_get_image", "pt_get_image_async", "pt_wait_image", "pt_sync", "pt_owned_pixels", "pt_samples", "pt_intersect", "pt_intersect_ex", "pt_copy_owned_sums",
    "pt_get_stats", "pt_reset_stats", "pt_median_filter", "pt_get_display_image", "pt_tonemap",
    "pt_write_png", "pt_write_pfm", "pt_check_division", "pt_check_fast_math",
    "pt_group_create", "pt_group_destroy", "pt_group_last_error", "pt_group_gather_kind", "pt_group_size",
    "pt_group_member", "pt_group_load_scene", "pt_group_set_camera", "pt_group_clear", "pt_group_render",
    "pt_group_get_image", "pt_group_timing",
]


def _load():
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME
    # libamdhip64.so.7, but its libraries NEED the plain file name), so if
    # libptcore.so were loaded first a second runtime would be mapped when
    # torch initialises and the two would fight over the device.  Loading torch
    # first makes libptcore.so bind to the already-loaded runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not LIB_PATH.exists():
        raise ImportError(f"libptcore.so not built ({LIB_PATH}); run __graft_entry__.build()")
    lib = C.CDLL(str(LIB_PATH))
    P, I32, U32, SZ = C.c_void_p, C.c_int32, C.c_uint32, C.c_size_t
    sigs = {
        "pt_api_version": (C.c_int, []),
        "pt_scene_load_dae": (C.c_int, [C.c_char_p, C.POINTER(P), C.c_char_p, SZ]),
        "pt_scene_from_triangles": (C.c_int, [C.POINTER(C.c_float), I32, C.POINTER(pt_bsdf),
                                              C.POINTER(pt_light), C.POINTER(pt_camera), C.POINTER(P)]),
        "pt_scene_from_mesh": (C.c_int, [C.POINTER(pt_mesh_desc), C.POINTER(P)]),
        "pt_scene_from_mesh_ex": (C.c_int, [C.POINTER(pt_mesh_desc), I32, C.POINTER(P)]),
        "pt_scene_build_gpu": (C.c_int, [C.POINTER(pt_mesh_desc), I32, I32, C.POINTER(P), C.POINTER(C.c_double)]),
        "pt_scene_build_gpu_ex": (C.c_int, [C.POINTER(pt_mesh_desc), I32, I32, I32, C.POINTER(P),
                                            C.POINTER(C.c_double)]),
        "pt_scene_camera_scotty": (C.c_int, [P, I32, I32, C.POINTER(pt_camera)]),
        "pt_scene_free": (None, [P]),
        "pt_median_filter": (C.c_int, [P, C.POINTER(C.c_float), C.POINTER(C.c_float), I32, I32]),
        "pt_get_display_image": (C.c_int, [P, C.POINTER(C.c_float), SZ]),
        "pt_tonemap": (C.c_int, [C.POINTER(C.c_float), I32, I32, C.c_float, C.c_float, C.POINTER(C.c_uint8)]),
        "pt_write_png": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint8), I32, I32]),
        "pt_write_pfm": (C.c_int, [C.c_char_p, C.POINTER(C.c_float), I32, I32]),
        "pt_scene_get_desc": (C.c_int, [P, C.POINTER(pt_scene_desc)]),
        "pt_scene_level_counts": (C.c_int, [P, C.POINTER(I32), I32, C.POINTER(I32)]),
        "pt_scene_sorted_to_input": (C.c_int, [P, C.POINTER(I32), I32]),
        "pt_create": (C.c_int, [C.POINTER(P), C.c_int]),
        "pt_destroy": (None, [P]),
        "pt_last_error": (C.c_char_p, [P]),
        "pt_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "pt_load_scene": (C.c_int, [P, C.POINTER(pt_scene_desc)]),
        "pt_set_camera": (C.c_int, [P, C.POINTER(pt_camera)]),
        "pt_render": (C.c_int, [P, C.POINTER(pt_render_params)]),
        "pt_clear": (C.c_int, [P]),
        "pt_get_image": (C.c_int, [P, C.POINTER(C.c_float), SZ]),
        "pt_get_image_async": (C.c_int, [P, C.POINTER(C.c_float), SZ]),
        "pt_wait_image": (C.c_int, [P]),
        "pt_sync": (C.c_int, [P]),
        "pt_owned_pixels": (C.c_int, [P, C.POINTER(I32), C.POINTER(I32), SZ, C.POINTER(P)]),
        "pt_samples": (C.c_int, [P, C.POINTER(I32)]),
        "pt_copy_owned_sums": (C.c_int, [P, P, SZ, I32]),
        "pt_intersect": (C.c_int, [P, C.POINTER(C.c_float), I32, C.POINTER(C.c_uint64)]),
        "pt_intersect_ex": (C.c_int, [P, C.POINTER(C.c_float), I32, C.POINTER(C.c_uint64), U32]),
        "pt_get_stats": (C.c_int, [P, C.POINTER(pt_stats)]),
        "pt_reset_stats": (C.c_int, [P]),
        "pt_check_division": (C.c_int, [P, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float), I32]),
        "pt_check_fast_math": (C.c_int, [P, I32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]),
        "pt_group_create": (C.c_int, [C.POINTER(P), C.POINTER(I32), I32, I32]),
        "pt_group_destroy": (None, [P]),
        "pt_group_last_error": (C.c_char_p, [P]),
        "pt_group_gather_kind": (C.c_int, [P, C.POINTER(I32)]),
        "pt_group_size": (C.c_int, [P, C.POINTER(I32)]),
        "pt_group_member": (P, [P, I32]),
        "pt_group_load_scene": (C.c_int, [P, C.POINTER(pt_scene_desc)]),
        "pt_group_set_camera": (C.c_int, [P, C.POINTER(pt_camera)]),
        "pt_group_clear": (C.c_int, [P]),
        "pt_group_render": (C.c_int, [P, C.POINTER(pt_render_params)]),
        "pt_group_get_image": (C.c_int, [P, C.POINTER(C.c_float), SZ]),
        "pt_group_timing": (C.c_int, [P, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.pt_api_version() != PT_API_VERSION:
        raise ImportError(f"libptcore.so has API version {lib.pt_api_version()}, this binding {PT_API_VERSION}")
    return lib


LIB = _load()


class PTError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"pt error {code}: {msg}")
        self.code = code


def _ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


class Scene:
    """Host-side scene: COLLADA subset -> reference BVH -> flattened arrays."""

    def __init__(self, handle):
        self.h = C.c_void_p(handle) if not isinstance(handle, C.c_void_p) else handle

    @classmethod
    def load_dae(cls, path):
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = LIB.pt_scene_load_dae(str(path).encode(), C.byref(h), err, 512)
        if rc != PT_OK:
            raise PTError(rc, err.value.decode())
        return cls(h)

    @classmethod
    def from_triangles(cls, tris, bsdf=None, light=None, camera=None):
        tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
        h = C.c_void_p()
        rc = LIB.pt_scene_from_triangles(_ptr(tris, C.c_float), len(tris),
                                         C.byref(bsdf) if bsdf else None,
                                         C.byref(light) if light else None,
                                         C.byref(camera) if camera else None, C.byref(h))
        if rc != PT_OK:
            raise PTError(rc, "pt_scene_from_triangles failed")
        return cls(h)

    @classmethod
    def from_mesh(cls, positions, bsdfs, normals=None, tri_bsdf=None, spheres=None, sphere_bsdf=None,
                  light=None, camera=None, gpu_device=None, max_leaf=32, builder="sah"):
        """General flattened input (pt_scene_from_mesh): triangles (n, 9),
        optional vertex normals (n, 9), per-triangle bsdf ids, spheres (m, 4)
        and a list of pt_bsdf.  gpu_device=k builds the BVH on GPU k
        (pt_scene_build_gpu_ex, wide leaves of <= max_leaf primitives;
        builder "ploc" or "lbvh")."""
        keep = []

        def arr(a, dt, k):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=dt).reshape(-1, k) if k else np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a

        pos = arr(positions, np.float32, 9)
        nrm = arr(normals, np.float32, 9)
        tb = arr(tri_bsdf, np.int32, 0)
        sph = arr(spheres, np.float32, 4)
        sb = arr(sphere_bsdf, np.int32, 0)
        bt = (pt_bsdf * len(bsdfs))(*bsdfs)
        m = pt_mesh_desc()
        m.n_tris = 0 if pos is None else len(pos)
        m.positions = _ptr(pos, C.c_float) if pos is not None else None
        m.normals = _ptr(nrm, C.c_float) if nrm is not None else None
        m.tri_bsdf = _ptr(tb, C.c_int32) if tb is not None else None
        m.n_spheres = 0 if sph is None else len(sph)
        m.spheres = _ptr(sph, C.c_float) if sph is not None else None
        m.sphere_bsdf = _ptr(sb, C.c_int32) if sb is not None else None
        m.n_bsdfs = len(bsdfs)
        m.bsdfs = C.cast(bt, C.POINTER(pt_bsdf))
        m.light = C.pointer(light) if light is not None else None
        m.camera = C.pointer(camera) if camera is not None else None
        h = C.c_void_p()
        if gpu_device is None:
            rc = LIB.pt_scene_from_mesh(C.byref(m), C.byref(h))
        else:
            ms = C.c_double()
            b = {"ploc": PT_GPU_BVH_PLOC, "lbvh": PT_GPU_BVH_LBVH, "sah": PT_GPU_BVH_SAH}[builder]
            rc = LIB.pt_scene_build_gpu_ex(C.byref(m), gpu_device, max_leaf, b, C.byref(h), C.byref(ms))
        if rc != PT_OK:
            raise PTError(rc, "pt_scene_from_mesh failed" if gpu_device is None else "pt_scene_build_gpu failed")
        sc = cls(h)
        if gpu_device is not None:
            sc.build_ms = ms.value
        return sc

    def __del__(self):
        # LIB is None once the interpreter tears the module down
        if getattr(self, "h", None) and self.h.value and LIB is not None:
            LIB.pt_scene_free(self.h)
            self.h = C.c_void_p()

    def desc(self) -> pt_scene_desc:
        d = pt_scene_desc()
        rc = LIB.pt_scene_get_desc(self.h, C.byref(d))
        if rc != PT_OK:
            raise PTError(rc, "pt_scene_get_desc")
        d._owner = self  # the desc borrows the scene's arrays
        return d

    def camera_scotty(self, width, height):
        """The Scotty3D framing of the COLLADA camera (pt_scene_camera_scotty)."""
        cam = pt_camera()
        rc = LIB.pt_scene_camera_scotty(self.h, width, height, C.byref(cam))
        if rc != PT_OK:
            raise PTError(rc, "pt_scene_camera_scotty")
        return cam

    def level_counts(self):
        counts = (C.c_int32 * 256)()
        n = C.c_int32()
        LIB.pt_scene_level_counts(self.h, counts, 256, C.byref(n))
        return [counts[i] for i in range(n.value)]

    def sorted_to_input(self):
        d = self.desc()
        out = np.zeros(d.n_prims, dtype=np.int32)
        LIB.pt_scene_sorted_to_input(self.h, _ptr(out, C.c_int32), d.n_prims)
        return out

    # numpy views (copies) of the flattened arrays
    def prims(self):
        d = self.desc()
        return np.ctypeslib.as_array(C.cast(d.prims, C.POINTER(C.c_float)), shape=(d.n_prims, 24)).copy()

    def nodes(self):
        d = self.desc()
        return [d.nodes[i] for i in range(d.n_nodes)]


def scene_to_arrays(scene: "Scene") -> dict:
    """The flattened pt_scene_desc of a Scene as plain numpy arrays."""
    d = scene.desc()
    f32 = lambda p, n, k: np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), shape=(n, k)).copy()
    nodes = np.frombuffer(C.string_at(d.nodes, C.sizeof(pt_node) * d.n_nodes), dtype=np.uint8).copy()
    bsdfs = np.frombuffer(C.string_at(d.bsdfs, C.sizeof(pt_bsdf) * d.n_bsdfs), dtype=np.uint8).copy()
    return {
        "prims": f32(d.prims, d.n_prims, 24),
        "shading": f32(d.shading, d.n_prims, 12),
        "nodes": nodes,
        "level_start": np.ctypeslib.as_array(d.level_start, shape=(d.n_levels + 1,)).copy(),
        "bsdfs": bsdfs,
        "bsdf_size": np.array([C.sizeof(pt_bsdf)], np.int32),
        "light": np.frombuffer(bytes(d.light), dtype=np.uint8).copy(),
        "camera": np.frombuffer(bytes(d.camera), dtype=np.uint8).copy(),
        # every light when there are several (pt_scene_desc.lights), else empty
        "lights": np.frombuffer(C.string_at(d.lights, C.sizeof(pt_light) * d.n_lights), dtype=np.uint8).copy()
        if d.n_lights > 1 else np.zeros(0, np.uint8),
    }


BSDF_V1_SIZE = 32  # pt_bsdf before its roughness field (rounds 1-3 fixtures)


def _upgrade_bsdfs(a: dict) -> dict:
    """Fixtures written before pt_bsdf grew `roughness` hold 32-byte records
    (no "bsdf_size" key): append roughness 0 -- every <roughness> in the
    reference's media is 0."""
    size = int(np.asarray(a["bsdf_size"]).reshape(-1)[0]) if "bsdf_size" in a else BSDF_V1_SIZE
    if size == C.sizeof(pt_bsdf):
        return a
    old = a["bsdfs"].reshape(-1, size)
    new = np.zeros((len(old), C.sizeof(pt_bsdf)), np.uint8)
    new[:, :size] = old
    a = dict(a)
    a["bsdfs"] = new.reshape(-1)
    a["bsdf_size"] = np.array([C.sizeof(pt_bsdf)], np.int32)
    return a


class ArrayScene:
    """A flattened scene held in numpy arrays (fixtures, synthetic scenes).
    Exposes the same desc() as Scene, so Context.load_scene accepts it."""

    def __init__(self, arrays: dict):
        self.a = {k: np.ascontiguousarray(v) for k, v in arrays.items()}

    @classmethod
    def load(cls, path):
        with np.load(path, allow_pickle=False) as z:
            a = {k: z[k] for k in z.files}
        return cls(_upgrade_bsdfs(a))

    def desc(self) -> pt_scene_desc:
        a = self.a
        d = pt_scene_desc()
        d.n_prims = len(a["prims"])
        d.prims = a["prims"].ctypes.data_as(C.POINTER(pt_prim))
        d.shading = a["shading"].ctypes.data_as(C.POINTER(pt_prim_shading))
        d.n_nodes = len(a["nodes"]) // C.sizeof(pt_node)
        d.nodes = a["nodes"].ctypes.data_as(C.POINTER(pt_node))
        ls = a["level_start"].astype(np.int32)
        self.a["level_start"] = ls
        d.n_levels = len(ls) - 1
        d.level_start = ls.ctypes.data_as(C.POINTER(C.c_int32))
        d.n_bsdfs = len(a["bsdfs"]) // C.sizeof(pt_bsdf)
        d.bsdfs = a["bsdfs"].ctypes.data_as(C.POINTER(pt_bsdf))
        d.light = pt_light.from_buffer_copy(a["light"].tobytes())
        d.camera = pt_camera.from_buffer_copy(a["camera"].tobytes())
        lights = a.get("lights")
        if lights is not None and len(lights) >= 2 * C.sizeof(pt_light):
            d.n_lights = len(lights) // C.sizeof(pt_light)
            d.lights = lights.ctypes.data_as(C.POINTER(pt_light))
        d._owner = self  # the desc points into our arrays: keep them alive
        return d

    def level_counts(self):
        return [int(x) for x in self.a.get("level_counts", [])]

    def nodes(self):
        d = self.desc()
        return [d.nodes[i] for i in range(d.n_nodes)]


class Context:
    """One device context (one GPU).  Mirrors cutracer::CudaRenderer."""

    def __init__(self, device=0):
        self.h = C.c_void_p()
        rc = LIB.pt_create(C.byref(self.h), device)
        if rc != PT_OK:
            raise PTError(rc, "pt_create failed (no GPU visible?)")
        self.width = self.height = 0

    def close(self):
        if getattr(self, "h", None) and self.h.value and LIB is not None:
            LIB.pt_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        self.close()

    def _chk(self, rc):
        if rc != PT_OK:
            raise PTError(rc, LIB.pt_last_error(self.h).decode(errors="replace"))

    def check_division(self, num, den):
        """num / den as the device's triangle test divides (pt_check_division)."""
        num = np.ascontiguousarray(num, dtype=np.float32)
        den = np.ascontiguousarray(den, dtype=np.float32)
        q = np.empty_like(num)
        self._chk(LIB.pt_check_division(self.h, _ptr(num, C.c_float), _ptr(den, C.c_float), _ptr(q, C.c_float),
                                        len(num)))
        return q

    def check_fast_math(self, which, lo, hi):
        """(mismatches, first mismatching bit pattern or None) of sqrt_rn
        (which 0) or rcp_rn (which 1) against IEEE over the fp32 bit patterns
        [lo, hi), on the device (pt_check_fast_math)."""
        n, first = C.c_uint64(0), C.c_uint32(0)
        self._chk(LIB.pt_check_fast_math(self.h, int(which), int(lo), int(hi), C.byref(n), C.byref(first)))
        return n.value, (None if first.value == 0xFFFFFFFF else first.value)

    def load_scene(self, scene: Scene):
        self._desc = scene.desc()
        self._scene = scene  # keep arrays alive while the context uses them
        self._chk(LIB.pt_load_scene(self.h, C.byref(self._desc)))

    def set_camera(self, cam: pt_camera):
        self._chk(LIB.pt_set_camera(self.h, C.byref(cam)))

    def render(self, width, height, spp, max_bounces=8, seed=15618, sample_offset=0,
               batch_paths=0, tile_size=32, rank=0, nranks=1, flags=0):
        p = pt_render_params(width, height, spp, max_bounces, seed, sample_offset, batch_paths,
                             tile_size, rank, nranks, flags)
        self.width, self.height = width, height
        self._chk(LIB.pt_render(self.h, C.byref(p)))

    def clear(self):
        self._chk(LIB.pt_clear(self.h))

    def samples(self):
        n = C.c_int32()
        self._chk(LIB.pt_samples(self.h, C.byref(n)))
        return n.value

    def get_image_async(self, out):
        """Queue the frame's copy into `out` (a host buffer: numpy array or
        torch CPU tensor, ideally pinned) and return at once; the next clear /
        render overlaps the copy.  `out` holds the frame after wait_image."""
        if isinstance(out, np.ndarray):
            assert out.dtype == np.float32 and out.flags.c_contiguous
            self._chk(LIB.pt_get_image_async(self.h, _ptr(out, C.c_float), out.size))
        else:  # torch tensor
            assert out.dtype.is_floating_point and out.is_contiguous() and out.device.type == "cpu"
            self._chk(LIB.pt_get_image_async(self.h, C.cast(out.data_ptr(), C.POINTER(C.c_float)), out.numel()))
        return out

    def wait_image(self):
        self._chk(LIB.pt_wait_image(self.h))

    def sync(self):
        """Wait for the frames queued with PT_FLAG_ASYNC (raises their failure)."""
        self._chk(LIB.pt_sync(self.h))

    def get_image(self, out=None):
        """The accumulated frame (H, W, 4) float32 on the host.  `out`: an
        optional preallocated host buffer (numpy array or torch CPU tensor,
        ideally pinned: the copy then runs at full PCIe rate)."""
        if out is None:
            img = np.zeros((self.height, self.width, 4), dtype=np.float32)
            self._chk(LIB.pt_get_image(self.h, _ptr(img, C.c_float), img.size))
            return img
        if isinstance(out, np.ndarray):
            assert out.dtype == np.float32 and out.flags.c_contiguous
            self._chk(LIB.pt_get_image(self.h, _ptr(out, C.c_float), out.size))
        else:  # torch tensor
            assert out.dtype.is_floating_point and out.is_contiguous() and out.device.type == "cpu"
            self._chk(LIB.pt_get_image(self.h, C.cast(out.data_ptr(), C.POINTER(C.c_float)), out.numel()))
        return out

    def copy_owned_sums(self, dst_ptr, nbytes, on_device=True):
        """pt_copy_owned_sums: the owned pixels' float4 sums into dst_ptr."""
        self._chk(LIB.pt_copy_owned_sums(self.h, C.c_void_p(dst_ptr), nbytes, 1 if on_device else 0))

    def get_display_image(self):
        """What CudaRenderer::getImage shows: median-filtered below 32 spp."""
        img = np.zeros((self.height, self.width, 4), dtype=np.float32)
        self._chk(LIB.pt_get_display_image(self.h, _ptr(img, C.c_float), img.size))
        return img

    def median_filter(self, img):
        """3x3 reference median filter of an (H, W, 4) float32 frame, on the GPU."""
        img = np.ascontiguousarray(img, dtype=np.float32)
        out = np.empty_like(img)
        self._chk(LIB.pt_median_filter(self.h, _ptr(img, C.c_float), _ptr(out, C.c_float), img.shape[1],
                                       img.shape[0]))
        return out

    def owned_count(self):
        """Pixels this context renders (its tile share of the last render)."""
        n = C.c_int32()
        self._chk(LIB.pt_owned_pixels(self.h, C.byref(n), None, 0, None))
        return n.value

    def owned_pixels(self):
        n = C.c_int32()
        self._chk(LIB.pt_owned_pixels(self.h, C.byref(n), None, 0, None))
        idx = np.zeros(max(1, n.value), dtype=np.int32)
        dptr = C.c_void_p()
        self._chk(LIB.pt_owned_pixels(self.h, C.byref(n), _ptr(idx, C.c_int32), idx.size, C.byref(dptr)))
        return idx[: n.value], dptr.value

    def intersect(self, rays, flags=0):
        """rays: (n, 8) float32 [o.xyz, tmax, d.xyz, tmin] -> uint64 hit keys
        (the closest hit with tmin <= t <= tmax).
        flags: PT_FLAG_REF_ARITH selects the reference's literal triangle test."""
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        hits = np.zeros(len(rays), dtype=np.uint64)
        if flags:
            self._chk(LIB.pt_intersect_ex(self.h, _ptr(rays, C.c_float), len(rays), _ptr(hits, C.c_uint64), flags))
        else:
            self._chk(LIB.pt_intersect(self.h, _ptr(rays, C.c_float), len(rays), _ptr(hits, C.c_uint64)))
        return hits

    def stats(self) -> pt_stats:
        s = pt_stats()
        self._chk(LIB.pt_get_stats(self.h, C.byref(s)))
        return s

    def reset_stats(self):
        self._chk(LIB.pt_reset_stats(self.h))


PT_GATHER_AUTO, PT_GATHER_RCCL, PT_GATHER_HOST = 0, 1, 2


class Group:
    """Several GPUs of one process rendering one frame (pt_group_*): member i
    renders tiles t % n == i on its own host thread; the sums are gathered to
    member 0 over RCCL (distinct devices) or through the host."""

    def __init__(self, devices, gather=PT_GATHER_AUTO):
        devs = (C.c_int32 * len(devices))(*devices)
        self.h = C.c_void_p()
        rc = LIB.pt_group_create(C.byref(self.h), devs, len(devices), gather)
        if rc != PT_OK:
            raise PTError(rc, f"pt_group_create({list(devices)}, gather={gather})")
        self.width = self.height = 0

    def close(self):
        if getattr(self, "h", None) and self.h.value and LIB is not None:
            LIB.pt_group_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        self.close()

    def _chk(self, rc):
        if rc != PT_OK:
            raise PTError(rc, LIB.pt_group_last_error(self.h).decode(errors="replace"))

    @property
    def gather_kind(self):
        k = C.c_int32()
        self._chk(LIB.pt_group_gather_kind(self.h, C.byref(k)))
        return k.value

    @property
    def note(self):
        return LIB.pt_group_last_error(self.h).decode(errors="replace")

    def load_scene(self, scene):
        self._desc = scene.desc()
        self._scene = scene
        self._chk(LIB.pt_group_load_scene(self.h, C.byref(self._desc)))

    def set_camera(self, cam):
        self._chk(LIB.pt_group_set_camera(self.h, C.byref(cam)))

    def clear(self):
        self._chk(LIB.pt_group_clear(self.h))

    def render(self, width, height, spp, max_bounces=8, seed=15618, sample_offset=0, batch_paths=0, tile_size=32,
               flags=0):
        p = pt_render_params(width, height, spp, max_bounces, seed, sample_offset, batch_paths, tile_size, 0, 1, flags)
        self.width, self.height = width, height
        self._chk(LIB.pt_group_render(self.h, C.byref(p)))

    def get_image(self):
        img = np.zeros((self.height, self.width, 4), dtype=np.float32)
        self._chk(LIB.pt_group_get_image(self.h, _ptr(img, C.c_float), img.size))
        return img

    def timing(self):
        g, r = C.c_double(), C.c_double()
        self._chk(LIB.pt_group_timing(self.h, C.byref(g), C.byref(r)))
        return g.value, r.value


def device_count():
    n = C.c_int()
    LIB.pt_device_count(C.byref(n))
    return n.value


def hit_t(keys):
    """fp32 t of uint64 hit keys (inf for misses)."""
    keys = np.asarray(keys, dtype=np.uint64)
    t = (keys >> np.uint64(32)).astype(np.uint32).view(np.float32).copy()
    t[keys == np.uint64(PT_HIT_NONE)] = np.inf
    return t


def hit_prim(keys):
    keys = np.asarray(keys, dtype=np.uint64)
    p = (keys & np.uint64(0xFFFFFFFF)).astype(np.int64)
    p[keys == np.uint64(PT_HIT_NONE)] = -1
    return p


def tonemap(img, gamma=2.2, level=1.0):
    """Scotty3D toColor (image.h:168-185): (H, W, 4) float32 -> (H, W, 4) uint8."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    out = np.zeros(img.shape, dtype=np.uint8)
    rc = LIB.pt_tonemap(_ptr(img, C.c_float), img.shape[1], img.shape[0], gamma, level, _ptr(out, C.c_uint8))
    if rc != PT_OK:
        raise PTError(rc, "pt_tonemap")
    return out


def write_png(path, rgba8):
    rgba8 = np.ascontiguousarray(rgba8, dtype=np.uint8)
    rc = LIB.pt_write_png(str(path).encode(), _ptr(rgba8, C.c_uint8), rgba8.shape[1], rgba8.shape[0])
    if rc != PT_OK:
        raise PTError(rc, f"pt_write_png {path}")


def write_pfm(path, img):
    img = np.ascontiguousarray(img, dtype=np.float32)
    rc = LIB.pt_write_pfm(str(path).encode(), _ptr(img, C.c_float), img.shape[1], img.shape[0])
    if rc != PT_OK:
        raise PTError(rc, f"pt_write_pfm {path}")


# ---- the Scotty3D surface on the GPU (scotty/scotty_capi.cpp) ----------------
SCOTTY_LIB_PATH = LIB_PATH.parent / "libscotty_gpu.so"
_SCOTTY = None


def _scotty():
    global _SCOTTY
    if _SCOTTY is None:
        if not SCOTTY_LIB_PATH.exists():
            raise ImportError(f"libscotty_gpu.so not built ({SCOTTY_LIB_PATH}); run __graft_entry__.build()")
        lib = C.CDLL(str(SCOTTY_LIB_PATH))
        P, I32, U32, SZ, F = C.c_void_p, C.c_int32, C.c_uint32, C.c_size_t, C.POINTER(C.c_float)
        lib.scotty_render.restype = C.c_int
        lib.scotty_render.argtypes = [C.POINTER(pt_scene_desc), I32, I32, I32, I32, U32, I32, I32, F, C.c_char_p, SZ]
        lib.scotty_render_multi.restype = C.c_int
        lib.scotty_render_multi.argtypes = [C.POINTER(pt_scene_desc), I32, I32, I32, I32, U32, I32, C.POINTER(I32), I32,
                                            I32, F, C.POINTER(I32), C.POINTER(C.c_double), C.c_char_p, SZ]
        lib.scotty_viewer.restype = C.c_int
        lib.scotty_viewer.argtypes = [C.POINTER(pt_scene_desc), I32, I32, I32, I32, U32, C.c_char_p, I32, F,
                                      C.POINTER(I32), C.c_char_p, SZ]
        D = C.POINTER(C.c_double)
        lib.scotty_generate_rays.restype = C.c_int
        lib.scotty_generate_rays.argtypes = [C.POINTER(pt_camera), I32, D, D]
        lib.scotty_camera_place.restype = C.c_int
        lib.scotty_camera_place.argtypes = [D, I32, I32, D, C.c_double, C.c_double, C.c_double, C.c_double,
                                            C.c_double, C.POINTER(pt_camera), I32, D, D, D]
        lib.scotty_bvh_create.restype = C.c_int
        lib.scotty_bvh_create.argtypes = [D, D, I32, C.POINTER(I32), I32, D, I32, I32, I32, C.POINTER(P),
                                          C.c_char_p, SZ]
        lib.scotty_bvh_intersect.restype = C.c_int
        lib.scotty_bvh_intersect.argtypes = [P, D, I32, I32, C.POINTER(I32), D, C.POINTER(I32), D]
        lib.scotty_bvh_occluded.restype = C.c_int
        lib.scotty_bvh_occluded.argtypes = [P, D, I32, C.POINTER(I32)]
        lib.scotty_bvh_destroy.restype = None
        lib.scotty_bvh_destroy.argtypes = [P]
        _SCOTTY = lib
    return _SCOTTY


def scotty_render(scene, width, height, spp, max_depth, flags=0, threads=0, device=0):
    """CMU462::PathTracer on the GPU: start_raytracing's 32x32 tile queue and
    `threads` workers (0 = hardware_concurrency) over one pt_render; the
    (H, W, 4) frame."""
    out = np.zeros((height, width, 4), dtype=np.float32)
    err = C.create_string_buffer(512)
    d = scene.desc()
    rc = _scotty().scotty_render(C.byref(d), width, height, spp, max_depth, flags, threads, device,
                                 _ptr(out, C.c_float), err, len(err))
    if rc:
        raise PTError(rc, err.value.decode(errors="replace"))
    return out


def scotty_render_multi(scene, width, height, spp, max_depth, devices, gather=0, flags=0, threads=0):
    """scotty::MultiGpuPathTracer: the same tile/worker loop over a pt_group
    of `devices` (one process).  Returns (frame, gather kind, gather ms)."""
    out = np.zeros((height, width, 4), dtype=np.float32)
    err = C.create_string_buffer(512)
    d = scene.desc()
    devs = (C.c_int32 * len(devices))(*devices)
    kind, gms = C.c_int32(), C.c_double()
    rc = _scotty().scotty_render_multi(C.byref(d), width, height, spp, max_depth, flags, threads, devs, len(devices),
                                       gather, _ptr(out, C.c_float), C.byref(kind), C.byref(gms), err, len(err))
    if rc:
        raise PTError(rc, err.value.decode(errors="replace"))
    return out, kind.value, gms.value


def scotty_viewer(scene, width, height, samples_per_frame, keys, max_bounces=2, flags=0, device=0):
    """The display.cpp viewer loop, headless: one renderPicture per character
    of `keys` after handleKeyPress(c) ('.' = no key).  Returns (the last
    displayed frame, samples accumulated in it)."""
    out = np.zeros((height, width, 4), dtype=np.float32)
    err = C.create_string_buffer(512)
    n = C.c_int32()
    d = scene.desc()
    rc = _scotty().scotty_viewer(C.byref(d), width, height, samples_per_frame, max_bounces, flags,
                                 keys.encode(), device, _ptr(out, C.c_float), C.byref(n), err, len(err))
    if rc:
        raise PTError(rc, err.value.decode(errors="replace"))
    return out, n.value


def _d(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def scotty_generate_rays(cam, xy):
    """CMU462::Camera::generate_ray (scotty::Camera over a pt_camera) for
    normalised sensor points xy (n, 2): (n, 6) float64 = origin, unit direction."""
    xy = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 2)
    out = np.zeros((len(xy), 6), dtype=np.float64)
    rc = _scotty().scotty_generate_rays(C.byref(cam), len(xy), _d(xy), _d(out))
    if rc:
        raise PTError(rc, "scotty_generate_rays")
    return out


def scotty_camera_place(hfov, vfov, width, height, target, phi, theta, r, min_r=0.0, max_r=np.inf,
                        xy=None, nclip=0.01, fclip=100.0):
    """Camera::configure + place (the Scotty3D framing): returns (pt_camera,
    rays (n, 6) for the sensor points xy, (hFov, vFov) fitted to the screen)."""
    info = np.array([hfov, vfov, nclip, fclip], dtype=np.float64)
    tgt = np.ascontiguousarray(target, dtype=np.float64)
    xy = np.zeros((0, 2)) if xy is None else np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 2)
    rays = np.zeros((len(xy), 6), dtype=np.float64)
    fov = np.zeros(2, dtype=np.float64)
    cam = pt_camera()
    rc = _scotty().scotty_camera_place(_d(info), width, height, _d(tgt), phi, theta, r, min_r, max_r,
                                       C.byref(cam), len(xy), _d(xy) if len(xy) else None,
                                       _d(rays) if len(xy) else None, _d(fov))
    if rc:
        raise PTError(rc, "scotty_camera_place")
    return cam, rays, (float(fov[0]), float(fov[1]))


class ScottyBVH:
    """StaticScene::BVHAccel(primitives, max_leaf_size) on the GPU over Scotty3D
    primitives (scotty_bvh_create): one Mesh's triangles (positions (v, 3),
    vertex normals (v, 3), indices (t, 3)) then spheres (s, 4)."""

    def __init__(self, positions, normals, indices, spheres=None, max_leaf=32, device=0):
        pos = np.ascontiguousarray(positions, dtype=np.float64).reshape(-1, 3)
        nrm = np.ascontiguousarray(normals, dtype=np.float64).reshape(-1, 3)
        idx = np.ascontiguousarray(indices, dtype=np.int32).reshape(-1, 3)
        sph = np.zeros((0, 4)) if spheres is None else np.ascontiguousarray(spheres, dtype=np.float64).reshape(-1, 4)
        self.h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = _scotty().scotty_bvh_create(_d(pos), _d(nrm), len(pos), idx.ctypes.data_as(C.POINTER(C.c_int32)),
                                         len(idx), _d(sph) if len(sph) else None, len(sph), max_leaf, device,
                                         C.byref(self.h), err, len(err))
        if rc:
            raise PTError(rc, err.value.decode(errors="replace"))

    def intersect(self, rays, single=False):
        """rays (n, 8) float64 = o, d, min_t, max_t -> (hit bool, t, prim index, normal (n, 3))."""
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 8)
        n = len(rays)
        hit = np.zeros(n, dtype=np.int32)
        t = np.zeros(n, dtype=np.float64)
        prim = np.zeros(n, dtype=np.int32)
        nrm = np.zeros((n, 3), dtype=np.float64)
        rc = _scotty().scotty_bvh_intersect(self.h, _d(rays), n, 1 if single else 0,
                                            hit.ctypes.data_as(C.POINTER(C.c_int32)), _d(t),
                                            prim.ctypes.data_as(C.POINTER(C.c_int32)), _d(nrm))
        if rc:
            raise PTError(rc, "scotty_bvh_intersect")
        return hit.astype(bool), t, prim, nrm

    def occluded(self, rays):
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 8)
        hit = np.zeros(len(rays), dtype=np.int32)
        rc = _scotty().scotty_bvh_occluded(self.h, _d(rays), len(rays), hit.ctypes.data_as(C.POINTER(C.c_int32)))
        if rc:
            raise PTError(rc, "scotty_bvh_occluded")
        return hit.astype(bool)

    def close(self):
        if getattr(self, "h", None) and self.h.value and _SCOTTY is not None:
            _SCOTTY.scotty_bvh_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        self.close()
