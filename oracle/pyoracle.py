"""ctypes binding of the CPU oracle (oracle/ptoracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "libptoracle.so"


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def _load():
    if not LIB_PATH.exists():
        build()
    lib = C.CDLL(str(LIB_PATH))
    P = C.c_void_p
    lib.pto_closest_brute.restype = C.c_uint64
    lib.pto_closest_brute.argtypes = [P, C.POINTER(C.c_float)]
    lib.pto_closest_bvh.restype = C.c_uint64
    lib.pto_closest_bvh.argtypes = [P, C.POINTER(C.c_float)]
    lib.pto_intersect.restype = None
    lib.pto_intersect.argtypes = [P, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_uint64), C.c_int]
    lib.pto_intersect_ex.restype = None
    lib.pto_intersect_ex.argtypes = [P, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_uint64), C.c_int, C.c_uint32]
    lib.pto_bfs_visits.restype = None
    lib.pto_bfs_visits.argtypes = [P, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_uint64), C.c_int]
    lib.pto_render.restype = C.c_uint64
    lib.pto_render.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_int, C.c_uint32,
                               C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
    lib.pto_median.restype = None
    lib.pto_median.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int, C.c_int]
    lib.pto_sample.restype = None
    lib.pto_sample.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32,
                               C.c_uint32, C.POINTER(C.c_float)]
    lib.pto_philox.restype = None
    lib.pto_philox.argtypes = [C.c_uint32] * 6 + [C.POINTER(C.c_uint32)]
    lib.pto_camera_ray.restype = None
    lib.pto_camera_ray.argtypes = [P, C.c_int, C.c_int, C.c_float, C.c_float, C.c_uint32, C.POINTER(C.c_float)]
    lib.pto_sincos2pi.restype = None
    lib.pto_sincos2pi.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    return lib


LIB = _load()


def _load_scotty():
    lib = C.CDLL(str(HERE / "build" / "libptscotty.so"))
    lib.pto_scotty_render.restype = C.c_uint64
    lib.pto_scotty_render.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_uint32,
                                      C.c_int, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_double),
                                      C.POINTER(C.c_int)]
    return lib


SCOTTY = _load_scotty()


def scotty_render(desc, width, height, spp, max_bounces=8, seed=15618, flags=0, threads=0, tile_stride=1):
    """The oracle through the Scotty3D PathTracer surface (oracle/scotty_cpu.cpp:
    32x32-tile work queue, `threads` workers, 0 = hardware_concurrency).
    Returns (image (H, W, 4) = sum / spp like pt_get_image, rays, seconds,
    threads used).  tile_stride > 1 renders only tiles t % tile_stride == 0."""
    img = np.zeros((height, width, 4), dtype=np.float32)
    sec, thr = C.c_double(), C.c_int()
    rays = SCOTTY.pto_scotty_render(C.addressof(desc), width, height, spp, max_bounces, seed, flags, threads,
                                    tile_stride, _f(img), C.byref(sec), C.byref(thr))
    return img, int(rays), sec.value, thr.value


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def intersect(desc, rays, use_bvh=True, flags=0):
    """Closest-hit keys; flags & PT_FLAG_REF_ARITH: the literal cu:217-270 test."""
    rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
    hits = np.zeros(len(rays), dtype=np.uint64)
    LIB.pto_intersect_ex(C.addressof(desc), _f(rays), len(rays),
                         hits.ctypes.data_as(C.POINTER(C.c_uint64)), 1 if use_bvh else 0, flags)
    return hits


def bfs_visits(desc, rays, max_levels=16):
    rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
    lv = np.zeros(max_levels, dtype=np.uint64)
    LIB.pto_bfs_visits(C.addressof(desc), _f(rays), len(rays), lv.ctypes.data_as(C.POINTER(C.c_uint64)),
                       max_levels)
    return lv


def render(desc, width, height, spp, max_bounces=8, seed=15618, sample_offset=0, flags=0, tile=32,
           rank=0, nranks=1, threads=None, use_bvh=True):
    """Returns (sums[H, W, 4] of per-sample radiance, rays cast)."""
    threads = threads or (os.cpu_count() or 1)
    sums = np.zeros((height, width, 4), dtype=np.float32)
    rays = LIB.pto_render(C.addressof(desc), width, height, spp, max_bounces, seed, sample_offset, flags,
                          tile, rank, nranks, threads, 1 if use_bvh else 0, _f(sums))
    return sums, int(rays)


def image(desc, width, height, spp, **kw):
    """The image a context shows after rendering spp samples: sums / spp (fp32)."""
    sums, rays = render(desc, width, height, spp, **kw)
    img = np.zeros_like(sums)
    img[..., :3] = sums[..., :3] / np.float32(spp)
    img[..., 3] = np.where(sums[..., 3] != 0, 1.0, 0.0)
    return img, rays


def philox(c, k):
    out = (C.c_uint32 * 4)()
    LIB.pto_philox(*[int(x) & 0xFFFFFFFF for x in c], *[int(x) & 0xFFFFFFFF for x in k], out)
    return list(out)


def camera_ray(cam, width, height, ssx, ssy, flags=0):
    """The kernels' camera ray (cu:338-354) through sensor point (ssx = row +
    jitter, ssy = column + jitter): (o.xyz, d.xyz) float32."""
    out = (C.c_float * 6)()
    LIB.pto_camera_ray(C.addressof(cam), width, height, ssx, ssy, flags, out)
    return np.array(out, dtype=np.float32)


def sincos2pi(u):
    s, c = C.c_float(), C.c_float()
    LIB.pto_sincos2pi(C.c_float(u), C.byref(s), C.byref(c))
    return s.value, c.value


def median(img):
    """kernelMedianFilter restated (cu:773-842) on an (H, W, 4) float32 frame."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    out = np.zeros_like(img)
    LIB.pto_median(_f(img), _f(out), img.shape[1], img.shape[0])
    return out
