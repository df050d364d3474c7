"""Synthetic workloads built from the reference's own media.

dragon_proxy(): BASELINE.json configs[3]/[4] name a ~100k-triangle "dragon"
scene, but media/pathtracer/dragon.dae is missing from the reference checkout
(.MISSING_LARGE_BLOBS).  The stand-in is built
deterministically from CBbunny.dae (flattened fixture tests/golden/scenes/
CBbunny.npz): the Cornell box walls and area light once, three copies of the
28,576-triangle bunny (scaled 0.6, rotated about y by 0/120/240 degrees, set
side by side on the floor) and a tessellated mirror sphere (60 x 120 UV
sphere, 14,160 triangles) under the light: 99,900 triangles in total, run
through the same reference BVH build (pt_scene_from_mesh) or, as
"dragon_proxy_gpubvh", through the GPU build (pt_scene_build_gpu: the
top-down SAH; "dragon_proxy_ploc" / "dragon_proxy_lbvh" are the same scene
with PLOC clustering / the radix tree).

bunny_lit(): bunny.dae (config 4's wide-level scene) with CBbunny's light.
rebuilt(name, ...): any fixture rebuilt from its meshes (host or GPU build).
"""
import math
from pathlib import Path

import numpy as np

import ptrace

ROOT = Path(__file__).resolve().parent.parent
FIXTURES = ROOT / "tests" / "golden" / "scenes"


def _bsdf(kind, albedo, trans=(0.0, 0.0, 0.0), ior=1.0):
    b = ptrace.pt_bsdf()
    b.type = kind
    for k in range(3):
        b.albedo[k] = albedo[k]
        b.transmittance[k] = trans[k]
    b.ior = ior
    return b


def _uv_sphere(centre, radius, nlat, nlon):
    """Triangles (n, 9) and vertex normals (n, 9) of a UV sphere."""
    cx, cy, cz = centre
    th = np.linspace(0.0, math.pi, nlat + 1)
    ph = np.linspace(0.0, 2.0 * math.pi, nlon + 1)
    n = np.stack([np.sin(th)[:, None] * np.cos(ph)[None, :],
                  np.cos(th)[:, None] * np.ones_like(ph)[None, :],
                  np.sin(th)[:, None] * np.sin(ph)[None, :]], axis=-1)  # (nlat+1, nlon+1, 3)
    p = n * radius + np.array([cx, cy, cz])
    tris, nrms = [], []
    for i in range(nlat):
        for j in range(nlon):
            a, b, c, d = (i, j), (i + 1, j), (i + 1, j + 1), (i, j + 1)
            quads = []
            if i != 0:
                quads.append((a, c, d))
            if i != nlat - 1:
                quads.append((a, b, c))
            for t in quads:
                tris.append(np.concatenate([p[v] for v in t]))
                nrms.append(np.concatenate([n[v] for v in t]))
    return np.asarray(tris, np.float32), np.asarray(nrms, np.float32)


def fixture_arrays(name):
    """A committed fixture back in mesh input order: dict of positions (n, 9),
    normals (n, 9), tri_bsdf, spheres (m, 4), sphere_bsdf, bsdfs, light,
    camera (the inputs of pt_scene_from_mesh / pt_scene_build_gpu)."""
    with np.load(FIXTURES / f"{name}.npz", allow_pickle=False) as z:
        z = ptrace._upgrade_bsdfs({k: z[k] for k in z.files})
        q = z["prims"]
        sh = z["shading"]
        order = np.argsort(z["sorted_to_input"], kind="stable")
        bs = np.frombuffer(z["bsdfs"].tobytes(), dtype=np.uint8)
        light = ptrace.pt_light.from_buffer_copy(z["light"].tobytes())
        camera = ptrace.pt_camera.from_buffer_copy(z["camera"].tobytes())
    q, sh = q[order], sh[order]
    meta = q[:, 3].view(np.uint32)
    tri = (meta >> 28) == ptrace.PT_PRIM_TRIANGLE
    sz = ptrace.C.sizeof(ptrace.pt_bsdf)
    bsdfs = [ptrace.pt_bsdf.from_buffer_copy(bs[i * sz:(i + 1) * sz].tobytes()) for i in range(len(bs) // sz)]
    t, sp = q[tri], q[~tri]
    return {"positions": np.concatenate([t[:, 0:3], t[:, 4:7], t[:, 8:11]], axis=1),
            "normals": np.concatenate([sh[tri][:, 0:3], sh[tri][:, 4:7], sh[tri][:, 8:11]], axis=1),
            "tri_bsdf": (meta[tri] & 0x0FFFFFFF).astype(np.int32),
            "spheres": np.concatenate([sp[:, 0:3], sp[:, 4:5]], axis=1) if len(sp) else None,
            "sphere_bsdf": (meta[~tri] & 0x0FFFFFFF).astype(np.int32) if len(sp) else None,
            "bsdfs": bsdfs, "light": light, "camera": camera}


def rebuilt(name, gpu_device=None, max_leaf=32, builder="sah"):
    """Fixture `name` rebuilt from its meshes: the host SAH build
    (pt_scene_from_mesh) or the GPU build (gpu_device=k)."""
    a = fixture_arrays(name)
    return ptrace.Scene.from_mesh(a["positions"], a["bsdfs"], normals=a["normals"], tri_bsdf=a["tri_bsdf"],
                                  spheres=a["spheres"], sphere_bsdf=a["sphere_bsdf"], light=a["light"],
                                  camera=a["camera"], gpu_device=gpu_device, max_leaf=max_leaf, builder=builder)


def bunny_lit():
    """bunny.dae (33,696 triangles; BVH level 6 holds the 1,167 nodes that
    overflow the reference's per-level buffers) lit by CBbunny.dae's area light:
    bunny.dae has no light of its own (the reference would add a default
    ambient light and read it as an area light, cu:1630-1633, 1741)."""
    sc = ptrace.ArrayScene.load(FIXTURES / "bunny.npz")
    with np.load(FIXTURES / "CBbunny.npz", allow_pickle=False) as z:
        sc.a["light"] = z["light"].copy()
    return sc


def dragon_proxy_arrays():
    """positions (n, 9), normals (n, 9), tri_bsdf (n,), bsdfs, light, camera."""
    with np.load(FIXTURES / "CBbunny.npz", allow_pickle=False) as z:
        z = ptrace._upgrade_bsdfs({k: z[k] for k in z.files})
        q = z["prims"]
        sh = z["shading"]
        order = np.argsort(z["sorted_to_input"], kind="stable")  # back to mesh input order
        bs = np.frombuffer(z["bsdfs"].tobytes(), dtype=np.uint8)
        light = ptrace.pt_light.from_buffer_copy(z["light"].tobytes())
        camera = ptrace.pt_camera.from_buffer_copy(z["camera"].tobytes())
    q, sh = q[order], sh[order]
    bid = q[:, 3].view(np.uint32) & 0x0FFFFFFF
    pos = np.concatenate([q[:, 0:3], q[:, 4:7], q[:, 8:11]], axis=1)
    nrm = np.concatenate([sh[:, 0:3], sh[:, 4:7], sh[:, 8:11]], axis=1)
    nb = len(bs) // ptrace.C.sizeof(ptrace.pt_bsdf)
    bsdfs = [ptrace.pt_bsdf.from_buffer_copy(bs[i * ptrace.C.sizeof(ptrace.pt_bsdf):(i + 1) *
                                                ptrace.C.sizeof(ptrace.pt_bsdf)].tobytes()) for i in range(nb)]
    bunny_id = int(np.bincount(bid).argmax())
    room = bid != bunny_id
    out_p, out_n, out_b = [pos[room]], [nrm[room]], [bid[room].astype(np.int32)]
    bp, bn = pos[~room].reshape(-1, 3), nrm[~room].reshape(-1, 3)
    for k, (x, z) in enumerate([(-0.55, 0.35), (0.0, -0.25), (0.55, 0.35)]):
        a = math.radians(120.0 * k)
        c, s = math.cos(a), math.sin(a)
        R = np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]], np.float64)
        p = (bp.astype(np.float64) * 0.6) @ R.T + np.array([x, 0.0, z])
        n = bn.astype(np.float64) @ R.T
        out_p.append(p.reshape(-1, 9).astype(np.float32))
        out_n.append(n.reshape(-1, 9).astype(np.float32))
        out_b.append(np.full(len(p) // 3, bunny_id, np.int32))
    mirror = len(bsdfs)
    bsdfs.append(_bsdf(ptrace.PT_BSDF_MIRROR, (0.9, 0.9, 0.9)))
    sp, sn = _uv_sphere((0.0, 1.0, 0.45), 0.25, 60, 120)
    out_p.append(sp)
    out_n.append(sn)
    out_b.append(np.full(len(sp), mirror, np.int32))
    return (np.concatenate(out_p), np.concatenate(out_n), np.concatenate(out_b), bsdfs, light, camera)


def dragon_proxy(gpu_device=None, max_leaf=32, builder="sah"):
    """The ~100k-triangle config-4/5 scene as a ptrace.Scene: the reference's
    host SAH build, or (gpu_device=k) the GPU build ("sah": the reference's
    12-plane SAH split rule, level-synchronous on the device, the default
    since round 6; "ploc" clustering; the "lbvh" radix tree) with wide leaves
    of <= max_leaf primitives (32, the
    reference's leaf size; the radix tree: 5,073 Mrays/s vs 4,918 at 16 and
    4,556 at 8 on the dragon proxy)."""
    pos, nrm, tb, bsdfs, light, camera = dragon_proxy_arrays()
    return ptrace.Scene.from_mesh(pos, bsdfs, normals=nrm, tri_bsdf=tb, light=light, camera=camera,
                                  gpu_device=gpu_device, max_leaf=max_leaf, builder=builder)


def load(name):
    """A bench/test workload by name: a committed fixture or a synthetic scene."""
    if name == "dragon_proxy":
        return dragon_proxy()
    if name == "dragon_proxy_gpubvh":
        return dragon_proxy(gpu_device=0)
    if name == "dragon_proxy_lbvh":
        return dragon_proxy(gpu_device=0, builder="lbvh")
    if name == "dragon_proxy_sah":
        return dragon_proxy(gpu_device=0, builder="sah")
    if name == "dragon_proxy_ploc":
        return dragon_proxy(gpu_device=0, builder="ploc")
    if name == "bunny":
        return bunny_lit()
    return ptrace.ArrayScene.load(FIXTURES / f"{name}.npz")
