"""Comparison of this build's radiance with the renders the reference itself
holds (media/pathtracer/reference_results/sky/*.png, 640x480, produced by the
course's completed Scotty3D CPU path tracer; settings in
reference_results/performance.txt:36-69).  Shared by the fixture generator
(tests/golden/make_reference_render_fixture.py, which reads the PNGs) and the
tests (tests/test_reference_renders.py on the oracle, tests/
test_gpu_reference_renders.py through libptcore.so), which read only the
committed fixture tests/golden/reference_renders.npz.

What a reference PNG is: HDRImageBuffer::toColor (image.h:168-185) of the
per-pixel mean radiance c, i.e. trunc(255 * clamp(pow(c * sqrt(2), 1/2.2)))
(ImageBuffer::update_pixel, image.h:49-58), rows written top first
(pathtracer.cpp:577-591).  linearize() inverts it at the centre of the
8-bit bin.

Regions: a pixel's region is the surface its centre ray hits first: (bsdf id,
geometric-normal axis and sign) for triangles, (bsdf id, sphere) for spheres.
Only region interiors count (the 3x3 neighbourhood has one region), so the
comparison does not depend on sub-pixel edge placement.
"""
import math

import numpy as np

W, H = 640, 480
GAMMA, LEVEL = 2.2, 1.0
EXPOSURE = math.sqrt(2.0 ** LEVEL)

# scene -> (reference image under media/pathtracer/reference_results, the
# reference's settings (performance.txt:36-69 for the sky/ renders; none
# published for basic/), the .dae under media/pathtracer)
REFERENCE_IMAGES = {
    "CBbunny": ("sky/CBbunny.png", "max depth 2, 2500 spp, 2 area-light samples", "advanced/CBbunny.dae"),
    "CBspheres_lambertian": ("sky/6400SPP_lambertian.png", "max depth 2, 5000 spp, 2 area-light samples",
                             "advanced/CBspheres_lambertian.dae"),
    "CBcoil": ("sky/CBcoil.png", "max depth 2, 2500 spp, 2 area-light samples", "advanced/CBcoil.dae"),
    "CBspheres": ("sky/6400SPP_classic.png", "max depth 4, 5000 spp, 2 area-light samples",
                  "advanced/CBspheres.dae"),
    # point light (light.cpp:50-57: radiance, pdf 1, no fall-off) over diffuse triangles
    "trigs1": ("basic/trigs1.png", "point light", "basic/trigs1.dae"),
    "trigs5": ("basic/trigs5.png", "point light", "basic/trigs5.dae"),
    "trigs10": ("basic/trigs10.png", "point light", "basic/trigs10.dae"),
    # material-less meshes (DEFAULT_ALBEDO below): a point light, an area light
    "plane4": ("basic/plane.png", "point light, mesh without material", "basic/plane4.dae"),
    "floating": ("basic/floating.png", "area light, meshes without material", "basic/floating.dae"),
    # directional + ambient (InfiniteHemisphereLight) lights over diffuse spheres
    # (the extended light model, pt_scene_desc.lights)
    "sphere_diffuse": ("basic/sphere_diffuse.png", "directional + hemisphere lights", "basic/sphere_diffuse.dae"),
    "sphere7_diffuse": ("basic/sphere7_diffuse.png", "directional + hemisphere lights",
                        "basic/sphere7_diffuse.dae"),
    "carim_diffuse": ("basic/carim_diffuse.png", "directional + hemisphere lights, a mesh without material",
                      "basic/carim_diffuse.dae"),
}
# Scenes the reference renders reproduce with no free factor (scale 1).  The
# four Cornell boxes share one constant (rendered without emission through
# specular bounces, as the reference renders were, they are 0.671-0.681 of
# this build's radiance on every wall, floor and ceiling, whatever the
# distance to the light; DESIGN.md §2.2 lists the hypotheses measured), so
# their scale is fitted -- within that common band -- and the structure is
# compared.
EXACT = ("trigs1", "trigs5", "trigs10", "plane4", "floating", "sphere_diffuse", "sphere7_diffuse", "carim_diffuse")
# A mesh without a material is DiffuseBSDF(1, 1, 1) in this repository
# (src/dynamic_scene/mesh.cpp:37, what pt_scene_load_dae restates) but was
# DiffuseBSDF(0.5, 0.5, 0.5) in the course build that rendered
# reference_results (the line left commented out at mesh.cpp:36): plane.png and
# floating.png are exactly half of the albedo-1 radiance.  The tests render
# those scenes with their default BSDFs at 0.5.
DEFAULT_ALBEDO = {"plane4": 0.5, "floating": 0.5, "carim_diffuse": 0.5}

ROLE_NAMES = ["side", "floor", "ceiling", "back", "object", "light", "mirror"]
SIDE, FLOOR, CEILING, BACK, OBJECT, LIGHT, MIRROR = range(7)
ROOM = (SIDE, FLOOR, CEILING, BACK)
SPHERE_CODE = 6


def course_bsdfs(name, bsdfs):
    """The scene's pt_bsdf array (raw bytes, 36 B records) as the course build
    had it: the material-less meshes' DiffuseBSDF(1) (diffuse, albedo 1)
    at DEFAULT_ALBEDO (mesh.cpp:36-37)."""
    b = np.array(np.frombuffer(np.asarray(bsdfs).tobytes(), np.uint8))
    if name in DEFAULT_ALBEDO:
        rec = b.view(np.float32).reshape(-1, 9)
        typ = b.view(np.int32).reshape(-1, 9)[:, 0]
        dflt = (typ == 0) & np.all(rec[:, 1:4] == 1.0, axis=1)
        rec[dflt, 1:4] = DEFAULT_ALBEDO[name]
    return b


def linearize(v8):
    """8-bit toColor output -> radiance at the centre of its bin."""
    return ((np.asarray(v8, np.float64) + 0.5) / 255.0) ** GAMMA / EXPOSURE


def pixel_rays(ray6):
    """(H*W, 6) origins + directions (scotty_generate_rays) -> pt_intersect
    records (o.xyz, tmax = inf, d.xyz, tmin = 0)."""
    r = np.zeros((len(ray6), 8), np.float32)
    r[:, 0:3] = ray6[:, 0:3]
    r[:, 3] = np.inf
    r[:, 4:7] = ray6[:, 3:6]
    return r


def pixel_centres():
    """Normalised sensor points of the pixel centres, rows bottom-up (the
    ABI's frame order): generate_ray(x, y) with y = 0 at the bottom."""
    r, c = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    return np.stack([(c + 0.5) / W, (r + 0.5) / H], -1).reshape(-1, 2)


def prim_array(prims):
    return np.asarray(prims, np.float32).reshape(-1, 24)


def prim_codes(prims):
    """Region id of every primitive: bsdf * 8 + (axis * 2 + positive) for a
    triangle's geometric normal N (pt_prim q3), bsdf * 8 + 6 for a sphere."""
    p = prim_array(prims)
    meta = p[:, 3].view(np.uint32)
    bsdf = (meta & 0x0FFFFFFF).astype(np.int64)
    sphere = (meta >> 28) == 1
    N = p[:, 12:15]
    ax = np.argmax(np.abs(N), 1)
    pos = N[np.arange(len(N)), ax] > 0
    return np.where(sphere, bsdf * 8 + SPHERE_CODE, bsdf * 8 + ax * 2 + pos)


def label_map(prims, prim_of_pixel):
    codes = prim_codes(prims)
    p = np.asarray(prim_of_pixel, np.int64)
    return np.where(p >= 0, codes[np.maximum(p, 0)], -1).reshape(H, W).astype(np.int32)


def roles(prims, bsdf_types):
    """Role of every region: a bsdf whose triangles all lie in one axis plane
    is a wall of the box (side: x, floor: +y normal side up, ceiling, back: z);
    the emitter is the light; mirrors/glass are `mirror`; the rest objects."""
    p = prim_array(prims)
    meta = p[:, 3].view(np.uint32)
    bsdf = (meta & 0x0FFFFFFF).astype(np.int64)
    sphere = (meta >> 28) == 1
    codes = prim_codes(prims)
    out = {}
    for b in np.unique(bsdf):
        sel = bsdf == b
        t = int(bsdf_types[b])
        for c in np.unique(codes[sel]):
            if t == 3:
                out[int(c)] = LIGHT
            elif t != 0:
                out[int(c)] = MIRROR
            elif sphere[sel].any():
                out[int(c)] = OBJECT
            else:
                v = np.concatenate([p[sel, 0:3], p[sel, 4:7], p[sel, 8:11]])
                ax = int(c % 8) // 2
                planar = v[:, ax].max() - v[:, ax].min() < 1e-4 and len(np.unique(codes[sel])) <= 2
                if not planar:
                    out[int(c)] = OBJECT
                else:
                    out[int(c)] = SIDE if ax == 0 else (BACK if ax == 2 else (
                        FLOOR if v[:, 1].mean() < 0.5 * (p[:, 1].min() + p[:, 1].max()) else CEILING))
    return out


def interior(lab):
    from scipy.ndimage import maximum_filter, minimum_filter
    return (minimum_filter(lab, 3) == lab) & (maximum_filter(lab, 3) == lab)


def region_means(lin, lab, mask, min_pixels=200):
    """{region: (pixels, mean RGB)} over mask & region."""
    out = {}
    for r in np.unique(lab[mask]):
        m = mask & (lab == r)
        n = int(m.sum())
        if r >= 0 and n >= min_pixels:
            out[int(r)] = (n, lin[m].mean(0))
    return out


def block_means(img, b=8):
    h, w = img.shape[0] // b, img.shape[1] // b
    return img[: h * b, : w * b].reshape(h, b, w, b, -1).mean((1, 3))


def tonemap8(lin):
    """toColor in numpy (image.h:168-185 + update_pixel's truncation)."""
    c = np.clip(np.power(np.maximum(lin, 0.0) * EXPOSURE, 1.0 / GAMMA), 0.0, 1.0)
    return np.floor(c * 255.0)


def compare(fx, img, scale=None):
    """Compare a rendered frame (H, W, >=3 linear radiance, bottom-up rows)
    with one scene's fixture entries fx (dict of arrays, names as the
    generator writes them).  Returns a dict of the measured quantities."""
    lab = fx["labels"]
    mask = fx["mask"]
    rid = fx["region_ids"]
    role = dict(zip(rid.tolist(), fx["region_roles"].tolist()))
    refm = dict(zip(rid.tolist(), fx["region_ref"]))
    ours = region_means(np.asarray(img, np.float64)[..., :3], lab, mask, min_pixels=1)
    ratio = {r: refm[r] / np.maximum(ours[r][1], 1e-12) for r in rid.tolist() if r in ours}
    room = [r for r in ratio if role[r] in (SIDE, FLOOR, CEILING)]
    if scale is None:  # the one global factor: median over the side walls, floor and ceiling
        scale = float(np.median(np.concatenate([ratio[r] for r in room])))
    rel = {r: ratio[r] / scale for r in ratio}
    # light-distance profile inside each wall: ref / ours per distance quintile
    spread = {}
    qb = fx["dist_bin"]
    for r in room + [r for r in ratio if role[r] == BACK]:
        prof = []
        for k in range(5):
            m = mask & (lab == r) & (qb == k)
            if m.sum() >= 50:
                ours_k = np.asarray(img, np.float64)[m][:, :3].mean()
                prof.append(fx["bin_ref"][list(rid).index(r), k].mean() / max(ours_k, 1e-12))
        if len(prof) == 5:  # (nearest / farthest quintile, max / min)
            spread[r] = (prof[0] / prof[-1], max(prof) / min(prof))
    # 8x8 block means of the 8-bit frames, ours scaled by the global factor
    # (a noisy frame's tone-mapped mean sits below its converged value: for
    # low sample counts compare block_lin, the blocks' linear radiance)
    lin = np.asarray(img, np.float64)[..., :3] * scale
    ours8 = block_means(tonemap8(lin))
    bdiff = np.abs(ours8 - fx["ref_blocks"]).max(-1)
    bref = fx["ref_blocks_lin"]
    blin = (np.abs(block_means(lin) - bref) / np.maximum(bref, 0.02)).max(-1)
    return dict(scale=scale, rel=rel, role=role, spread=spread, block_diff=bdiff, block_lin=blin)


def load(path):
    """The fixture as {scene: {key: array}} with the packed masks unpacked."""
    out = {}
    with np.load(path, allow_pickle=False) as z:
        for k in z.files:
            scene, key = k.split("/", 1)
            out.setdefault(scene, {})[key] = z[k]
    n = H * W
    for fx in out.values():
        fx["labels"] = fx["labels"].astype(np.int32)
        fx["mask"] = np.unpackbits(fx["mask"])[:n].reshape(H, W).astype(bool)
        fx["ref_masks"] = np.unpackbits(fx["ref_masks"])[: 4 * n].reshape(4, H, W).astype(bool)
    return out
