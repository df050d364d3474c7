"""Radiance checks that do not share the oracle's math (the GPU and
the oracle restate the same estimator, so a shared mistake in NEE, the pdf or
the BSDF weights would pass every parity test).  Each scene here has an
answer from first principles, computed in the test with numpy / scipy:

* furnace sphere (default arithmetic): the inside of a diffuse sphere of albedo
  rho with a point light of radiance Le at its centre.  Every path vertex lies
  on the wall facing the light (cos = 1), so each vertex adds throughput x
  rho Le / pi by NEE (kernelDirectLightRays, cu:380-481, with the point-light
  extension of SURVEY §8(a) v), and the BSDF sample (cu:616-639) multiplies the
  throughput by rho in expectation (2 |cos| rho under uniform hemisphere
  sampling, exactly rho under cosine sampling).  A pixel's mean radiance is
  the truncated geometric series Le / pi * sum_{k=1}^{K+1} rho^k, K = max_bounces;
* closed emissive box (PT_FLAG_REF_ARITH, the reference kernels' literal
  arithmetic): every wall an EmissionBSDF of radiance Le, which the reference
  reads as a DiffuseBSDF of albedo Le (cu:1705-1711) and whose radiance it adds
  at every hit, light += radiance * importance (cu:1243): mean radiance
  Le * sum_{k=0}^{K} Le^k;
* area light over a diffuse plane (default: the light pdf of light.cpp:81-92,
  whose unnormalised cosine makes it the solid-angle pdf times the distance;
  PT_FLAG_EXACT_LIGHT_PDF: the solid-angle pdf): a one-sided square light of radiance Le at
  height h over a plane of albedo rho.  The default estimator's expectation is
  rho / pi * Le * integral cos cos / r dA, PT_FLAG_EXACT_LIGHT_PDF's rho / pi * E
  with E = Le * integral cos cos / r^2 dA (the irradiance); the reference
  kernels' literal formula (PT_FLAG_REF_ARITH: pdf from the unnormalised cosine,
  cu:422-430, and BSDF_DIFFUSE_MULTIPLIER 0.3183) has expectation
  rho * 0.3183 * Le * integral cos cos / r dA.  Both integrals by scipy
  quadrature, at the point under the light's centre and under a corner.

Each scene runs twice: as a single BVH leaf (k_path_leaf) and split into many
primitives (the breadth-first traversal + k_shade_push wavefront).
Tolerance: 6 standard errors of the image mean (from the spread of the pixel
means) plus 2e-6 relative for fp32 rounding; the cosine-sampled furnace is
deterministic up to rounding (every pixel within 2e-5 relative)."""
import math

import numpy as np
import pytest

import ptrace

gpu = pytest.mark.gpu  # (every test but the quadrature check; gpu_ctx skips without a GPU)

W = H = 1024
SPP = 256


def _bsdf(kind, rgb):
    b = ptrace.pt_bsdf()
    b.type = kind
    for k in range(3):
        b.albedo[k] = rgb[k]
    return b


def _light(kind, radiance, position=(0, 0, 0), direction=(0, -1, 0), dim_x=(0, 0, 0), dim_y=(0, 0, 0)):
    L = ptrace.pt_light()
    L.type = kind
    for k in range(3):
        L.radiance[k] = radiance[k]
        L.position[k] = position[k]
        L.direction[k] = direction[k]
        L.dim_x[k] = dim_x[k]
        L.dim_y[k] = dim_y[k]
    L.area = float(np.linalg.norm(dim_x) * np.linalg.norm(dim_y))
    return L


def _camera(origin, look, left, up):
    c = ptrace.pt_camera()
    for k in range(3):
        c.origin[k], c.look_at[k], c.left[k], c.up[k] = origin[k], look[k], left[k], up[k]
    return c


def _render(ctx, scene, bounces, flags=0):
    ctx.load_scene(scene)
    ctx.clear()
    ctx.render(W, H, SPP, max_bounces=bounces, seed=15618, flags=flags)
    img = ctx.get_image()[..., :3].astype(np.float64)
    assert np.isfinite(img).all()
    return img


def _assert_mean(img, expected):
    px = img.mean(axis=2).ravel()
    se = px.std() / math.sqrt(px.size)
    err = abs(px.mean() - expected)
    assert err < 6 * se + 2e-6 * expected, (px.mean(), expected, se)
    # the image is uniform: no pixel's mean far outside its sampling spread
    assert np.abs(px - expected).max() < 8 * px.std() + 1e-5 * expected
    return err / se if se > 0 else 0.0


def _grid_quads(corner, eu, ev, n):
    """n x n grid of quads (two triangles each) spanning corner + [0,1] eu + [0,1] ev."""
    c, eu, ev = (np.asarray(x, np.float64) for x in (corner, eu, ev))
    tris = []
    for i in range(n):
        for j in range(n):
            p00 = c + eu * (i / n) + ev * (j / n)
            p10 = c + eu * ((i + 1) / n) + ev * (j / n)
            p01 = c + eu * (i / n) + ev * ((j + 1) / n)
            p11 = c + eu * ((i + 1) / n) + ev * ((j + 1) / n)
            tris += [np.concatenate([p00, p10, p11]), np.concatenate([p00, p11, p01])]
    return np.array(tris, np.float32)


# ---- furnace sphere ----------------------------------------------------------------
def _furnace_sphere(rho, Le, split):
    centre, R = np.array([0.3, 1.1, -0.4]), 2.0
    sph = [[*centre, R]]
    if split:
        # small spheres in the corners of the big sphere's box (outside the
        # sphere, never hit from inside) make a multi-level BVH whose boxes the
        # inside rays still enter
        rng = np.random.default_rng(3)
        for _ in range(600):
            while True:
                p = centre + rng.uniform(-R, R, 3)
                if np.linalg.norm(p - centre) > R + 0.08:
                    break
            sph.append([*p, 0.03])
    sph = np.array(sph, np.float32)
    bsdf = _bsdf(ptrace.PT_BSDF_DIFFUSE, (rho, rho, rho))
    light = _light(ptrace.PT_LIGHT_POINT, (Le, Le, Le), position=centre)
    cam = _camera(centre + [0.1, 0.2, -0.3], (0, 0, -1), (1, 0, 0), (0, -1, 0))
    return ptrace.Scene.from_mesh(None, [bsdf], spheres=sph, light=light, camera=cam)


def _series(rho, Le, K):
    return Le / math.pi * sum(rho ** k for k in range(1, K + 2))


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("K", [0, 3, 8])
@gpu
def test_furnace_sphere_cosine_sampling_is_exact(gpu_ctx, split, K):
    """Cosine-weighted diffuse sampling: the throughput is exactly rho^k, so
    every sample (hence every pixel) equals the series."""
    rho, Le = 0.7, 2.0
    img = _render(gpu_ctx, _furnace_sphere(rho, Le, split), K, flags=ptrace.PT_FLAG_COSINE_DIFFUSE)
    exp = _series(rho, Le, K)
    assert np.abs(img - exp).max() < 2e-5 * exp, (img.min(), img.max(), exp)


@pytest.mark.parametrize("split", [False, True])
@gpu
def test_furnace_sphere_uniform_hemisphere(gpu_ctx, split):
    """The reference's uniform hemisphere sampling (cu:619-639): throughput x
    2 |cos| rho per bounce, rho in expectation."""
    rho, Le, K = 0.8, 1.5, 8
    img = _render(gpu_ctx, _furnace_sphere(rho, Le, split), K)
    _assert_mean(img, _series(rho, Le, K))


# ---- closed emissive box (reference arithmetic) --------------------------------------
def _emissive_box(Le, split):
    n = 12 if split else 1
    lo, hi = np.array([-1.0, -0.5, -1.5]), np.array([1.2, 1.5, 0.8])
    d = hi - lo
    ex, ey, ez = np.array([d[0], 0, 0]), np.array([0, d[1], 0]), np.array([0, 0, d[2]])
    faces = [(lo, ex, ey), (lo, ey, ez), (lo, ez, ex), (hi, -ex, -ey), (hi, -ey, -ez), (hi, -ez, -ex)]
    tris = np.concatenate([_grid_quads(c, u, v, n) for c, u, v in faces])
    bsdf = _bsdf(ptrace.PT_BSDF_EMISSION, (Le, Le, Le))
    cam = _camera((lo + hi) / 2 + [0.05, -0.1, 0.2], (0, 0, -1), (1, 0, 0), (0, -1, 0))
    return ptrace.Scene.from_mesh(tris, [bsdf], light=_light(ptrace.PT_LIGHT_NONE, (0, 0, 0)), camera=cam)


@pytest.mark.parametrize("split", [False, True])
@gpu
def test_closed_emissive_box_ref_arith(gpu_ctx, split):
    Le, K = 0.6, 8
    img = _render(gpu_ctx, _emissive_box(Le, split), K, flags=ptrace.PT_FLAG_REF_ARITH)
    _assert_mean(img, Le * sum(Le ** k for k in range(K + 1)))


# ---- area light over a diffuse plane ---------------------------------------------------
A_SIDE, HGT = 1.2, 0.9   # light edge, height over the plane
LIGHT_C = np.array([0.2, 0.0, -0.3])
# The estimator shades the hit point moved back along the ray by 1e-3
# (its.pt += -r->d * 1e-3, cu:1224): the camera looks straight down, so NEE
# starts 1e-3 above the plane (0.15 % more irradiance at this height).
HIT_OFFSET = 1e-3


def _light_integral(px, pz, power, h=HGT - HIT_OFFSET):
    """integral over the light of cos_n cos_l / r^power dA for the point
    (px, HGT - h, pz) (both cosines = h / r for a parallel light)."""
    from scipy import integrate
    x0, z0 = LIGHT_C[0] - A_SIDE / 2 - px, LIGHT_C[2] - A_SIDE / 2 - pz
    f = lambda z, x: h * h / (x * x + z * z + h * h) ** (1 + power / 2)
    v, err = integrate.dblquad(f, x0, x0 + A_SIDE, z0, z0 + A_SIDE, epsabs=1e-13, epsrel=1e-11)
    return v


def _plane_scene(rho, Le, target, split):
    n = 48 if split else 1
    tris = _grid_quads((-30, 0, -30), (60, 0, 0), (0, 0, 60), n)
    bsdf = _bsdf(ptrace.PT_BSDF_DIFFUSE, (rho, rho, rho))
    light = _light(ptrace.PT_LIGHT_AREA, (Le, Le, Le), position=LIGHT_C + [0, HGT, 0], direction=(0, -1, 0),
                   dim_x=(A_SIDE, 0, 0), dim_y=(0, 0, A_SIDE))
    # straight down from above the light, a narrow field (|left| = |up| = s:
    # the frame covers +-1.5 s around the target), so the pixels sample one point
    s = 0.002
    cam = _camera((target[0], 3.0, target[1]), (0, -1, 0), (s, 0, 0), (0, 0, s))
    return ptrace.Scene.from_mesh(tris, [bsdf], light=light, camera=cam)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("where", ["centre", "corner"])
@gpu
def test_area_light_over_plane(gpu_ctx, split, where):
    rho, Le, K = 0.75, 3.0, 4
    tgt = (LIGHT_C[0], LIGHT_C[2]) if where == "centre" else (LIGHT_C[0] + A_SIDE / 2, LIGHT_C[2] - A_SIDE / 2)
    sc = _plane_scene(rho, Le, tgt, split)
    # default, the light pdf of AreaLight::sample_L (light.cpp:81-92: the
    # unnormalised cosine, pdf x dist): rho / pi * Le * int cos cos / r dA
    img = _render(gpu_ctx, sc, K)
    _assert_mean(img, rho / math.pi * Le * _light_integral(tgt[0], tgt[1], 1))
    # PT_FLAG_EXACT_LIGHT_PDF: rho / pi * E, E = Le * int cos cos / r^2 dA (the irradiance)
    img = _render(gpu_ctx, sc, K, flags=ptrace.PT_FLAG_EXACT_LIGHT_PDF)
    _assert_mean(img, rho / math.pi * Le * _light_integral(tgt[0], tgt[1], 2))
    # the reference's NEE formula (cu:416-446): rho * 0.3183 * Le * int cos cos / r dA
    img = _render(gpu_ctx, sc, K, flags=ptrace.PT_FLAG_REF_ARITH)
    _assert_mean(img, rho * np.float32(0.3183) * Le * _light_integral(tgt[0], tgt[1], 1))


def test_light_integral_closed_forms():
    """The quadrature against the closed forms (point under the centre): the
    parallel-rectangle form factor and h * atan(XY / (h sqrt(h^2 + X^2 + Y^2)))."""
    X = Y = A_SIDE / 2
    h = HGT
    a, b = X / h, Y / h
    F = (a / math.sqrt(1 + a * a) * math.atan(b / math.sqrt(1 + a * a))
         + b / math.sqrt(1 + b * b) * math.atan(a / math.sqrt(1 + b * b))) / (2 * math.pi)
    assert abs(_light_integral(LIGHT_C[0], LIGHT_C[2], 2, h=h) - 4 * math.pi * F) < 1e-10
    g = h * math.atan(X * Y / (h * math.sqrt(h * h + X * X + Y * Y)))
    assert abs(_light_integral(LIGHT_C[0], LIGHT_C[2], 1, h=h) - 4 * g) < 1e-10
