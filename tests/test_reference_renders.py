"""The oracle's estimator against the renders the reference itself holds
(media/pathtracer/reference_results/sky, 640x480, Scotty3D's completed CPU
path tracer; tests/refrender.py says what a PNG is and how regions are
formed; the numbers come from tests/golden/reference_renders.npz, made by
tests/golden/make_reference_render_fixture.py).  No GPU: this pins the CPU
oracle, which every GPU parity test then equals bit for bit.

Exact scenes (refrender.EXACT: basic/trigs1, trigs5, trigs10 and plane4 --
a point light over diffuse triangles --, floating -- an area light, a
floating quad's shadow --, sphere_diffuse, sphere7_diffuse and carim_diffuse
-- a directional and an ambient (InfiniteHemisphereLight) light over diffuse
spheres, the extended light model): no free factor.  Every region's mean
radiance is within 1.5 % of the reference render's (measured at 64 spp:
<= 1.0 %; at 256: <= 0.6 %), the ratio is flat in the distance to the light
(max/min over distance quintiles <= 1.03), and 98 % of the 8x8 blocks' linear
radiance is within 10 % of the reference's (the GPU test, at 1024 spp, also
holds 97 % of the 8-bit blocks within 2 levels).  plane.png, floating.png
and carim_diffuse.png come from the course build, in which a mesh without a
material is DiffuseBSDF(0.5) (mesh.cpp:36; this repository's mesh.cpp:37
says 1.0, which pt_scene_load_dae follows): they render with their default
BSDFs at 0.5 (refrender.DEFAULT_ALBEDO).

Cornell boxes -- what their reference renders establish (stated tolerances below):
  * the area-light estimator is AreaLight::sample_L's (light.cpp:81-92, the
    unnormalised cosine): inside every wall the ratio reference / oracle is
    flat in the distance to the light (max/min over distance quintiles
    <= 1.03), while the solid-angle pdf (PT_FLAG_EXACT_LIGHT_PDF) is off by
    the distance itself (>= 1.3 across the side walls);
  * the renders count no emission reached through a specular bounce (round
    6): rendered with PT_FLAG_NO_EMISSION (no emitter counted anywhere; the
    light's own pixels are saturated in the reference and so outside the
    compared regions), the four Cornell files share one factor, 0.671-0.681
    at 64 spp, and CBspheres' ceiling, floor and side walls come within 1 %;
    with this build's default (an emitter seen through a mirror or glass
    counts) CBspheres' factor drops to 0.622, its ceiling sits 5 % low and
    CBcoil's ceiling 7 % low -- the caustic paths the reference drops
    (test_specular_emission_is_not_in_the_reference);
  * paths are not cut at the reference's "max depth 2": with 2 bounces the
    colour bleed and the ceiling (lit only indirectly) fall short (ceiling /
    floor ratio 1.14 at 2 bounces, 1.05 at 3, 1.02 at 4, 1.00 at 8), so the
    comparison renders 8 bounces, the bench's count;
  * one factor common to the four Cornell files remains, 0.677 +- 0.005,
    while the exact scenes above (the same tone map, camera, BSDF and light
    code) need none.  Hypotheses measured and rejected:
    the light node's 0.6 x 0.8 scale (area, sample extent, axes swapped:
    the factor stays 0.68-0.69 and the distance profiles get worse), the
    log-average tone map left commented out at pathtracer.cpp:134 (image.h:
    143-167: it would give 0.04-560), a starter-stub light sampler that
    always returns the light's centre (sampler.cpp:7-12: hard shadows, worse
    blocks), the coil's phong colour or the course default DiffuseBSDF(0.5)
    in place of its <mirror> (the coil stays at 0.14-0.5);
  * residuals after that factor (documented, asserted as bands): the back
    wall is 4-8 % brighter in the reference, the objects (bunny, spheres)
    4-14 % darker, two of CBcoil's three coil regions 0.29-0.31 and the third
    0.6-0.76 of ours.
"""
import numpy as np
import pytest

import ptrace
import pyoracle
import refrender as rr
from conftest import ROOT

FIXTURE = ROOT / "tests" / "golden" / "reference_renders.npz"
DIFFUSE = ["CBbunny", "CBspheres_lambertian"]
SPP_CPU = 16  # region means average >= 10^4 pixels: noise well under the bands
SPP_EXACT = 64  # the exact scenes' smaller regions and blocks


@pytest.fixture(scope="module")
def fixture():
    return rr.load(FIXTURE)


def course_scene(name):
    """The scene fixture with the course build's default BSDF (refrender.course_bsdfs)."""
    sc = ptrace.ArrayScene.load(ROOT / "tests" / "golden" / "scenes" / f"{name}.npz")
    sc.a["bsdfs"] = rr.course_bsdfs(name, sc.a["bsdfs"])
    return sc


def oracle_frame(name, fx, spp, flags=0, max_bounces=8):
    d = course_scene(name).desc()
    d.camera = ptrace.pt_camera.from_buffer_copy(fx["camera"].tobytes())
    img, _ = pyoracle.image(d, rr.W, rr.H, spp, max_bounces=max_bounces, flags=flags)
    return img


# The reference's emission rule for the Cornell renders (module docstring):
# no emitter counted through a specular bounce.
CORNELL_FLAGS = ptrace.PT_FLAG_NO_EMISSION
SPECULAR = ["CBspheres", "CBcoil"]
CORNELL_SCALE = (0.665, 0.690)  # the one factor common to the four Cornell files


def check_cornell(c, block_frac, specular=False):
    """The bands every Cornell scene meets (module docstring)."""
    assert CORNELL_SCALE[0] <= c["scale"] <= CORNELL_SCALE[1], c["scale"]
    mirrors = sorted(r for r in c["rel"] if c["role"][r] == rr.MIRROR)
    for r, v in c["rel"].items():
        role = c["role"][r]
        if role in (rr.SIDE, rr.FLOOR, rr.CEILING):
            assert np.all(np.abs(v - 1.0) <= 0.03), (r, rr.ROLE_NAMES[role], v)
        elif role == rr.BACK:
            assert np.all((v >= 1.0) & (v <= 1.10)), (r, v)
        elif role == rr.OBJECT:
            assert np.all((v >= 0.80) & (v <= 1.0)), (r, v)
        elif role == rr.MIRROR and len(mirrors) == 2:  # CBspheres: the glass and mirror spheres
            assert np.all(np.abs(v - 1.0) <= 0.06), (r, v)
        elif role == rr.MIRROR:  # CBcoil's coil (measured 0.29-0.31, 0.29-0.31, 0.6-0.76)
            assert np.all((v >= 0.25) & (v <= 0.85)), (r, v)
    for r, (near_far, mx) in c["spread"].items():
        role = c["role"][r]
        lim = 1.03 if role == rr.SIDE else (1.13 if specular and role in (rr.FLOOR, rr.BACK) else 1.09)
        assert mx <= lim, (r, rr.ROLE_NAMES[role], near_far, mx)
    assert (c["block_diff"] <= 8).mean() >= block_frac, (c["block_diff"] <= 8).mean()


def check_diffuse(c, block_frac):
    check_cornell(c, block_frac)


def check_exact(c, converged=False):
    """The bands every exact scene meets (module docstring).  converged (GPU,
    1024 spp): the 8-bit blocks too -- a noisy frame's tone-mapped block
    means sit below their converged values, the linear ones do not."""
    assert c["scale"] == 1.0
    for r, v in c["rel"].items():
        assert np.all(np.abs(v - 1.0) <= 0.015), (r, v)
    for r, (near_far, mx) in c["spread"].items():
        assert mx <= 1.03, (r, near_far, mx)
    bl = c["block_lin"]
    assert (bl <= 0.10).mean() >= 0.98, (bl <= 0.10).mean()
    if converged:
        bd = c["block_diff"]
        assert (bd <= 2).mean() >= 0.97 and bd.max() <= 6, ((bd <= 2).mean(), bd.max())


def test_fixture_framing(fixture):
    """The reference framing was recovered: its red / blue walls, light and
    background coincide with the scene's regions under the stored camera."""
    assert set(fixture) == set(rr.REFERENCE_IMAGES)
    for name, fx in fixture.items():
        assert fx["framing_agreement"] >= 0.985, (name, fx["framing_agreement"])
        if name not in rr.EXACT:
            roles = set(fx["region_roles"].tolist())
            assert {rr.SIDE, rr.FLOOR, rr.CEILING, rr.BACK} <= roles, name
    assert float(fixture["CBbunny"]["zoom"]) == 1.0  # Scotty3D's own placement
    assert 0.6 < float(fixture["CBspheres_lambertian"]["zoom"]) < 0.7


@pytest.mark.parametrize("name", DIFFUSE + SPECULAR)
def test_oracle_matches_reference_render(fixture, name):
    c = rr.compare(fixture[name], oracle_frame(name, fixture[name], SPP_CPU, flags=CORNELL_FLAGS))
    check_cornell(c, block_frac=0.80, specular=name in SPECULAR)


def test_specular_emission_is_not_in_the_reference(fixture):
    """The discriminating check for the emission rule: counting the emitter
    through the spheres (this build's default) leaves CBspheres' factor
    outside the common band and its ceiling >= 3 % below the other walls."""
    c = rr.compare(fixture["CBspheres"], oracle_frame("CBspheres", fixture["CBspheres"], SPP_CPU))
    assert c["scale"] < CORNELL_SCALE[0] - 0.02, c["scale"]
    ceil = [v for r, v in c["rel"].items() if c["role"][r] == rr.CEILING]
    assert len(ceil) == 1 and ceil[0].mean() <= 0.97, ceil


def test_exact_light_pdf_does_not_match(fixture):
    """The discriminating check: the solid-angle pdf leaves the distance in
    the ratio (the reference's pdf is light.cpp:81-92's)."""
    c = rr.compare(fixture["CBbunny"], oracle_frame("CBbunny", fixture["CBbunny"], SPP_CPU,
                                                    flags=ptrace.PT_FLAG_EXACT_LIGHT_PDF | CORNELL_FLAGS))
    sides = [mx for r, (nf, mx) in c["spread"].items() if c["role"][r] == rr.SIDE]
    assert len(sides) == 2 and min(sides) >= 1.3, sides


@pytest.mark.parametrize("name", rr.EXACT)
def test_oracle_reproduces_reference_render(fixture, name):
    """No free factor: the oracle's frame is the reference's render."""
    check_exact(rr.compare(fixture[name], oracle_frame(name, fixture[name], SPP_EXACT), scale=1.0))


def test_course_default_albedo_is_what_plane_png_shows(fixture):
    """This repository's default BSDF (albedo 1, mesh.cpp:37) renders plane4
    at exactly twice the reference's radiance: the render is the course
    build's, whose default was 0.5 (mesh.cpp:36)."""
    d = ptrace.ArrayScene.load(ROOT / "tests" / "golden" / "scenes" / "plane4.npz").desc()
    d.camera = ptrace.pt_camera.from_buffer_copy(fixture["plane4"]["camera"].tobytes())
    img, _ = pyoracle.image(d, rr.W, rr.H, 4, max_bounces=8)
    c = rr.compare(fixture["plane4"], img, scale=1.0)
    for v in c["rel"].values():
        assert np.all(np.abs(v - 0.5) <= 0.005), v
