"""CMU462::Camera on the Scotty3D surface (scotty/scotty_pt.h, C entry points
scotty_generate_rays / scotty_camera_place): host code, no GPU.

generate_ray(x, y) (camera.h:71-81; a stub in the reference, camera.cpp:111-117)
must give the ray the kernels trace for that sensor point: the oracle's camera
ray (oracle/ptoracle.c camera_dir, cu:338-354), which the GPU matches bit for bit
in every image parity test.  The surface works in double, the kernels in fp32:
directions agree within 4e-7 (a few fp32 ulps), origins exactly.  The Scotty3D
framing (configure + place, camera.cpp:15-46, 86-108) is checked against its
defining properties."""
import math

import numpy as np
import pytest

import ptrace
import pyoracle
from conftest import load_fixture

DIR_TOL = 4e-7  # fp64 surface vs fp32 kernels (stated tolerance)


@pytest.mark.parametrize("name", ["CBempty", "CBbunny", "CBspheres", "CBgems"])
@pytest.mark.parametrize("flags", [0, ptrace.PT_FLAG_REF_ARITH])
def test_generate_ray_matches_oracle_camera(name, flags):
    d = load_fixture(name).desc()
    W, H = 320, 240
    rng = np.random.default_rng(7)
    # sensor points: pixel (row, col) + jitter, as the kernels sample them
    ss = rng.random((400, 2), dtype=np.float32) * np.array([H, W], np.float32)
    ss[:4] = [[0, 0], [H - 1e-3, W - 1e-3], [H / 2, W / 2], [0, W / 2]]
    ss = ss.astype(np.float32)
    xy = np.stack([ss[:, 1].astype(np.float64) / W, ss[:, 0].astype(np.float64) / H], axis=1)
    got = ptrace.scotty_generate_rays(d.camera, xy)
    for i in range(len(ss)):
        ref = pyoracle.camera_ray(d.camera, W, H, ss[i, 0], ss[i, 1], flags).astype(np.float64)
        assert np.array_equal(got[i, :3], ref[:3])
        rd = ref[3:] / np.linalg.norm(ref[3:])  # (REF_ARITH leaves the direction unnormalised, cu:354)
        assert np.abs(got[i, 3:] - rd).max() < DIR_TOL, (i, got[i, 3:], rd)
        assert abs(np.linalg.norm(got[i, 3:]) - 1.0) < 1e-12


def test_generate_ray_centre_is_look_at():
    d = load_fixture("CBbunny").desc()
    r = ptrace.scotty_generate_rays(d.camera, [[0.5, 0.5]])[0]
    look = np.array(d.camera.look_at, np.float64)
    assert np.allclose(r[3:], look / np.linalg.norm(look), atol=1e-15)


@pytest.mark.parametrize("w,h", [(640, 480), (480, 640), (256, 256)])
def test_configure_place_framing(w, h):
    """configure fits the fields of view to the screen's aspect (camera.cpp:
    21-31); place puts the camera at target + r (sin phi sin theta, cos phi,
    sin phi cos theta) (camera.cpp:86-96); generate_ray(0.5, 0.5) looks at the
    target, the sensor edges lie hFov / vFov apart, y is up."""
    hfov, vfov = 49.13434, 29.0
    target = np.array([0.1, 0.75, -0.2])
    phi, theta, r = 1.2, 0.4, 4.5
    xy = [[0.5, 0.5], [0.0, 0.5], [1.0, 0.5], [0.5, 0.0], [0.5, 1.0]]
    cam, rays, (hf, vf) = ptrace.scotty_camera_place(hfov, vfov, w, h, target, phi, theta, r, 0.1, 100.0, xy)
    ar = w / h
    ar1 = math.tan(math.radians(hfov) / 2) / math.tan(math.radians(vfov) / 2)
    if ar1 < ar:
        assert abs(math.tan(math.radians(hf) / 2) - math.tan(math.radians(vfov) / 2) * ar) < 1e-12 and vf == vfov
    else:
        assert abs(math.tan(math.radians(vf) / 2) - math.tan(math.radians(hfov) / 2) / ar) < 1e-12 and hf == hfov
    pos = target + r * np.array([math.sin(phi) * math.sin(theta), math.cos(phi), math.sin(phi) * math.cos(theta)])
    assert np.allclose(rays[:, :3], pos, atol=1e-12)
    assert np.allclose(np.array(cam.origin, np.float64), pos, atol=1e-6)
    to_target = (target - pos) / np.linalg.norm(target - pos)
    assert np.allclose(rays[0, 3:], to_target, atol=1e-12)
    ang = lambda a, b: math.degrees(math.acos(min(1.0, float(a @ b))))
    assert abs(ang(rays[1, 3:], rays[2, 3:]) - hf) < 1e-9
    assert abs(ang(rays[3, 3:], rays[4, 3:]) - vf) < 1e-9
    # y = 1 is the top of the sensor: its ray climbs relative to the centre ray
    assert rays[4, 4] > rays[0, 4] > rays[3, 4]
    # the pt_camera handed to the kernels spans the same rays
    again = ptrace.scotty_generate_rays(cam, xy)
    assert np.abs(again[:, 3:] - rays[:, 3:]).max() < 1e-6


def test_place_clamps_radius():
    _, rays, _ = ptrace.scotty_camera_place(50, 35, 64, 64, [0, 0, 0], 1.0, 0.0, 1000.0, 0.5, 10.0, [[0.5, 0.5]])
    assert abs(np.linalg.norm(rays[0, :3]) - 10.0) < 1e-12
