"""The Scotty3D surface on the GPU (scotty/scotty_pt.h through
scotty/scotty_capi.cpp): CMU462::PathTracer's tile queue and worker threads
over the GPU estimator (pathtracer.cpp:183-213, 499-558), and the progressive
viewer loop of display.cpp:99-190 with CudaRenderer::renderAccumulate /
setViewpoint (cu:1845-1870, 2419-2457).  Both must give exactly the frames the
C ABI gives for the same work, and those equal the CPU oracle's frames."""
import numpy as np
import pytest

import ptrace
import pyoracle
from conftest import load_fixture

pytestmark = pytest.mark.gpu
W, H = 64, 48


@pytest.mark.parametrize("threads", [1, 5])
def test_pathtracer_surface_matches_c_abi(gpu_ctx, threads):
    scene = load_fixture("CBgems")
    img = ptrace.scotty_render(scene, W, H, 4, 4, threads=threads)
    gpu_ctx.load_scene(scene)
    gpu_ctx.clear()
    gpu_ctx.render(W, H, 4, max_bounces=4)
    ref = gpu_ctx.get_image()
    assert np.array_equal(img, ref)
    assert img[..., :3].mean() > 0
    # and the frame is the oracle's (not only the C ABI's)
    o, _ = pyoracle.image(scene.desc(), W, H, 4, max_bounces=4)
    assert np.array_equal(img, o)


def _moved(cam, dx, dz):
    c = ptrace.pt_camera()
    for k in range(3):
        c.origin[k], c.look_at[k], c.left[k], c.up[k] = cam.origin[k], cam.look_at[k], cam.left[k], cam.up[k]
    # Vector3D (double) origin += (dx, 0, dz), then v2f3 (cu:1847)
    c.origin[0] = float(np.float32(np.float64(cam.origin[0]) + dx))
    c.origin[2] = float(np.float32(np.float64(cam.origin[2]) + dz))
    return c


@pytest.mark.parametrize("keys,frames_after_move,dx,dz", [
    ("...", 3, 0.0, 0.0),          # three progressive frames, no key
    ("..d..", 3, 0.01, 0.0),       # 'd' moves the camera +x and restarts the accumulation
    (".w.a.", 2, -0.01, -0.01),    # two moves: origin (-0.01, 0, -0.01)
])
def test_viewer_loop_matches_progressive_render(gpu_ctx, keys, frames_after_move, dx, dz):
    scene = load_fixture("CBgems")
    spf = 2
    img, n = ptrace.scotty_viewer(scene, W, H, spf, keys, max_bounces=2)
    assert n == spf * frames_after_move
    gpu_ctx.load_scene(scene)
    gpu_ctx.set_camera(_moved(scene.desc().camera, dx, dz))
    for f in range(frames_after_move):
        gpu_ctx.render(W, H, spf, max_bounces=2, sample_offset=f * spf)
    ref = gpu_ctx.get_display_image()  # median filtered below 32 samples, like getImage
    assert np.array_equal(img, ref)
    # the oracle's frame from the moved camera: the progressive frames sum the
    # samples in order, as one render of all of them does
    d = scene.desc()
    d.camera = _moved(d.camera, dx, dz)
    o, _ = pyoracle.image(d, W, H, spf * frames_after_move, max_bounces=2)
    assert np.array_equal(img, pyoracle.median(o))


def test_viewer_pause():
    """'p' toggles pauseSim, which display.cpp's renderPicture never reads
    (display.cpp:145-174 clears the update flag and renders regardless): every
    displayed frame renders samples_per_frame more samples, paused or not, and
    the frames equal those of a loop without the key."""
    scene = load_fixture("CBgems")
    img_p, n = ptrace.scotty_viewer(scene, W, H, 2, "..p..")
    assert n == 2 * 5
    img, n2 = ptrace.scotty_viewer(scene, W, H, 2, ".....")
    assert n2 == n and np.array_equal(img_p, img)
    _, n = ptrace.scotty_viewer(scene, W, H, 2, ".p.p.")
    assert n == 2 * 5
