"""The single-leaf kernel's candidate clusters (DESIGN §4 "candidate
clusters"; k_path_leaf's PT_PATH_CLUSTER / PT_PATH_CLUSTER_OCC /
PT_PATH_OCC_AABB): a ray is tested only against the primitives whose cluster
box it enters (its segment's box, for a shadow ray).  The result must be the
full loop's, bit for bit, so these scenes put the cases that could tell them
apart into one leaf: exact ties (a triangle and its duplicate, paired into one
cluster, and a duplicated triangle in a cluster of its own), coplanar
neighbours, spheres among triangles (clusters of one), a cluster starting at
an odd primitive, grazing and box-edge rays -- rendered on the GPU and by the
oracle, compared bit for bit."""
import numpy as np
import pytest

import ptrace
import pyoracle




def _bsdf(kind, rgb, ior=1.5):
    b = ptrace.pt_bsdf()
    b.type = kind
    for k in range(3):
        b.albedo[k] = rgb[k]
        b.transmittance[k] = rgb[k]
    b.ior = ior
    return b


def _area_light(Le, position, dim_x, dim_y):
    L = ptrace.pt_light()
    L.type = ptrace.PT_LIGHT_AREA
    for k in range(3):
        L.radiance[k] = Le
        L.position[k] = position[k]
        L.direction[k] = (0.0, -1.0, 0.0)[k]
        L.dim_x[k] = dim_x[k]
        L.dim_y[k] = dim_y[k]
    L.area = float(np.linalg.norm(dim_x) * np.linalg.norm(dim_y))
    return L


def _camera(origin, look, left, up):
    c = ptrace.pt_camera()
    for k in range(3):
        c.origin[k], c.look_at[k], c.left[k], c.up[k] = origin[k], look[k], left[k], up[k]
    return c


def _quad(p, eu, ev):
    p, eu, ev = (np.asarray(x, np.float64) for x in (p, eu, ev))
    return [np.concatenate([p, p + eu, p + eu + ev]), np.concatenate([p, p + eu + ev, p + ev])]


def room_with_ties(spheres):
    """A Cornell-like room (5 walls of 2 triangles), the floor's triangles
    duplicated (an exact tie inside one cluster pair), the back wall's first
    triangle duplicated after a single sphere (a tie across clusters, the
    second starting at an odd index), a small coplanar patch on the left wall,
    the light quad's two triangles, optional spheres."""
    t = []
    t += _quad((-1, 0, 1), (2, 0, 0), (0, 0, -2)) * 2             # floor, twice: ties
    t += _quad((-1, 1.5, -1), (2, 0, 0), (0, 0, 2))               # ceiling
    back = _quad((-1, 0, -1), (2, 0, 0), (0, 1.5, 0))
    t += back
    t += _quad((-1, 0, 1), (0, 0, -2), (0, 1.5, 0))               # left wall
    t += _quad((-1, 0.4, 0.2), (0, 0, -0.3), (0, 0.3, 0))         # coplanar patch on it
    t += _quad((1, 0, -1), (0, 0, 2), (0, 1.5, 0))                # right wall
    t += [back[0]]                                                # back wall's first triangle again
    t += _quad((-0.3, 1.49, -0.2), (0.6, 0, 0), (0, 0, 0.4))      # light quad
    tris = np.array(t, np.float32)
    nb = len(tris)
    bsdfs = [_bsdf(ptrace.PT_BSDF_DIFFUSE, (0.7, 0.6, 0.5)), _bsdf(ptrace.PT_BSDF_DIFFUSE, (0.8, 0.1, 0.1)),
             _bsdf(ptrace.PT_BSDF_EMISSION, (4.0, 4.0, 4.0)), _bsdf(ptrace.PT_BSDF_MIRROR, (0.9, 0.9, 0.9)),
             _bsdf(ptrace.PT_BSDF_GLASS, (0.95, 0.95, 0.95))]
    tb = np.zeros(nb, np.int32)
    tb[10:14] = 1  # the left wall and its patch
    tb[-2:] = 2    # the light
    sph = sb = None
    if spheres:
        sph = np.array([[-0.4, 0.35, -0.3, 0.35], [0.45, 0.3, 0.2, 0.3]], np.float32)
        sb = np.array([3, 4], np.int32)
    light = _area_light(4.0, (0.0, 1.489, 0.0), (0.6, 0, 0), (0, 0, 0.4))
    cam = _camera((0, 0.75, 3.2), (0, 0, -1), (1, 0, 0), (0, 1, 0))
    return ptrace.Scene.from_mesh(tris, bsdfs, tri_bsdf=tb, spheres=sph, sphere_bsdf=sb, light=light, camera=cam)


def triangle_soup(seed, n):
    """n random triangles (some sharing an edge or a plane) and 3 spheres in
    a unit box, under a point light: one leaf of <= 32 primitives."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-1, 1, (n, 1, 3))
    tris = (c + 0.5 * rng.uniform(-1, 1, (n, 3, 3))).reshape(n, 9)
    tris[1, :3], tris[1, 3:6] = tris[0, :3], tris[0, 6:9]        # a shared edge
    tris[3] = tris[2][[3, 4, 5, 6, 7, 8, 0, 1, 2]]               # the same triangle, rotated vertices
    sph = np.array([[0.2, -0.1, 0.3, 0.25], [-0.5, 0.4, -0.2, 0.2], [0.6, 0.6, 0.6, 0.15]], np.float32)
    bsdfs = [_bsdf(ptrace.PT_BSDF_DIFFUSE, (0.7, 0.7, 0.7)), _bsdf(ptrace.PT_BSDF_MIRROR, (0.8, 0.8, 0.8))]
    L = ptrace.pt_light()
    L.type = ptrace.PT_LIGHT_POINT
    for k in range(3):
        L.radiance[k] = 3.0
        L.position[k] = (0.1, 1.6, 0.2)[k]
    cam = _camera((0.3, 0.2, 3.0), (0, 0, -1), (1, 0, 0), (0, 1, 0))
    return ptrace.Scene.from_mesh(tris.astype(np.float32), bsdfs, tri_bsdf=np.zeros(n, np.int32), spheres=sph,
                                  sphere_bsdf=np.array([0, 1, 0], np.int32), light=L, camera=cam)


SCENES = {"room": lambda: room_with_ties(False), "room_spheres": lambda: room_with_ties(True),
          "soup7": lambda: triangle_soup(7, 24), "soup8": lambda: triangle_soup(8, 29)}


def test_scenes_are_one_leaf():
    """(CPU) every scene here is a single-leaf tree: the clustered kernel path."""
    for name, make in SCENES.items():
        d = make().desc()
        assert d.nodes[0].prim_count == d.n_prims and d.n_prims <= 32, name


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCENES))
@pytest.mark.parametrize("flags", [0, ptrace.PT_FLAG_COSINE_DIFFUSE])
def test_clustered_render_bit_exact(gpu_ctx, name, flags):
    sc = SCENES[name]()
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    gpu_ctx.clear()
    gpu_ctx.render(64, 48, 4, max_bounces=8, seed=15618, flags=flags)
    g = gpu_ctx.get_image()
    o, _ = pyoracle.image(d, 64, 48, 4, max_bounces=8, seed=15618, flags=flags)
    assert o[..., :3].mean() > 1e-3
    diff = np.abs(g[..., :3] - o[..., :3])
    assert diff.max() == 0.0, (name, float(diff.max()), int((diff > 0).any(axis=-1).sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCENES) + ["CBempty", "CBspheres"])
def test_counting_build_same_frame_and_counts(gpu_ctx, name):
    """PT_FLAG_COUNT_TESTS (the bench's executed-work figures) runs the
    counting build of k_path_leaf: the frame is the timed build's bit for bit;
    every traced ray ran one box test per cluster (extension rays the slab
    test, shadow segments the overlap test), and no ray tested more
    primitives than the leaf holds."""
    from conftest import load_fixture
    sc = SCENES[name]() if name in SCENES else load_fixture(name)
    d = sc.desc()
    gpu_ctx.load_scene(sc)
    imgs, st = [], None
    for flags in (0, ptrace.PT_FLAG_COUNT_TESTS):
        gpu_ctx.reset_stats()
        gpu_ctx.clear()
        gpu_ctx.render(96, 64, 8, max_bounces=8, seed=15618, flags=flags)
        imgs.append(gpu_ctx.get_image())
        st = gpu_ctx.stats()
    assert np.array_equal(imgs[0], imgs[1])
    traced = st.rays - st.culled_rays
    assert traced > 0 and st.cluster_box_tests > 0
    nclus = st.cluster_box_tests // traced
    assert st.cluster_box_tests == nclus * traced and 1 <= nclus <= d.nodes[0].prim_count
    tests = st.prim_tests_tri + st.prim_tests_sph
    assert 0 < tests < d.nodes[0].prim_count * traced
    if name == "CBspheres":
        assert st.prim_tests_sph > 0
