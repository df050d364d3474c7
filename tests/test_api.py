"""C-ABI boundary: the library loads, exports every declared entry point and
reports errors through return codes (no GPU needed)."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

import ptrace
from conftest import ROOT, have_gpu


def test_header_symbols_exported():
    header = (ROOT / "include" / "pt_api.h").read_text()
    declared = set(re.findall(r"\b(pt_[a-z_]+)\s*\(", header))
    assert declared == set(ptrace.API_SYMBOLS)
    lib = C.CDLL(str(ptrace.LIB_PATH))
    for name in declared:
        assert hasattr(lib, name), name


def test_no_device_reports_error():
    if have_gpu():
        pytest.skip("GPU present")
    with pytest.raises(ptrace.PTError) as e:
        ptrace.Context(0)
    assert e.value.code in (ptrace.PT_E_NODEVICE, ptrace.PT_E_HIP)


def test_load_missing_file():
    with pytest.raises(ptrace.PTError) as e:
        ptrace.Scene.load_dae("/nonexistent/scene.dae")
    assert e.value.code == ptrace.PT_E_IO
    assert "could not open" in str(e.value)


def test_from_triangles_builds_bvh():
    rng = np.random.default_rng(3)
    tris = rng.random((500, 9), dtype=np.float32)
    sc = ptrace.Scene.from_triangles(tris)
    d = sc.desc()
    assert d.n_prims == 500
    assert d.n_levels >= 2
    perm = sc.sorted_to_input()
    assert sorted(perm.tolist()) == list(range(500))
    # every leaf range inside the primitive array; children breadth-first
    for i in range(d.n_nodes):
        nd = d.nodes[i]
        assert 0 <= nd.prim_start and nd.prim_start + nd.prim_count <= 500
        for c in nd.child:
            assert c == -1 or c > i


def test_scotty_surface_library_exports():
    """The Scotty3D surface's C entry points (scotty/scotty_capi.cpp) load;
    without a GPU they report the device error through the return code."""
    lib = ptrace._scotty()
    header = (ROOT / "include" / "scotty_capi.h").read_text()
    declared = set(re.findall(r"\b(scotty_[a-z_]+)\s*\(", header))
    assert {"scotty_render", "scotty_viewer", "scotty_generate_rays", "scotty_camera_place", "scotty_bvh_create",
            "scotty_bvh_intersect", "scotty_bvh_occluded", "scotty_bvh_destroy"} <= declared
    for name in declared:
        assert hasattr(lib, name), name
    if have_gpu():
        return
    with pytest.raises(ptrace.PTError) as e:
        ptrace.ScottyBVH(np.eye(3), np.eye(3), [[0, 1, 2]])
    assert e.value.code in (ptrace.PT_E_NODEVICE, ptrace.PT_E_HIP)
    scene = ptrace.ArrayScene.load(ROOT / "tests" / "golden" / "scenes" / "CBempty.npz")
    with pytest.raises(ptrace.PTError) as e:
        ptrace.scotty_render(scene, 8, 8, 1, 2, threads=2)
    assert e.value.code in (ptrace.PT_E_NODEVICE, ptrace.PT_E_HIP)
    with pytest.raises(ptrace.PTError):
        ptrace.scotty_viewer(scene, 8, 8, 1, "..")
