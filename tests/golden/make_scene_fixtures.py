"""Generate the flattened-scene fixtures the GPU box uses (it has no /root/reference).

Run in the build container:  python tests/golden/make_scene_fixtures.py
For every Cornell-box scene of media/pathtracer it loads the COLLADA file with
the product's scene adapter (pt_scene_load_dae: restated COLLADA parse,
halfedge normals, reference BVH, 4-wide compaction) and stores the exact
pt_scene_desc arrays the kernels consume, plus the reference-layout level
profile.  The .dae inputs themselves are not copied.
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "cuda-raytracer_amd"))
import ptrace  # noqa: E402

MEDIA = Path("/root/reference/media/pathtracer")
SCENES = {
    "CBempty": "advanced/CBempty.dae",
    "CBspheres": "advanced/CBspheres.dae",
    "CBspheres_lambertian": "advanced/CBspheres_lambertian.dae",
    "CBgems": "advanced/CBgems.dae",
    "CBcoil": "advanced/CBcoil.dae",
    "CBbunny": "advanced/CBbunny.dae",
    # the Stanford bunny alone (33,696 triangles, no light): its level 6 holds
    # 1,167 nodes, the level that overflows the reference's fixed per-level
    # buffers (BASELINE config 4)
    "bunny": "advanced/bunny.dae",
    # basic/ scenes whose reference renders the tests compare against
    # (tests/refrender.py): point lights, an area light, material-less meshes
    "trigs1": "basic/trigs1.dae",
    "trigs5": "basic/trigs5.dae",
    "trigs10": "basic/trigs10.dae",
    "plane4": "basic/plane4.dae",
    "floating": "basic/floating.dae",
    # directional + ambient (hemisphere) lights, spheres (the extended light model)
    "sphere_diffuse": "basic/sphere_diffuse.dae",
    "sphere7_diffuse": "basic/sphere7_diffuse.dae",
    "carim_diffuse": "basic/carim_diffuse.dae",
}


def main():
    out = Path(__file__).resolve().parent / "scenes"
    out.mkdir(exist_ok=True)
    only = set(sys.argv[1:])
    for name, rel in SCENES.items():
        if only and name not in only:
            continue
        sc = ptrace.Scene.load_dae(MEDIA / rel)
        arr = ptrace.scene_to_arrays(sc)
        arr["level_counts"] = np.array(sc.level_counts(), dtype=np.int32)
        arr["sorted_to_input"] = sc.sorted_to_input()
        np.savez_compressed(out / f"{name}.npz", **arr)
        print(name, {k: v.shape for k, v in arr.items()})


if __name__ == "__main__":
    main()
