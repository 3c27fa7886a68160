"""Write a synthetic scene's triangle mesh and first area light in the layout tools/bvh_sim.cpp and
tools/bvh_quality.cpp read: u32 nv, u32 nt, float32 [nv][3] vertices, u32 [nt][3] indices, float32 [9]
light anchor | v1 | v2.  Design-tool input only (scratch/, not shipped).
    python tools/dump_scene_bin.py SyntheticHall scratch/hall.bin"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oppositerenderer_amd import scenes  # noqa: E402


def main():
    name, out = sys.argv[1], sys.argv[2]
    sc = scenes.scene_by_name(name)
    area = [l for l in sc.lights if np.any(np.asarray(l.v1) != 0)]
    L = area[0]
    with open(out, "wb") as f:
        np.array([len(sc.vertices), len(sc.triangles)], np.uint32).tofile(f)
        np.ascontiguousarray(sc.vertices, np.float32).tofile(f)
        np.ascontiguousarray(sc.triangles, np.uint32).tofile(f)
        np.concatenate([L.position, L.v1, L.v2]).astype(np.float32).tofile(f)
    print(name, len(sc.vertices), len(sc.triangles), "lights", len(sc.lights))


if __name__ == "__main__":
    main()
