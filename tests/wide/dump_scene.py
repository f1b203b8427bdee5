"""TEST INFRASTRUCTURE: writes a scene in wide_sim's input format (tests/wide/wide_sim.cpp)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "opengl-path-tracing_amd"))


def write_bin(path, sb):
    with open(path, "wb") as f:
        np.array([len(sb["tris"]), len(sb["nodes"]), len(sb["spheres"])], np.int32).tofile(f)
        for k in ("tris", "nodes", "spheres", "cam"):
            np.ascontiguousarray(sb[k], np.float32).tofile(f)


def dump(scene, path, tris=0):
    import pt_host
    import pt_scenes
    kw = {"target_tris": tris} if tris else {}
    obj, mtl = pt_scenes.write_scene(scene, os.path.join(REPO, "scenes"), **kw)
    write_bin(path, pt_host.setupBuffers(obj, mtl))


if __name__ == "__main__":
    dump(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 0)
