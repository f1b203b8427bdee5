"""Regenerates the committed fixtures in tests/golden/ (run in the dev container).

ship_scene.npz     : the reference's scene_data/ship{obj,mtl}.txt as loaded by the product
                     loader (pt_scene_load_obj) -- loader parity vs the oracle's istream
                     restatement is tested on CPU where /root/reference exists; the GPU box
                     has no /root/reference, so the loaded arrays travel as data.
ref_scenes.npz     : the reference's scene_data/drift*, p* and p2* scenes (11,846 / 6,258 / 6,258
                     triangles, the inputs that take the global-memory walk), loaded the same way
                     and checked against the oracle's loader; keys <scene>_tris / <scene>_mats.
python tests/golden/make_golden.py [ref|images|all]   (default all)
golden_images.npz  : small RGBA32F renders, each produced by the C++ oracle AND the
                     independent numpy twin and written only if the two agree bit for bit.
                     Keys: <scene>_<W>_<H>_<max_bounce>_<mode>_<spp>.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), os.path.join(REPO, "opengl-path-tracing_amd")]

import numpy_twin  # noqa: E402
import oracle_lib  # noqa: E402
import pt_host  # noqa: E402
import pt_scenes  # noqa: E402

REF = "/root/reference/LearnOpenGL/scene_data"

CASES = [
    ("cornell", 64, 48, 5, 1, 1), ("cornell", 64, 48, 5, 1, 4), ("cornell", 64, 48, 8, 1, 16),
    ("cornell", 64, 48, 5, 2, 1), ("cornell", 64, 48, 5, 3, 1), ("cornell", 64, 48, 5, 4, 1),
    ("ship", 64, 48, 5, 1, 4), ("ship", 64, 48, 5, 2, 1),
]


def main(part="all"):
    if os.path.isdir(REF) and part in ("all", "ref"):
        t, m = pt_host.load_vertex_data(os.path.join(REF, "shipobj.txt"), os.path.join(REF, "shipmtl.txt"))
        to, mo = oracle_lib.load_obj(os.path.join(REF, "shipobj.txt"), os.path.join(REF, "shipmtl.txt"))
        assert np.array_equal(t.view(np.uint32), to.view(np.uint32)) and np.array_equal(m.view(np.uint32), mo.view(np.uint32))
        np.savez_compressed(os.path.join(HERE, "ship_scene.npz"), tris=t, mats=m)
        ref = {}
        for name in ("drift", "p", "p2"):
            obj, mtl = os.path.join(REF, name + "obj.txt"), os.path.join(REF, name + "mtl.txt")
            t, m = pt_host.load_vertex_data(obj, mtl)
            to, mo = oracle_lib.load_obj(obj, mtl)
            assert np.array_equal(t.view(np.uint32), to.view(np.uint32)) and np.array_equal(m.view(np.uint32), mo.view(np.uint32))
            ref[name + "_tris"], ref[name + "_mats"] = t, m
        np.savez_compressed(os.path.join(HERE, "ref_scenes.npz"), **ref)
    if part == "ref":
        return
    z = np.load(os.path.join(HERE, "ship_scene.npz"))
    scenes = {"cornell": pt_host.setupBuffers(*pt_scenes.write_scene("cornell", os.path.join(REPO, "scenes"))),
              "ship": pt_host.scene_from_arrays(z["tris"], z["mats"])}
    out = {}
    for scene, W, H, mb, mode, spp in CASES:
        a = oracle_lib.render(scenes[scene], W, H, max_bounce=mb, mode=mode, n_frames=spp)
        b = numpy_twin.render(scenes[scene], W, H, max_bounce=mb, mode=mode, n_frames=spp)
        assert np.array_equal(a.view(np.uint32), np.asarray(b, np.float32).view(np.uint32)), (scene, mode, spp)
        out["%s_%d_%d_%d_%d_%d" % (scene, W, H, mb, mode, spp)] = a
    np.savez_compressed(os.path.join(HERE, "golden_images.npz"), **out)
    print("wrote %d golden images" % len(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "all")
