"""The wide global-memory walk (pt_wide.h) on the GPU, bit-exact.

Every global-memory scene of the suite takes the wide walk by default (nested trees inside
the scene guard); these cases pin it directly: wide on / off (tuning key 16) give the same
bits and the oracle's on the C3 / C4 stand-ins and the reference's own drift / p scenes, in
every instantiation (frame-split and register mode, raysPerPixel > 1, the progressive graph),
on a far-translated scene (large margins), and a tree that is not nested falls back to the
binary walk.  tests/test_wide_walk.py checks the per-lane functions on the CPU.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import pt_host as H
from test_gpu_parity import assert_bitwise

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def scenes(tmp_path_factory):
    import pt_scenes
    d = str(tmp_path_factory.mktemp("wide"))
    z = np.load(os.path.join(GOLDEN, "ref_scenes.npz"))
    out = {k: H.scene_from_arrays(z[k + "_tris"], z[k + "_mats"]) for k in ("drift", "p")}
    out["bunny"] = H.setupBuffers(*pt_scenes.write_scene("bunny", d))
    out["sponza"] = H.setupBuffers(*pt_scenes.write_scene("sponza", d))
    return out


def render(sc, W, Hh, frames, wide=True, variant=0, frame_first=1, rpp=1, group=None, graph=False, mb=8):
    pt = H.PathTracer(W, Hh, max_bounce=mb, rays_per_pixel=rpp)
    pt.set_kernel(variant)
    pt.set_key(16, 0 if wide else 1)
    if group:
        pt.set_key(5, group)
    pt.upload(sc)
    if graph:
        pt.progressive_setup(frames_per_launch=frames // 2, launches_per_replay=2)
        pt.progressive_run(replays=1)
    else:
        pt.render(frame_first, frames, 0)
    img = pt.read_rgba32f()
    pt.close()
    return img


@pytest.mark.parametrize("name", ["bunny", "sponza", "drift", "p"])
def test_wide_equals_binary_and_oracle(scenes, name):
    sc = scenes[name]
    W, Hh = 160, 120
    a = render(sc, W, Hh, 4, wide=True)
    b = render(sc, W, Hh, 4, wide=False)
    assert_bitwise(a, b, "%s: wide vs binary walk" % name)
    rng = np.random.default_rng(7)
    xs, ys = rng.integers(0, W, 1500), rng.integers(0, Hh, 1500)
    want = O.render_pixels(sc, W, Hh, xs, ys, max_bounce=8, n_frames=4)
    assert_bitwise(a[ys, xs], want, "%s: wide vs oracle" % name)


def test_wide_instantiations(scenes):
    """Register mode (one item per pixel: key 5 = n_frames), raysPerPixel 3, the progressive
    graph, and a frame offset past the seed's signed-overflow frame."""
    sc = scenes["bunny"]
    W, Hh = 96, 64
    rng = np.random.default_rng(9)
    xs, ys = rng.integers(0, W, 800), rng.integers(0, Hh, 800)
    reg = render(sc, W, Hh, 4, group=4)
    assert_bitwise(reg[ys, xs], O.render_pixels(sc, W, Hh, xs, ys, max_bounce=8, n_frames=4), "register mode")
    multi = render(sc, W, Hh, 2, rpp=3)
    assert_bitwise(multi[ys, xs], O.render_pixels(sc, W, Hh, xs, ys, max_bounce=8, n_frames=2, rpp=3), "rpp 3")
    gr = render(sc, W, Hh, 4, graph=True)
    assert_bitwise(gr, render(sc, W, Hh, 4, wide=False), "graph replay")
    late = render(sc, W, Hh, 3, frame_first=3000)
    assert_bitwise(late[ys, xs], O.render_pixels(sc, W, Hh, xs, ys, max_bounce=8, frame_first=3000, n_frames=3),
                   "frames 3000..3002")


def test_wide_far_scene_and_small_scenes_forced_global():
    """Small soups forced to the global walk (variant 3), near the origin and 3,000 units away
    (the margins grow with |o| and the scene's extent), against the oracle in full."""
    import fuzz_scenes
    for seed, far in ((11, False), (12, True), (13, True), (14, False)):
        sc, _ = fuzz_scenes.random_case(seed, n_tris=700, far=far)
        W, Hh = 48, 36
        got = render(sc, W, Hh, 2, variant=3)
        want = O.render(sc, W, Hh, max_bounce=8, n_frames=2)
        assert_bitwise(got, want, "seed %d far %s" % (seed, far))


def test_not_nested_tree_falls_back(scenes):
    """A tree whose root box no longer contains a child fails pt_bvh_culling_ok: no wide tree
    is built and the global walk is the binary one (same image as the oracle)."""
    sc = dict(scenes["p"])
    nodes = np.array(sc["nodes"], np.float32)
    child = int(nodes[0, 10])
    nodes[child, 0] = nodes[0, 0] - 1.0          # the left child pokes out of the root box
    assert not H.bvh_culling_ok(nodes)
    sc["nodes"] = nodes
    W, Hh = 64, 48
    got = render(sc, W, Hh, 2)
    want = O.render(sc, W, Hh, max_bounce=8, n_frames=2)
    assert_bitwise(got, want, "non-nested tree")


def test_wide_key_validation(cornell_scene):
    pt = H.PathTracer(8, 8)
    with pytest.raises(H.PTError):
        pt.set_key(16, 2)
    pt.set_key(16, 1)
    pt.set_key(16, 0)
    pt.close()


def test_orphan_leaf_node_is_skipped(cornell_scene):
    """A leaf record no link from the root reaches (appended to a nested tree) is accepted by
    pt_upload_scene (links are checked on every node, cycles from the root).  The wide tree
    gives it no index, and the upload must not place its triangles (it used to write before the
    wide triangle array); the image is the oracle's, on the wide global walk (variant 3)."""
    sc = dict(cornell_scene)
    nodes = np.asarray(sc["nodes"], np.float32).reshape(-1, 12)
    leaf = next(i for i in range(len(nodes)) if nodes[i, 8] > -1.0)
    orphan = nodes[leaf].copy()
    orphan[10] = orphan[11] = -1.0
    sc["nodes"] = np.concatenate([nodes, orphan[None]], axis=0)
    W, Hh = 96, 72
    want = O.render(cornell_scene, W, Hh, max_bounce=8, n_frames=3)
    for variant in (3, 0):
        got = render(sc, W, Hh, 3, variant=variant)
        assert_bitwise(got, want, "orphan leaf, variant %d" % variant)


def test_leaf_certificate_gate_and_key19(scenes, cornell_scene):
    """The leaf re-test certificate stands on every leaf box containing its
    triangles' vertices (checked at upload).  A nested tree with leaf boxes shrunk so that they
    exclude part of their triangles still takes the wide walk, but must keep the exact re-test
    everywhere: the reference tests those leaves against the shrunk boxes, and the image is the
    oracle's.  And tuning key 19 (certificate off) never changes the image."""
    for name, sc0, variant, n_shrunk in (("cornell", cornell_scene, 3, 8), ("p", scenes["p"], 0, None)):
        sc = dict(sc0)
        nodes = np.array(sc["nodes"], np.float32).reshape(-1, 12)
        leaves = [i for i in range(len(nodes)) if nodes[i, 8] > -1.0]
        ext = lambda i: float(np.prod(np.maximum(nodes[i, 4:7] - nodes[i, 0:3], 1e-3)))
        for i in sorted(leaves, key=ext, reverse=True)[:n_shrunk]:   # the largest (Cornell) or all (p)
            ax = int(np.argmax(nodes[i, 4:7] - nodes[i, 0:3]))
            nodes[i, 4 + ax] = np.float32(0.5 * (nodes[i, ax] + nodes[i, 4 + ax]))   # max shrinks to the middle
        assert H.bvh_culling_ok(nodes)                           # still nested: the wide walk runs
        sc["nodes"] = nodes
        W, Hh = 64, 48
        got = render(sc, W, Hh, 3, variant=variant)
        want = O.render(sc, W, Hh, max_bounce=8, n_frames=3)
        assert_bitwise(got, want, "%s: shrunk leaf boxes" % name)
        assert not np.array_equal(want, O.render(sc0, W, Hh, max_bounce=8, n_frames=3)), \
            "%s: the shrunk boxes must change the reference's image (else the test tests nothing)" % name
    sc = scenes["bunny"]
    W, Hh = 96, 64
    imgs = []
    for k19 in (0, 1):
        pt = H.PathTracer(W, Hh, max_bounce=8)
        pt.set_key(19, k19)
        pt.upload(sc)
        pt.render(1, 4, 0)
        imgs.append(pt.read_rgba32f())
        pt.close()
    assert_bitwise(imgs[0], imgs[1], "key 19 = 0 vs 1")
