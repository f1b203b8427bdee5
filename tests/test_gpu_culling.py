"""The culling walk: the LDS walk tests nodes with a conservative slab test
and re-tests a leaf's own box exactly before one of its triangles may move t.  On a tree that
qualifies (a full binary tree threaded in preorder whose internal boxes contain their
children's) the image is the reference's bit for bit; any other tree walks with the exact test.

Tolerance: NONE -- uint32 bit patterns, as every parity test.
"""
import numpy as np
import pytest

import oracle_lib as O
import pt_host as H

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def render(sc, W, Hh, n_frames, frame_first=1, culling=True, max_bounce=8, variant=0):
    pt = H.PathTracer(W, Hh, max_bounce=max_bounce)
    pt.set_kernel(variant)
    pt.set_culling(culling)
    pt.upload(sc)
    active = pt.diag()["culling_walk"]
    pt.render(frame_first, n_frames, 0)
    img = pt.read_rgba32f()
    pt.close()
    return img, active


def check(sc, label, W=64, Hh=48, n_frames=6, frame_first=1, expect_active=True):
    want = O.render(sc, W, Hh, max_bounce=8, frame_first=frame_first, n_frames=n_frames)
    for culling in (True, False):
        got, active = render(sc, W, Hh, n_frames, frame_first, culling)
        assert active == (culling and expect_active), (label, culling, active)
        bad = int(np.count_nonzero(bits(got) != bits(want)))
        assert bad == 0, "%s (culling %s): %d words differ" % (label, culling, bad)


def preorder_depths(nodes):
    """Depth of every node of a preorder-threaded tree (hit link = left child, the left
    child's miss link = the right child)."""
    depth = np.zeros(len(nodes), np.int64)
    st = [(0, 0)]
    while st:
        x, dd = st.pop()
        depth[x] = dd
        if nodes[x, 8] <= -1.0:            # internal
            left = int(nodes[x, 10])
            right = int(nodes[left, 11])
            st += [(left, dd + 1), (right, dd + 1)]
    return depth


def test_culling_on_benchmark_and_reference_scenes(cornell_scene, ship_scene):
    check(cornell_scene, "cornell")
    check(cornell_scene, "cornell, frames 3001..3006", frame_first=3001)
    check(ship_scene, "ship")


def test_culling_mid_size_lds_scene(tmp_path):
    """A scene past the padded walk image (run-time plane stride)."""
    import pt_scenes
    sc = H.setupBuffers(*pt_scenes.write_scene("bunny", str(tmp_path), target_tris=80))
    check(sc, "80-triangle LDS scene", n_frames=4)


def test_loose_nested_boxes(cornell_scene):
    """Boxes grown by an amount that shrinks with depth: still nested, no longer tight."""
    sc = dict(cornell_scene)
    nodes = np.array(sc["nodes"], np.float32)
    depth = preorder_depths(nodes)
    grow = (0.01 * (depth.max() + 1 - depth)).astype(np.float32)[:, None]
    nodes[:, 0:3] -= grow
    nodes[:, 4:7] += grow
    sc["nodes"] = nodes
    check(sc, "loose boxes")


def test_not_nested_falls_back_to_exact(cornell_scene):
    """A root box that no longer contains a child: the tree does not qualify, the walk uses
    the exact test, and the image is still the reference's."""
    sc = dict(cornell_scene)
    nodes = np.array(sc["nodes"], np.float32)
    left = int(nodes[0, 10])
    nodes[0, 0] = np.float32(nodes[left, 0] + 0.25)    # the root's min.x inside its child's box
    sc["nodes"] = nodes
    check(sc, "not nested", expect_active=False)


def test_far_from_origin(cornell_scene):
    """Scene and camera translated far from the origin: |o| and the culling margins are large
    against the box gaps."""
    sc = dict(cornell_scene)
    off = np.array([1000.0, -3000.0, 500.0], np.float32)
    tris = np.array(sc["tris"], np.float32)
    for v in (0, 4, 8):
        tris[:, v:v + 3] += off
    nodes = np.array(sc["nodes"], np.float32)
    nodes[:, 0:3] += off
    nodes[:, 4:7] += off
    sph = np.array(sc["spheres"], np.float32).reshape(-1, 8)
    sph[:, 0:3] += off
    cam = np.array(sc["cam"], np.float32).reshape(12)
    cam[0:3] += off
    sc.update(tris=tris, nodes=nodes, spheres=sph, cam=cam)
    check(sc, "translated scene")


@pytest.mark.parametrize("variant", [3])
def test_global_walk_ignores_the_setting(cornell_scene, variant):
    """Only the LDS walk culls; the global-memory walk (variant 3) is unchanged by key 15."""
    want = O.render(cornell_scene, 40, 24, max_bounce=8, n_frames=3)
    for culling in (True, False):
        got, _ = render(cornell_scene, 40, 24, 3, culling=culling, variant=variant)
        assert np.array_equal(bits(got), bits(want)), (variant, culling)


def test_culling_key_validation_and_graph(cornell_scene):
    """Tuning key 15 accepts 0 / 1 only; switching it drops a captured progressive graph
    (the graph bakes the walk in), and the recaptured loop is the reference's image either
    way."""
    want = O.render(cornell_scene, 40, 24, max_bounce=8, n_frames=8)
    pt = H.PathTracer(40, 24, max_bounce=8)
    try:
        pt.upload(cornell_scene)
        with pytest.raises(H.PTError):
            pt.set_key(15, 2)
        pt.progressive_setup(4, 2)
        pt.progressive_run(1)
        assert np.array_equal(bits(pt.read_rgba32f()), bits(want))
        pt.set_culling(False)
        with pytest.raises(H.PTError) as e:
            pt.progressive_run(1)
        assert e.value.code == -6     # PT_E_STATE: set up again first
        pt.progressive_setup(4, 2)
        pt.progressive_reset(1)
        pt.progressive_run(1)
        assert np.array_equal(bits(pt.read_rgba32f()), bits(want))
        assert not pt.diag()["culling_walk"]
    finally:
        pt.close()


def blocks_per_cu(lds, mw):
    return min(mw, 160 * 1024 // lds) if lds else mw


def test_sink_image_never_costs_a_workgroup(cornell_scene, tmp_path):
    """The sink image adds 32 B per node to the LDS copy; the walk culls only while that
    leaves the resident workgroups per CU unchanged at the set waves per SIMD (key 3).  Scan
    scene sizes for one the rule turns off, and render it exactly either way."""
    import pt_scenes
    pt = H.PathTracer(48, 32, max_bounce=8)
    found, seen = None, []
    try:
        for target in range(2, 120, 2):
            sc = H.setupBuffers(*pt_scenes.write_scene("bunny", str(tmp_path / str(target)), target_tris=target))
            pt.upload(sc)
            d = pt.diag()
            seen.append((target, len(sc["tris"]) // 16 if np.ndim(sc["tris"]) == 1 else len(sc["tris"]),
                         d["lds_bytes"], d["lds_bytes_sinks"]))
            if d["lds_bytes_sinks"] == 0 or d["lds_bytes"] > 48 * 1024:
                continue
            for ws in (0, 5, 6, 7, 8):
                pt.set_key(3, ws)
                mw = ws or 7
                want_on = blocks_per_cu(d["lds_bytes_sinks"], mw) >= blocks_per_cu(d["lds_bytes"], mw)
                assert pt.diag()["culling_walk"] == want_on, (target, ws, d)
                if not want_on and found is None:
                    found = (sc, ws)
            pt.set_key(3, 0)
            if d["lds_bytes"] > 48 * 1024:
                break
    finally:
        pt.close()
    assert found is not None, "no scene size in the scan hits the occupancy rule: %s" % seen
    sc, ws = found
    want = O.render(sc, 32, 24, max_bounce=8, n_frames=3)
    pt = H.PathTracer(32, 24, max_bounce=8)
    try:
        pt.set_key(3, ws)
        pt.upload(sc)
        assert not pt.diag()["culling_walk"]
        pt.render(1, 3, 0)
        assert np.array_equal(bits(pt.read_rgba32f()), bits(want))
    finally:
        pt.close()


@pytest.mark.parametrize("target", [200, 380])
def test_wide_workgroup_lds_scenes(tmp_path, target):
    """Scenes past the 256-thread workgroups' LDS budget (48 KiB) are staged once per 768- or
    1024-thread workgroup (lds_threads); culling on and off, the reference's image."""
    import pt_scenes
    sc = H.setupBuffers(*pt_scenes.write_scene("bunny", str(tmp_path), target_tris=target))
    pt = H.PathTracer(16, 16, max_bounce=8)
    try:
        pt.upload(sc)
        d = pt.diag()
    finally:
        pt.close()
    assert 48 * 1024 < d["lds_bytes"] <= 152 * 1024, d
    on = blocks_per_cu(d["lds_bytes_sinks"], 7) >= blocks_per_cu(d["lds_bytes"], 7)
    check(sc, "%d-triangle wide-workgroup scene" % target, n_frames=3, expect_active=on)
