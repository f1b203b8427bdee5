"""Host scene ingest: product loader / BVH builder vs the oracle's literal restatements.

Reference: geometry_loader.h:15-142 (load_vertex_data), bvh.h:84-268 (buildSAHTree,
find_split, build_links), ogl_path_trace.h:415-507 (built-ins).  Bit-exact on every array.
The reference's own scene files are used when /root/reference is mounted (dev container).
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import pt_host as H
import pt_scenes
from conftest import REF_SCENES

SHIPPED = {"ship": (2520, 6), "p": (6258, 11), "p2": (6258, 11), "drift": (11846, 24)}


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def same(a, b):
    return a.shape == b.shape and np.array_equal(bits(a), bits(b))


needs_ref = pytest.mark.skipif(not os.path.isdir(REF_SCENES), reason="reference scene_data not mounted")


@needs_ref
@pytest.mark.parametrize("name", sorted(SHIPPED))
def test_loader_matches_oracle_on_reference_scenes(name):
    obj, mtl = os.path.join(REF_SCENES, name + "obj.txt"), os.path.join(REF_SCENES, name + "mtl.txt")
    tp, mp = H.load_vertex_data(obj, mtl)
    to, mo = O.load_obj(obj, mtl)
    assert (len(tp), len(mp)) == SHIPPED[name]
    assert same(tp, to) and same(mp, mo)


@needs_ref
@pytest.mark.parametrize("name", ["ship", "p", "p2"])
def test_bvh_matches_oracle_on_reference_scenes(name):
    tp, _ = H.load_vertex_data(os.path.join(REF_SCENES, name + "obj.txt"), os.path.join(REF_SCENES, name + "mtl.txt"))
    assert same(H.buildSAHTree(tp), O.build_bvh(tp))


def test_ship_fixture_bvh(ship_scene):
    assert same(ship_scene["nodes"], O.build_bvh(ship_scene["tris"]))


def test_cornell_scene_counts(cornell_scene):
    assert len(cornell_scene["tris"]) == 36
    assert cornell_scene["n_loaded_mats"] == 6 and len(cornell_scene["mats"]) == 11
    assert len(cornell_scene["spheres"]) == 1
    s = cornell_scene["spheres"][0]
    assert list(s[:5]) == [-0.5, 3.0, 1.0, 0.8, 10.0]


def test_builtins_match_oracle(cornell_scene):
    bm, sph = O.builtins(cornell_scene["n_loaded_mats"])
    assert same(cornell_scene["mats"][-5:], bm) and same(cornell_scene["spheres"], sph)


def random_soup(n, seed, dup_frac=0.0, flat=False):
    rng = np.random.default_rng(seed)
    t = np.zeros((n, 16), np.float32)
    c = rng.random((n, 3)) * 10
    for v in range(3):
        p = c + rng.normal(0, 0.3, (n, 3))
        if flat:
            p[:, 2] = 1.0
        t[:, 4 * v: 4 * v + 3] = p
    t[:, 12] = rng.integers(0, 4, n)
    if dup_frac:
        k = int(n * dup_frac)
        src = rng.integers(0, n, k)
        dst = rng.integers(0, n, k)
        t[dst] = t[src]
    # quantise some coordinates so centroid ties happen
    t[: n // 3, :12] = np.round(t[: n // 3, :12])
    return t


@pytest.mark.parametrize("n,seed,dup,flat", [(3, 0, 0, False), (7, 1, 0, False), (100, 2, 0.2, False),
                                             (777, 3, 0.05, False), (2000, 4, 0, True), (5000, 5, 0.01, False)])
def test_bvh_matches_oracle_random(n, seed, dup, flat):
    t = random_soup(n, seed, dup, flat)
    assert same(H.buildSAHTree(t), O.build_bvh(t))


def test_bvh_degenerate_all_identical():
    t = np.tile(random_soup(1, 9), (9, 1))
    a, b = H.buildSAHTree(t), O.build_bvh(t)
    assert same(a, b)
    leaves = a[a[:, 8] > -1]
    assert np.all(leaves[:, 8] == 0) and np.all(leaves[:, 9] == 0)   # find() -> first equal


def check_threaded_bvh(nodes, tris):
    """verify_tree (bvh.h:112-170) + link-walk coverage: the all-hit walk visits every
    node exactly once in preorder; every leaf box contains its triangles."""
    n = len(nodes)
    seen = []
    i = 0
    while i > -1:
        seen.append(i)
        i = int(nodes[i, 10])
        assert len(seen) <= n
    assert sorted(seen) == list(range(n))
    assert int(nodes[0, 11]) == -1                      # all-miss walk from the root ends
    for k in range(n):
        nd = nodes[k]
        if nd[8] > -1:
            for ti in (int(nd[8]), int(nd[9])):
                v = tris[ti, :12].reshape(3, 4)[:, :3]
                assert np.all(v >= nd[:3]) and np.all(v <= nd[4:7])
            assert nd[10] == nd[11]


def test_bvh_invariants(ship_scene):
    check_threaded_bvh(ship_scene["nodes"], ship_scene["tris"])
    t = random_soup(3000, 11)
    check_threaded_bvh(H.buildSAHTree(t), t)


@pytest.mark.slow
def test_bvh_standin_scenes_invariants(tmp_path):
    obj, mtl = pt_scenes.write_scene("bunny", str(tmp_path))
    sb = H.setupBuffers(obj, mtl)
    assert 60000 < len(sb["tris"]) < 80000
    check_threaded_bvh(sb["nodes"], sb["tris"])


def write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


MTL = """# comment
newmtl A
Ns 500
Ka 1 1 1
Kd 0.5 0.25 1
Ks 0.1 0.2 0.3
Ke 1 2 3
Ni 1.45
d 1
illum 2

newmtl Short
Ns 0
Kd 1 0 0
newmtl Skipped
Ns 10
Kd 0 1 0
Ks 1 1 1
Ke 0 0 0
	Kd 9 9 9
x
y
"""

OBJ = """# quirks
v 0 0 0
v 1 0 0
v 0 1 0
vn 0.1 0.2 0.3
v 1 1 1e-3
usemtl A
f 1 2 3
usemtl Nope
f 1 2 5
usemtl Short
f 2 3 4
v 2 2 2.5
usemtl A
f 5 6 1
"""


def test_loader_quirks_match_oracle(tmp_path):
    obj, mtl = write(tmp_path, "q.obj", OBJ), write(tmp_path, "q.mtl", MTL)
    tp, mp = H.load_vertex_data(obj, mtl)
    to, mo = O.load_obj(obj, mtl)
    assert same(tp, to) and same(mp, mo)
    # "Short" (block shorter than 8 lines) swallows the next newmtl: only 2 materials
    assert len(mp) == 2
    assert mp[0, 12] == 7.5 and mp[0, 13] == 1.0 and mp[0, 14] == np.float32(0.5)
    assert tp[1, 12] == 0.0                       # unknown material -> index 0
    assert np.all(tp[2, 8:11] == 0.0)             # `vn` line consumed as vertex (0,0,0)


def test_loader_errors(tmp_path):
    mtl = write(tmp_path, "e.mtl", MTL)
    with pytest.raises(H.PTError) as e:
        H.load_vertex_data(str(tmp_path / "missing.obj"), mtl)
    assert e.value.code == -2
    bad = write(tmp_path, "bad.obj", "v 0 0 0\nf 1 2 3\n")
    with pytest.raises(H.PTError) as e:
        H.load_vertex_data(bad, mtl)
    assert e.value.code == -3
    slashes = write(tmp_path, "sl.obj", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1/1 2/2 3/3\n")
    with pytest.raises(H.PTError):
        H.load_vertex_data(slashes, mtl)
    long_line = write(tmp_path, "long.obj", "v 0 0 0 " + "0" * 200 + "\n")
    with pytest.raises(H.PTError) as e:
        H.load_vertex_data(long_line, mtl)
    assert e.value.code == -3


def test_empty_scene_is_rejected():
    with pytest.raises(H.PTError):
        H.buildSAHTree(np.zeros((0, 16), np.float32))


def test_aces_host_matches_oracle():
    rng = np.random.default_rng(4)
    img = (rng.random((17, 13, 4), dtype=np.float32) * 4).astype(np.float32)
    img[0, 0, :3] = [np.nan, -1.0, np.inf]
    assert np.array_equal(H.aces_rgba8_host(img), O.aces_rgba8(img))
