"""General Wavefront ingest (pt_scene_load_obj_ex with PT_LOAD_ROBUST).

1. On files the reference parser reads correctly (geometry_loader.h:15-142: 8-line MTL
   blocks, `v`, `f a b c`, `usemtl`) it yields the reference loader's arrays bit for bit.
2. Beyond that it reads real exports: v/vt/vn corners, negative indices, polygons (fan),
   comments, continuations, long lines, free-form MTL, `mtllib`.
3. Malformed input is an error with file:line, not istream's silent zeros.
No GPU needed.
"""
import os

import numpy as np
import pytest

import pt_host as H
import pt_scenes
from conftest import REF_SCENES


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("name", ["cornell", "bunny", "sponza"])
def test_robust_equals_reference_loader(name, tmp_path):
    obj, mtl = pt_scenes.write_scene(name, str(tmp_path))
    t_ref, m_ref = H.load_vertex_data(obj, mtl)
    t_rob, m_rob = H.load_obj_robust(obj, mtl)
    assert np.array_equal(bits(t_ref), bits(t_rob)) and np.array_equal(bits(m_ref), bits(m_rob))


@pytest.mark.skipif(not os.path.isdir(REF_SCENES), reason="reference scene_data not mounted")
@pytest.mark.parametrize("name", ["ship", "p", "p2", "drift"])
def test_robust_equals_reference_loader_on_shipped_scenes(name):
    obj, mtl = os.path.join(REF_SCENES, name + "obj.txt"), os.path.join(REF_SCENES, name + "mtl.txt")
    t_ref, m_ref = H.load_vertex_data(obj, mtl)
    t_rob, m_rob = H.load_obj_robust(obj, mtl)
    assert np.array_equal(bits(t_ref), bits(t_rob)) and np.array_equal(bits(m_ref), bits(m_rob))


MTL = """# exported materials
newmtl red
Ns 250.000000
Kd 0.8 0.1 0.1
illum 2
newmtl lamp
Ke 1 1 0.5
Kd 0.5
d 1.0
map_Kd ignored.png
newmtl  plain
"""

OBJ = """# a quad, a pentagon and a triangle in every corner notation
mtllib mats.mtl
o thing
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
vt 0 0
vt 1 0
vn 0 0 1
g quad
usemtl red
f 1/1/1 2/2/1 3/2/1 4/1/1
s off
v 2 0 0
v 3 0 0 1.0
v 3.5 1 0
v 2.5 2 0
v 1.5 \\
  1 0
usemtl lamp
f -5 -4 -3 -2 -1
usemtl nosuchmaterial
f 1//1 3//1 4//1   # trailing comment
usemtl plain
f 2 3 5 """ + " " * 200 + """
"""


def write(tmp_path, obj=OBJ, mtl=MTL):
    (tmp_path / "mats.mtl").write_text(mtl)
    p = tmp_path / "thing.obj"
    p.write_text(obj)
    return str(p), str(tmp_path / "mats.mtl")


def test_robust_reads_real_exports(tmp_path):
    obj, mtl = write(tmp_path)
    tris, mats = H.load_obj_robust(obj)                 # MTL from `mtllib`
    t2, m2 = H.load_obj_robust(obj, mtl)                # or given explicitly
    assert np.array_equal(bits(tris), bits(t2)) and np.array_equal(bits(mats), bits(m2))
    V = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [2, 0, 0], [3, 0, 0], [3.5, 1, 0],
                  [2.5, 2, 0], [1.5, 1, 0]], np.float32)
    faces = [((0, 1, 2), 0), ((0, 2, 3), 0),                      # quad -> fan
             ((4, 5, 6), 1), ((4, 6, 7), 1), ((4, 7, 8), 1),      # pentagon, negative indices
             ((0, 2, 3), 0),                                      # unknown material -> 0
             ((1, 2, 4), 2)]
    want = np.zeros((len(faces), 16), np.float32)
    for i, ((a, b, c), m) in enumerate(faces):
        want[i, 0:3], want[i, 4:7], want[i, 8:11], want[i, 12] = V[a], V[b], V[c], m
    assert np.array_equal(bits(tris), bits(want))
    # materials: color, emission, specular, {strength 7.5, smoothness, specProb, 0}
    assert mats.shape == (3, 16)
    assert np.allclose(mats[0, 0:3], [0.8, 0.1, 0.1]) and mats[0, 13] == 1.0
    assert mats[0, 14] == np.float32(np.float64(np.float32(250.0)) / 1000.0)
    assert np.allclose(mats[1, 0:3], [0.5, 0.5, 0.5]) and np.allclose(mats[1, 4:7], [1, 1, 0.5])
    assert mats[1, 13] == 0.0 and mats[1, 14] == 0.0
    assert np.all(mats[:, 12] == 7.5)
    assert np.all(mats[2, :12] == 0)


@pytest.mark.parametrize("obj,needle", [
    ("v 0 0 0\nv 1 0 0\nf 1 2 3\n", "thing.obj:3"),              # index past the vertices
    ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2\n", "fewer than 3"),
    ("v 0 0 zero\n", "malformed number"),
    ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n", "not a valid vertex"),   # OBJ indices are 1-based
    ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf -4 -3 -2\n", "not a valid vertex"),
])
def test_robust_reports_malformed_obj(tmp_path, obj, needle):
    p, _ = write(tmp_path, obj=obj)
    with pytest.raises(H.PTError) as e:
        H.load_obj_robust(p)
    assert e.value.code == -3 and needle in str(e.value)


def test_robust_reports_malformed_mtl_and_io(tmp_path):
    p, _ = write(tmp_path, mtl="newmtl a\nKd 1 x 1\n")
    with pytest.raises(H.PTError) as e:
        H.load_obj_robust(p)
    assert e.value.code == -3 and "mats.mtl:2" in str(e.value)
    with pytest.raises(H.PTError) as e:
        H.load_obj_robust(str(tmp_path / "missing.obj"))
    assert e.value.code == -2


def test_reference_mode_still_rejects_what_the_reference_cannot_read(tmp_path):
    """The reference-semantics loader keeps its contract: `f a/b/c` is an error there."""
    obj, mtl = write(tmp_path)
    with pytest.raises(H.PTError):
        H.load_vertex_data(obj, mtl)
