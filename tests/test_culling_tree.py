"""Host check of the culling walk's precondition (pt_bvh_culling_ok): a full
binary tree threaded in preorder whose internal boxes contain their children's boxes.  Trees
built by the reference builder qualify; any break of the structure or of containment does not
(pt_upload_scene then keeps the exact walk).  CPU only."""
import numpy as np

import pt_host as H


def nodes_of(sc):
    return np.array(sc["nodes"], np.float32)


def test_reference_built_trees_qualify(cornell_scene, ship_scene):
    assert H.bvh_culling_ok(nodes_of(cornell_scene))
    assert H.bvh_culling_ok(nodes_of(ship_scene))


def test_single_leaf_and_empty():
    one = np.zeros((1, 12), np.float32)
    one[0, 4:7] = 1.0
    one[0, 8:12] = (0, 0, -1, -1)          # a leaf: tri 0 twice, hit = miss = -1
    assert H.bvh_culling_ok(one)
    assert not H.bvh_culling_ok(np.zeros((0, 12), np.float32))


def test_loose_but_nested_boxes_qualify(cornell_scene):
    n = nodes_of(cornell_scene)
    n[0, 0:3] -= 1.0                       # only the root grows: still contains its children
    n[0, 4:7] += 1.0
    assert H.bvh_culling_ok(n)


def test_containment_break_disqualifies(cornell_scene):
    n = nodes_of(cornell_scene)
    left = int(n[0, 10])
    n[left, 4] = n[0, 4] + 0.5             # a child's max.x beyond its parent's
    assert not H.bvh_culling_ok(n)


def test_threading_break_disqualifies(cornell_scene):
    n = nodes_of(cornell_scene)
    left = int(n[0, 10])
    right = int(n[left, 11])
    n[right, 11] = right                   # the right child's miss link no longer the parent's
    assert not H.bvh_culling_ok(n)
    n = nodes_of(cornell_scene)
    n[0, 11] = 1                           # the root's miss link must end the walk
    assert not H.bvh_culling_ok(n)


def test_nan_bounds_disqualify(cornell_scene):
    n = nodes_of(cornell_scene)
    n[int(n[0, 10]), 1] = np.nan
    assert not H.bvh_culling_ok(n)


def test_bad_link_floats_disqualify(cornell_scene):
    """Link fields that are NaN, huge, fractional or out of range are refused before any
    float-to-int cast: the tree no longer qualifies."""
    for bad in (np.nan, 1e30, -1e30, 2.5, 1e9):
        n = nodes_of(cornell_scene)
        n[int(n[0, 10]), 11] = bad
        assert not H.bvh_culling_ok(n), bad
        n = nodes_of(cornell_scene)
        n[0, 10] = bad
        assert not H.bvh_culling_ok(n), bad


def test_leaf_with_distinct_hit_and_miss_disqualifies(cornell_scene):
    """A leaf's hit link must equal its miss link (both next-right, bvh.h:84-98); the public
    check no longer relies on its caller for that."""
    n = nodes_of(cornell_scene)
    leaf = int(np.argmax(n[:, 8] > -1.0))
    n[leaf, 10] = 0 if n[leaf, 11] != 0 else 1
    assert not H.bvh_culling_ok(n)
