"""CPU checks of the wide global-memory walk (pt_wide.h).

tests/wide/wide_sim.cpp runs the kernel's own per-lane functions (ptw::wide_hits /
wide_visit / wide_pop, compiled for the host) beside the reference's binary walk
(calculateRayCollision, computeShader.c:367-432) on diffuse paths and adversarial rays, and
fails on any segment whose closest t (bitwise) or triangle differs, or on any record child
whose exact box test passes while the conservative test rejects it.  The GPU parity tests
(tests/test_gpu_wide.py and every global-memory scene of the suite) then compare the kernel
with the oracle.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import fuzz_scenes
import pt_host as H

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "wide", "wide_sim.cpp")
WIDE_CPP = os.path.join(REPO, "opengl-path-tracing_amd", "csrc", "pt_wide.cpp")


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    d = tmp_path_factory.mktemp("wide")
    exe = str(d / "wide_sim")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-march=x86-64-v3", "-o", exe, SRC,
                           WIDE_CPP])

    def run(sb, stride=32, bounces=8, adversarial=5000):
        path = str(d / "scene.bin")
        with open(path, "wb") as f:
            np.array([len(sb["tris"]), len(sb["nodes"]), len(sb["spheres"])], np.int32).tofile(f)
            for k in ("tris", "nodes", "spheres", "cam"):
                np.ascontiguousarray(sb[k], np.float32).tofile(f)
        r = subprocess.run([exe, path, str(stride), str(bounces), str(adversarial)], capture_output=True, text=True)
        assert r.returncode in (0, 1, 3), r.stderr
        out = json.loads(r.stdout.strip().splitlines()[-1])
        out["rc"], out["stderr"] = r.returncode, r.stderr
        return out
    return run


def _ok(res):
    assert res["rc"] == 0 and res["mismatches"] == 0 and res["cons_violations"] == 0, res["stderr"][:2000]
    # every retest the leaf certificate skips (pt_wide.h) would have passed the exact test
    assert res["cert_violations"] == 0, res["stderr"][:2000]


def test_cornell(sim, cornell_scene):
    res = sim(cornell_scene, stride=8, adversarial=20000)
    _ok(res)
    assert res["records"] >= 1 and res["segments"] > 20000


def test_ship(sim, ship_scene):
    _ok(sim(ship_scene, stride=16, adversarial=20000))


@pytest.mark.parametrize("seed", range(40))
def test_random_scenes(sim, seed):
    """Triangle soups with flat quads, degenerate / duplicate triangles, floors and far-off
    placements (tests/fuzz_scenes.py), sizes up to 9000 triangles."""
    sc, _ = fuzz_scenes.random_case(seed)
    if len(sc["nodes"]) == 0:
        pytest.skip("no triangles")
    _ok(sim(sc, stride=96, adversarial=3000))


def test_stand_in_mesh(sim):
    """A 6k-triangle bunny stand-in (the C3 generator at a smaller size): a deep tree whose
    leaves the wide walk reaches through several record levels, partly outside LDS."""
    import pt_scenes
    obj, mtl = pt_scenes.write_scene("bunny", os.path.join(REPO, "scenes", "bunny_6000"), target_tris=6000)
    res = sim(H.setupBuffers(obj, mtl), stride=48, adversarial=10000)
    _ok(res)
    # fewer record visits than the binary walk's node visits, and about as many leaves
    assert res["wide_visits"] < 0.5 * res["ref_visits"]
    assert res["wide_leaves"] < 1.2 * res["ref_leaves"] + 0.5


def test_single_leaf_and_two_leaf_trees(sim):
    """Roots that are a leaf (one record with one leaf child) and one internal node."""
    for n in (1, 2, 3, 4):
        tris = np.zeros((n, 16), np.float32)
        for i in range(n):
            tris[i, 0:3], tris[i, 4:7], tris[i, 8:11] = (i, 0, 0), (i + 1, 0, 1), (i, 1, 0.5)
        mats = np.zeros((1, 16), np.float32)
        mats[0, 0:3] = 0.5
        sc = H.scene_from_arrays(tris, mats)
        sc["cam"] = np.array([0.5, -6, 0.5, 0, 0.1, 1, 0.05, 0, 0, 0, 0, 0], np.float32)
        _ok(sim(sc, stride=64, adversarial=4000))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_leaf_certificate_fuzz(tmp_path, seed):
    """ptw::leaf_certificate against the reference's exact slab test of the leaf box
    (tests/wide/cert_fuzz.cpp): rays aimed at vertices, edges and interior points of leaf
    triangles (nudged a few ulps), flat axis-aligned leaves among them, near and far origins;
    for every hit that could move t, a certified hit must pass the exact test at t just above
    t_h and beyond.  The sample is adversarial (tens of thousands of exact-test failures);
    none may be certified, and most ordinary hits certify."""
    exe = str(tmp_path / "cert_fuzz")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-march=x86-64-v3", "-o", exe,
                           os.path.join(REPO, "tests", "wide", "cert_fuzz.cpp")])
    r = subprocess.run([exe, "3000000", str(seed)], capture_output=True, text=True)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and out["violations"] == 0, r.stderr[:2000]
    assert out["exact_fail"] > 1000                   # the sample does reach the failing cases
    assert out["certified"] > 0.8 * out["hits"] and out["flat_certified"] > 0.7 * out["flat_hits"]


def test_select_transition_matches_rules(tmp_path):
    """The walk's select-only transition (ptw::wide_visit / wide_pop) against its rules written
    out as branches (tests/wide/visit_equiv.cpp): pushes, flushes of a full stack, resumed
    records, pops down to the resume position, stack depths 2, 3 and 4."""
    exe = str(tmp_path / "visit_equiv")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-march=x86-64-v3", "-o", exe,
                           os.path.join(REPO, "tests", "wide", "visit_equiv.cpp")])
    r = subprocess.run([exe, "400000", "7"], capture_output=True, text=True)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and out["mismatches"] == 0, r.stderr[:2000]
    assert out["flushes"] > 10000 and out["empty_pops"] > 10000 and out["pushes"] > 100000


def _order_sim(tmp_path, sb, stride):
    exe = str(tmp_path / "order_sim")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                           os.path.join(REPO, "tests", "wide", "order_sim.cpp")])
    path = str(tmp_path / "scene.bin")
    with open(path, "wb") as f:
        np.array([len(sb["tris"]), len(sb["nodes"]), len(sb["mats"]), len(sb["spheres"])], np.int32).tofile(f)
        for k in ("tris", "nodes", "mats", "spheres", "cam"):
            np.ascontiguousarray(sb[k], np.float32).tofile(f)
    r = subprocess.run([exe, path, str(stride)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_any_order_closest_hit(tmp_path, cornell_scene, ship_scene):
    """A walk in another order (near child first, or a static per-node order), culled by the
    best hit so far and keeping (distance, preorder rank), gives the reference's closest hit on
    every segment whose winning leaf passes its exact box test at the winning distance
    (tests/wide/order_sim.cpp).  It saves few visits: about 1% on Cornell (7% / 11% on the C3 /
    C4 stand-ins), which is why the walks keep the reference's order."""
    for sb, stride in ((cornell_scene, 11), (ship_scene, 17)):
        res = _order_sim(tmp_path, sb, stride)
        assert res["segments"] > 8000
        assert res["mismatches_near_first"] == 0 and res["mismatches_static_order"] == 0, res
        assert res["uncertified_winners"] <= res["segments"] // 1000, res
        assert res["visits_near_first"] <= res["visits_reference"] * 1.02, res


def test_k_wide_cut_visits(tmp_path, cornell_scene, ship_scene):
    """K-wide trees cut from the reference's tree by the surface-area-optimal rule (K = 2, 4,
    8; tests/wide/widek_sim.cpp), walked in preorder with children culled at the t of the
    record visit: the reference's hits on every segment, and fewer record visits for wider
    records but more child box tests from K = 4 to 8 -- the cost that sets the wide walk's pace
    (on the C3 / C4 stand-ins +25% / +18% child tests for 36% / 40% fewer visits)."""
    exe = str(tmp_path / "widek_sim")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                           os.path.join(REPO, "tests", "wide", "widek_sim.cpp")])
    for name, sb, stride in (("cornell", cornell_scene, 11), ("ship", ship_scene, 17)):
        path = str(tmp_path / ("%s.bin" % name))
        with open(path, "wb") as f:
            np.array([len(sb["tris"]), len(sb["nodes"]), len(sb["mats"]), len(sb["spheres"])], np.int32).tofile(f)
            for k in ("tris", "nodes", "mats", "spheres", "cam"):
                np.ascontiguousarray(sb[k], np.float32).tofile(f)
        r = subprocess.run([exe, path, str(stride)], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["segments"] > 4000, res
        for k in ("K2", "K4", "K8"):
            assert res[k]["mismatches"] == 0, (name, res)
        assert res["K8"]["visits"] < res["K4"]["visits"] < res["K2"]["visits"], (name, res)
        assert res["K8"]["records"] < res["K4"]["records"] < res["K2"]["records"], (name, res)
