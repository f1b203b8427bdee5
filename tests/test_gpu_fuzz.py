"""Seeded random scenes (tests/fuzz_scenes.py), HIP path vs CPU oracle, bit for bit.

Each case draws a triangle soup with flat, degenerate and duplicated triangles, extra
spheres, random materials, camera, image size, bounces, frame numbers, toggles and display
mode; the sizes cover the LDS walk (culling, sink images), the wide-workgroup LDS walk and
the global-memory walk.  Every case also runs as variant 3 (the scene kept in global memory),
every third one with the accumulation seeded from a random prior image; every fourth renders
several rays per pixel, split over 2-3 row-interleaved contexts and reassembled; and a subset
runs the counting build, whose per-segment counters must equal the oracle's.

Tolerance: NONE (uint32 bit patterns).
"""
import numpy as np
import pytest

import fuzz_scenes as F
import oracle_lib as O
import pt_host as H

pytestmark = pytest.mark.gpu

N_CASES = 96


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _render_gpu(sc, kw, variant, prior=None, counting=False, rpp=1, rank=0, world=1):
    pt = H.PathTracer(kw["W"], kw["H"], max_bounce=kw["max_bounce"], display_mode=kw["mode"], flags=kw["flags"],
                      rays_per_pixel=rpp, rank=rank, world=world)
    try:
        pt.set_kernel(variant)
        pt.upload(sc)
        if prior is not None:
            pt.write_rgba32f(prior)
        if counting:
            pt.set_counting(True)
        pt.render(kw["frame_first"], kw["n_frames"], 0 if prior is None else 1)
        img = pt.read_rgba32f()
        return (img, pt.stats()[1]) if counting else img
    finally:
        pt.close()


@pytest.mark.parametrize("seed", range(N_CASES))
def test_random_scene_bitwise(seed):
    sc, kw = F.random_case(1000 + seed)
    W, Hh = kw["W"], kw["H"]
    prior = None
    if seed % 3 == 2:
        prior = np.random.default_rng(seed).random((Hh, W, 4), dtype=np.float32)
    want = O.render(sc, W, Hh, max_bounce=kw["max_bounce"], mode=kw["mode"], frame_first=kw["frame_first"],
                    n_frames=kw["n_frames"], acc_first=0 if prior is None else 1,
                    accum=None if prior is None else prior.copy(), flags=kw["flags"])
    for variant in (0, 3):
        got = _render_gpu(sc, kw, variant, prior)
        _check(got, want, "seed %d variant %d (%d tris, %s)" % (seed, variant, len(sc["tris"]), kw))


def _check(got, want, label):
    bad = np.argwhere(bits(got) != bits(want))
    assert bad.size == 0, "%s: %d words differ, first %s got %r want %r" % (
        label, len(bad), bad[0].tolist(), got[tuple(bad[0])], want[tuple(bad[0])])


@pytest.mark.parametrize("seed", range(0, N_CASES, 4))
def test_random_scene_rays_per_pixel_and_row_split(seed):
    sc, kw = F.random_case(4000 + seed)
    W, Hh = kw["W"], kw["H"]
    rpp, world = 2 + seed % 2, 2 + (seed // 4) % 2
    want = O.render(sc, W, Hh, max_bounce=kw["max_bounce"], mode=kw["mode"], frame_first=kw["frame_first"],
                    n_frames=kw["n_frames"], flags=kw["flags"], rpp=rpp)
    parts = [_render_gpu(sc, kw, 0, rpp=rpp, rank=r, world=world) for r in range(world)]
    _check(H.assemble_rows(parts, Hh), want, "seed %d rpp %d world %d (%d tris, %s)" % (
        seed, rpp, world, len(sc["tris"]), kw))


@pytest.mark.parametrize("seed", range(0, N_CASES, 3))
def test_random_scene_counters(seed):
    sc, kw = F.random_case(2000 + seed)
    W, Hh = kw["W"], kw["H"]
    want, wcnt = O.render(sc, W, Hh, max_bounce=kw["max_bounce"], mode=kw["mode"], frame_first=kw["frame_first"],
                          n_frames=kw["n_frames"], flags=kw["flags"], counters=True)
    got, cnt = _render_gpu(sc, kw, 0, counting=True)
    assert np.array_equal(bits(got), bits(want)), (seed, kw)
    assert [cnt["segments"], cnt["node_visits"], cnt["tri_tests"], cnt["sphere_tests"], cnt["hits"]] == \
        [int(x) for x in wcnt], (seed, len(sc["tris"]), kw)


@pytest.mark.parametrize("seed", range(1, N_CASES, 4))
def test_random_scene_one_frame_loop(seed):
    """The reference's loop shape: one pt_render_async per frame, back to back (the
    overlapped slot launches), the same image as the oracle's multi-frame render."""
    sc, kw = F.random_case(5000 + seed)
    W, Hh = kw["W"], kw["H"]
    n = 2 + seed % 5
    want = O.render(sc, W, Hh, max_bounce=kw["max_bounce"], mode=kw["mode"], frame_first=kw["frame_first"],
                    n_frames=n, flags=kw["flags"])
    pt = H.PathTracer(W, Hh, max_bounce=kw["max_bounce"], display_mode=kw["mode"], flags=kw["flags"])
    try:
        pt.upload(sc)
        for i in range(n):
            pt.render_async(kw["frame_first"] + i, 1, 0 if i == 0 else 1)
        pt.sync()
        got = pt.read_rgba32f()
    finally:
        pt.close()
    _check(got, want, "seed %d, %d one-frame renders (%d tris, %s)" % (seed, n, len(sc["tris"]), kw))
