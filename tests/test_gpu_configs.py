"""The benchmark configurations' shapes on one GPU, bit-exact against the oracle.

SURVEY.md §8(d) C3-C5 and the reference's own shipped scenes:
  * C5 shape: 3840x2160 through the captured progressive hipGraph (pt_progressive_*), the
    reference's render loop (ogl_path_trace.h:160-204) without a host round trip per frame;
  * C4 shape: the Sponza-style stand-in at 1920x1080 split over 8 row-interleaved rank
    contexts (world = 8) on one device, assembled as the 8-GPU run's gather assembles it;
  * C3 at its full 1920x1080 size;
  * the reference's scene_data/drift (11,846 triangles, 24 materials), p and p2 (6,258 each)
    scenes, which take the global-memory walk (tests/golden/ref_scenes.npz, made by
    make_golden.py).
Full-size frames are checked at oracle-rendered sample pixels plus every pixel of the first
and last rows (computeShader.c:505-554 per pixel); small ones in full.  No tolerance.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import pt_host as H
from test_gpu_parity import assert_bitwise

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sample_xy(W, Hh, n, seed):
    rng = np.random.default_rng(seed)
    xs = np.concatenate([rng.integers(0, W, n), np.arange(W), np.arange(W)])
    ys = np.concatenate([rng.integers(0, Hh, n), np.zeros(W, int), np.full(W, Hh - 1)])
    return xs, ys


@pytest.fixture(scope="module")
def ref_scenes():
    z = np.load(os.path.join(GOLDEN, "ref_scenes.npz"))
    return {k: H.scene_from_arrays(z[k + "_tris"], z[k + "_mats"]) for k in ("drift", "p", "p2")}


@pytest.fixture(scope="module")
def sponza_scene(tmp_path_factory):
    import pt_scenes
    return H.setupBuffers(*pt_scenes.write_scene("sponza", str(tmp_path_factory.mktemp("c4"))))


@pytest.fixture(scope="module")
def bunny_scene(tmp_path_factory):
    import pt_scenes
    return H.setupBuffers(*pt_scenes.write_scene("bunny", str(tmp_path_factory.mktemp("c3"))))


def test_c5_shape_4k_progressive_graph(cornell_scene):
    """3840x2160, 8 bounces, 8 frames as 2 replays of a graph of 2 launches x 2 frames: the
    captured loop at the C5 image size, with the frame counter advanced on the device."""
    W, Hh = 3840, 2160
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.upload(cornell_scene)
    pt.progressive_setup(frames_per_launch=2, launches_per_replay=2)
    pt.progressive_run(replays=2)
    got = pt.read_rgba32f()
    pt.close()
    xs, ys = sample_xy(W, Hh, 8192, 51)
    want = O.render_pixels(cornell_scene, W, Hh, xs, ys, max_bounce=8, n_frames=8)
    assert_bitwise(got[ys, xs], want, "4K graph replay")
    assert np.all(got[..., 3] == np.float32(1.0))


def test_c4_shape_eight_rank_contexts(sponza_scene):
    """The C4 row split at full size: 8 contexts (rank r of world 8 renders rows r, r+8, ...)
    on one device, assembled by the gather's row interleave, equal the world-1 frame bit for
    bit and the oracle at sampled pixels."""
    W, Hh, frames = 1920, 1080, 2
    parts = []
    for r in range(8):
        pt = H.PathTracer(W, Hh, max_bounce=8, rank=r, world=8)
        pt.upload(sponza_scene)
        pt.render(1, frames, 0)
        parts.append(pt.read_rgba32f())
        pt.close()
    import torch
    import pt_dist
    rmax = pt_dist.rows_max(Hh, 8)
    blocks = np.zeros((8, rmax, W, 4), np.float32)     # the gather's padded row blocks
    for r, part in enumerate(parts):
        blocks[r, : len(part)] = part
    img = pt_dist.interleave(torch.from_numpy(blocks), Hh).numpy()
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.upload(sponza_scene)
    pt.render(1, frames, 0)
    full = pt.read_rgba32f()
    pt.close()
    assert_bitwise(img, full, "8-way split vs one context")
    xs, ys = sample_xy(W, Hh, 3000, 52)
    want = O.render_pixels(sponza_scene, W, Hh, xs, ys, max_bounce=8, n_frames=frames)
    assert_bitwise(full[ys, xs], want, "C4 1080p samples")


def test_c3_full_size_sampled(bunny_scene):
    """The C3 stand-in (69k triangles, global-memory walk) at 1920x1080, frames 1..3."""
    W, Hh = 1920, 1080
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.upload(bunny_scene)
    pt.render(1, 3, 0)
    got = pt.read_rgba32f()
    pt.close()
    xs, ys = sample_xy(W, Hh, 3000, 53)
    want = O.render_pixels(bunny_scene, W, Hh, xs, ys, max_bounce=8, n_frames=3)
    assert_bitwise(got[ys, xs], want, "C3 1080p samples")


@pytest.mark.parametrize("name", ["drift", "p", "p2"])
@pytest.mark.parametrize("variant", [0, 3])
def test_reference_scenes_full_image(ref_scenes, name, variant):
    """The reference's own scenes, whole image, 4 frames, 8 bounces, frame offset 11 on a
    prior image."""
    sc = ref_scenes[name]
    W, Hh = 96, 64
    prior = np.random.default_rng(6).random((Hh, W, 4), dtype=np.float32)
    want = O.render(sc, W, Hh, max_bounce=8, frame_first=11, n_frames=4, acc_first=1, accum=prior.copy())
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.set_kernel(variant)
    pt.upload(sc)
    pt.write_rgba32f(prior)
    pt.render(11, 4, 1)
    got = pt.read_rgba32f()
    pt.close()
    assert_bitwise(got, want, "%s, variant %d" % (name, variant))


@pytest.mark.parametrize("name", ["drift", "p", "p2"])
def test_reference_scenes_full_hd_sampled(ref_scenes, name):
    """The reference's scenes at 1920x1080, 2 frames, sampled, and their reference-semantics
    work counts at a small size."""
    sc = ref_scenes[name]
    W, Hh = 1920, 1080
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.upload(sc)
    pt.render(1, 2, 0)
    got = pt.read_rgba32f()
    pt.close()
    xs, ys = sample_xy(W, Hh, 3000, 54)
    want = O.render_pixels(sc, W, Hh, xs, ys, max_bounce=8, n_frames=2)
    assert_bitwise(got[ys, xs], want, "%s 1080p samples" % name)
    want_img, want_cnt = O.render(sc, 40, 30, max_bounce=8, n_frames=2, counters=True)
    pt = H.PathTracer(40, 30, max_bounce=8)
    pt.upload(sc)
    pt.set_counting(True)
    pt.render(1, 2, 0)
    img = pt.read_rgba32f()
    _, cnt = pt.stats()
    pt.close()
    assert_bitwise(img, want_img, "%s counting build" % name)
    assert [cnt["segments"], cnt["node_visits"], cnt["tri_tests"], cnt["sphere_tests"], cnt["hits"]] == \
        [int(x) for x in want_cnt]


def test_c5_graph_frame_range_strip(cornell_scene):
    """The C5 frame range through the captured graph: a 3840-wide strip of the 4K frame
    (rows 0, 135, ..., rank 0 of a 135-way row split: the full-width camera rays) replayed
    from pt_progressive_reset(2980) across frame 2986, where frame * 719393 passes 2^31
    (computeShader.c:514-515: the seed wraps mod 2^32), then from 4090 across 4096, on top of
    the first replay's image (the running mean :548-551 at float(frame) ~ 4096).  Sampled
    pixels span every x, including x >= 2325, where the x term alone passes 2^31."""
    W, Hh, world = 3840, 2160, 135
    pt = H.PathTracer(W, Hh, max_bounce=8, rank=0, world=world)
    pt.upload(cornell_scene)
    pt.progressive_setup(frames_per_launch=4, launches_per_replay=2)
    pt.progressive_reset(2980)
    pt.progressive_run(replays=1)                  # frames 2980..2987, accumulate from frame 2980
    a = pt.read_rgba32f()
    pt.progressive_reset(4090)
    pt.progressive_run(replays=1)                  # frames 4090..4097
    b = pt.read_rgba32f()
    pt.close()
    rows = np.arange(0, Hh, world)
    assert a.shape == (len(rows), W, 4)
    rng = np.random.default_rng(57)
    li = np.concatenate([rng.integers(0, len(rows), 3000), np.zeros(W, int), np.full(W, len(rows) - 1)])
    xs = np.concatenate([rng.integers(0, W, 3000), np.arange(W), np.arange(W)])
    ys = rows[li]
    wa = O.render_pixels(cornell_scene, W, Hh, xs, ys, max_bounce=8, frame_first=2980, n_frames=8, acc_first=1)
    assert_bitwise(a[li, xs], wa, "graph frames 2980..2987")
    wb = O.render_pixels(cornell_scene, W, Hh, xs, ys, max_bounce=8, frame_first=4090, n_frames=8, acc_first=1,
                         prior=wa)
    assert_bitwise(b[li, xs], wb, "graph frames 4090..4097")
