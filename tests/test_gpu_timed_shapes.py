"""The launch shapes bench.py times, in shading mode (display mode 1), against the oracle.

bench.py's C2 step is one render of frames 1..1024 at 1920x1080 (one fused launch), C3 / C4
one render of frames 1..256, C5 frames 1..4096 at 3840x2160 as replays of a captured graph
(computeShader.c:505-554 per pixel and frame, the running mean of :548-551).  Those launches take branches that short test renders never reach:
  * a fresh context's first long render runs a 2-frame probe launch, sorts the tile costs and
    then renders the rest as the continuation (pt_render.hip enqueue_frames);
  * frame-split work items of 16 frames (LDS scenes) or 4 (global-memory scenes), which only
    images of more than ~100k pixels get (plan_group);
  * the queue reservation sized from the launch's ids, and the scratch reserved for the
    undivided launch by the probe branch, then reused by the next identical render.
Each test renders like the bench: a fresh context, one render (probe + rest), a second render
of the same frames (warm: sorted order, scratch in place), and compares both images with the
oracle -- in full at small sizes, at seeded sample pixels plus the first and last rows at the
timed sizes.  No tolerance.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import pt_host as H
from test_gpu_parity import assert_bitwise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scenes(tmp_path_factory, cornell_scene):
    import pt_scenes
    d = str(tmp_path_factory.mktemp("timed"))
    return {"cornell": cornell_scene,
            "bunny": H.setupBuffers(*pt_scenes.write_scene("bunny", d)),
            "sponza": H.setupBuffers(*pt_scenes.write_scene("sponza", d))}


def _bench_like(sc, W, Hh, spp, bounces=8):
    """Two renders of frames 1..spp on one fresh context, as bench.py's warm-up + timed step."""
    pt = H.PathTracer(W, Hh, max_bounce=bounces)
    pt.upload(sc)
    pt.render(1, spp, 0)
    first = pt.read_rgba32f()
    pt.render(1, spp, 0)
    second = pt.read_rgba32f()
    pt.close()
    return first, second


def _sample(W, Hh, n, seed):
    rng = np.random.default_rng(seed)
    flat = rng.choice(W * Hh, size=min(n, W * Hh), replace=False)
    xs = np.concatenate([flat % W, np.arange(W), np.arange(W)])
    ys = np.concatenate([flat // W, np.zeros(W, int), np.full(W, Hh - 1)])
    return xs, ys


def test_c2_launch_1024_frames_small_full_image(cornell_scene):
    """C2's 1024-frame launch at 64x48, every pixel: probe launch, tile sort, continuation."""
    W, Hh, spp = 64, 48, 1024
    want = O.render(cornell_scene, W, Hh, max_bounce=8, n_frames=spp)
    first, second = _bench_like(cornell_scene, W, Hh, spp)
    assert_bitwise(first, want, "C2 1024 frames 64x48, cold")
    assert_bitwise(second, want, "C2 1024 frames 64x48, warm")


@pytest.mark.parametrize("W,Hh", [(480, 256), (1920, 1080)])
def test_c2_launch_1024_frames_items_of_16(cornell_scene, W, Hh):
    """C2's launch where the work items hold 16 frames (>= ~115k pixels), up to the timed
    1920x1080 itself: sampled pixels plus the first and last rows."""
    spp = 1024
    xs, ys = _sample(W, Hh, 1500, W + Hh)
    want = O.render_pixels(cornell_scene, W, Hh, xs, ys, max_bounce=8, n_frames=spp)
    first, second = _bench_like(cornell_scene, W, Hh, spp)
    assert_bitwise(first[ys, xs], want, "C2 1024 frames %dx%d, cold" % (W, Hh))
    assert_bitwise(second[ys, xs], want, "C2 1024 frames %dx%d, warm" % (W, Hh))


@pytest.mark.parametrize("name", ["bunny", "sponza"])
def test_c3_c4_launch_256_frames_small_full_image(scenes, name):
    """C3 / C4's 256-frame launch at 40x24 on the 69k / 249k-triangle stand-ins (global-memory
    wide walk), every pixel."""
    W, Hh, spp = 40, 24, 256
    sc = scenes[name]
    want = O.render(sc, W, Hh, max_bounce=8, n_frames=spp)
    first, second = _bench_like(sc, W, Hh, spp)
    assert_bitwise(first, want, "%s 256 frames 40x24, cold" % name)
    assert_bitwise(second, want, "%s 256 frames 40x24, warm" % name)


@pytest.mark.parametrize("name", ["bunny", "sponza"])
def test_c3_c4_launch_256_frames_timed_size(scenes, name):
    """C3 / C4's timed launch itself: 1920x1080, frames 1..256 in one render (items of 4
    frames), sampled pixels plus the first and last rows."""
    W, Hh, spp = 1920, 1080, 256
    sc = scenes[name]
    xs, ys = _sample(W, Hh, 600, 17 if name == "bunny" else 19)
    want = O.render_pixels(sc, W, Hh, xs, ys, max_bounce=8, n_frames=spp)
    first, second = _bench_like(sc, W, Hh, spp)
    assert_bitwise(first[ys, xs], want, "%s 256 frames 1080p, cold" % name)
    assert_bitwise(second[ys, xs], want, "%s 256 frames 1080p, warm" % name)


def test_c5_graph_4096_frames_timed_shape(cornell_scene):
    """C5's timed shape: 3840x2160, frames 1..4096 as two replays of a captured graph of 8
    launches x 256 frames (the device frame counter crosses the seed's signed-overflow frame
    2986 inside a launch), sampled pixels plus the first and last rows against the oracle."""
    W, Hh, spp = 3840, 2160, 4096
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.upload(cornell_scene)
    pt.progressive_setup(frames_per_launch=256, launches_per_replay=8)
    pt.progressive_reset(1)
    pt.progressive_run(replays=spp // (256 * 8))
    got = pt.read_rgba32f()
    pt.close()
    xs, ys = _sample(W, Hh, 600, 23)
    keep = np.concatenate([np.arange(600), 600 + np.arange(0, 2 * W, 16)])   # every 16th pixel of the two rows
    xs, ys = xs[keep], ys[keep]
    want = O.render_pixels(cornell_scene, W, Hh, xs, ys, max_bounce=8, n_frames=spp)
    assert_bitwise(got[ys, xs], want, "C5 4K 4096 frames through the graph")
