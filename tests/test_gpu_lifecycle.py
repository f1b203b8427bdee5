"""Context lifecycle on the GPU: scratch ownership across graph capture and later renders,
renders split by the scratch budget and by the 32-bit queue-id range, counting vs graph
replay, and one process driving contexts on two devices.  Every image check is bit-exact.
"""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
import pt_host as H
from test_gpu_parity import assert_bitwise

pytestmark = pytest.mark.gpu


def test_graph_survives_larger_render(cornell_scene):
    """A graph captured with a small frame-split scratch must keep working after a later
    pt_render grew (reallocated) the context's scratch: setup, larger render, replay."""
    want = O.render(cornell_scene, 40, 24, max_bounce=8, n_frames=6)
    pt = H.PathTracer(40, 24, max_bounce=8)
    pt.set_tuning(group=1)                      # frame-split items in every launch
    pt.upload(cornell_scene)
    pt.progressive_setup(frames_per_launch=2, launches_per_replay=3)
    pt.render(1, 12, 0)                         # needs 6x the scratch the graph holds
    pt.progressive_reset(1)
    pt.progressive_run(replays=1)
    got = pt.read_rgba32f()
    pt.render(1, 24, 0)                         # grows it again, then replays once more
    pt.progressive_reset(1)
    pt.progressive_run(replays=1)
    got2 = pt.read_rgba32f()
    pt.close()
    assert_bitwise(got, want, "graph after a larger render")
    assert_bitwise(got2, want, "graph after two larger renders")


@pytest.mark.parametrize("variant", [0, 3])
def test_scratch_budget_splits_render(cornell_scene, variant):
    """A 1 MiB scratch budget holds 34 frames of a 64x40 image: a 100-frame render runs as
    3 launches (accumulate continues across them), in direct and graph mode, with the
    counting build's totals those of the oracle."""
    want, cnt = O.render(cornell_scene, 64, 40, max_bounce=8, n_frames=100, counters=True)
    pt = H.PathTracer(64, 40, max_bounce=8)
    pt.set_kernel(variant)
    pt.set_tuning(group=2, scratch_mib=1)
    pt.upload(cornell_scene)
    pt.set_counting(True)
    pt.render(1, 100, 0)
    st = pt.stats()[1]
    got = pt.read_rgba32f()
    pt.set_counting(False)
    pt.progressive_setup(frames_per_launch=50, launches_per_replay=2)
    pt.progressive_run(replays=1)
    got_graph = pt.read_rgba32f()
    pt.close()
    assert_bitwise(got, want, "budget split")
    assert_bitwise(got_graph, want, "budget split, graph")
    assert [st["segments"], st["node_visits"], st["tri_tests"], st["sphere_tests"], st["hits"]] == \
        [int(x) for x in cnt]


def test_queue_ids_stay_32_bit(cornell_scene):
    """1024x1024 with one frame per work item and 4096 frames is 2^32 queue ids: the render
    must be split (it used to wrap and silently skip work).  Checked against the same
    frames rendered as four 1024-frame launches (each far inside the id range)."""
    W = Hh = 1024
    pt = H.PathTracer(W, Hh, max_bounce=0, display_mode=2)
    pt.set_tuning(group=1, scratch_mib=60000)  # the budget alone would allow one launch
    pt.upload(cornell_scene)
    pt.render(1, 4096, 0)
    got = pt.read_rgba32f()
    pt.set_tuning(scratch_mib=0)
    for f0 in range(1, 4097, 1024):
        pt.render(f0, 1024, 0 if f0 == 1 else 1)
    want = pt.read_rgba32f()
    pt.close()
    assert np.all(np.isfinite(got[..., 3])) and np.all(got[..., 3] == np.float32(1.0))
    assert_bitwise(got, want, "2^32 queue ids")


def test_counting_after_graph_setup_refused(cornell_scene):
    """Switching counting on after the capture drops the graph: a replay would count
    nothing, so pt_progressive_run reports PT_E_STATE instead."""
    pt = H.PathTracer(32, 16, max_bounce=4)
    pt.upload(cornell_scene)
    pt.progressive_setup(frames_per_launch=2, launches_per_replay=1)
    pt.set_counting(True)
    with pytest.raises(H.PTError) as e:
        pt.progressive_run(replays=1)
    assert e.value.code == -6
    pt.close()


def _device_count():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif("_device_count() < 2")
def test_two_devices_one_process(cornell_scene):
    """Contexts on devices 0 and 1 driven alternately from one thread: every entry point
    selects its context's device (sync, readback, ACES, tuning)."""
    want = O.render(cornell_scene, 48, 32, max_bounce=6, n_frames=3)
    pts = [H.PathTracer(48, 32, max_bounce=6, device=d) for d in (0, 1)]
    for pt in pts:
        pt.upload(cornell_scene)
    for pt in pts:
        pt.render_async(1, 3, 0)
    for pt in pts:
        pt.sync()
        pt.set_tuning(adaptive=0)
        assert_bitwise(pt.read_rgba32f(), want, "device context")
        assert np.array_equal(pt.read_rgba8(), O.aces_rgba8(want))
    for pt in pts:
        pt.close()


def test_budget_below_one_frame_still_renders(cornell_scene):
    """A 1 MiB scratch budget at 1920x1080 is smaller than one frame's split scratch (24.9 MB):
    short renders must run one frame per launch (over budget) and return, not spin on the
    host.  Checked at sampled pixels against the oracle."""
    W, Hh = 1920, 1080
    pt = H.PathTracer(W, Hh, max_bounce=4)
    pt.set_tuning(scratch_mib=1)
    pt.upload(cornell_scene)
    pt.render(1, 1, 0)
    pt.render(2, 2, 1)
    pt.progressive_setup(frames_per_launch=1, launches_per_replay=2)
    pt.progressive_reset(4)
    pt.progressive_run(replays=1)
    got = pt.read_rgba32f()
    pt.close()
    rng = np.random.default_rng(2)
    xs, ys = rng.integers(0, W, 2000), rng.integers(0, Hh, 2000)
    want = O.render_pixels(cornell_scene, W, Hh, xs, ys, max_bounce=4, n_frames=5)
    assert_bitwise(got[ys, xs], want, "sub-frame budget")


@pytest.mark.parametrize("overlap", [0, 1])
def test_overlapped_short_launches_bitwise(cornell_scene, overlap):
    """Short renders enqueued back to back (pt_render_async, no host wait) run their render
    kernels on two alternating streams (tuning key 9), with the running mean applied in frame
    order on the context's stream.  Mixed with a long launch, tile-order sorts (after the 8th
    short launch, then every 64th), a graph replay and a reset: the oracle's image, on and
    off."""
    W, Hh = 64, 40
    want = O.render(cornell_scene, W, Hh, max_bounce=8, n_frames=120)
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.set_key(9, 0 if overlap else 1)
    pt.upload(cornell_scene)
    pt.write_rgba32f(np.full((Hh, W, 4), np.nan, np.float32))
    f = 1
    for _ in range(29):                          # frames 1..29, one per launch
        pt.render_async(f, 1, 0 if f == 1 else 1)
        f += 1
    pt.render_async(f, 20, 1)                    # 30..49: a long launch on the main stream
    f += 20
    for n in [1, 2, 3, 1, 1] * 6:                # 50..97: short launches of 1-3 frames
        pt.render_async(f, n, 1)
        f += n
    pt.sync()
    mid = pt.read_rgba32f()
    assert f == 98
    pt.progressive_setup(frames_per_launch=2, launches_per_replay=2)
    pt.progressive_reset(98)
    pt.progressive_run(replays=2)                # 98..105 from the graph
    for g in range(106, 121):                    # 106..120 overlapped again after the replay
        pt.render_async(g, 1, 1)
    got = pt.read_rgba32f()
    pt.close()
    want_mid = O.render(cornell_scene, W, Hh, max_bounce=8, n_frames=97)
    assert_bitwise(mid, want_mid, "97 frames, overlap %d" % overlap)
    assert_bitwise(got, want, "120 frames, overlap %d" % overlap)


def test_overlapped_reset_and_camera_change(cornell_scene):
    """The interactive loop's reset (ogl_path_trace.h:199-203): after a camera move the next
    frame is frame 1 with accumulate = 0, enqueued while earlier frames may still render."""
    W, Hh = 48, 32
    cam2 = np.array([0.5, -5.5, 1.2, 0, 0.1, 1, 0, 0, 0, 0, 0, 0], np.float32)
    sc2 = dict(cornell_scene)
    sc2["cam"] = cam2
    want = O.render(sc2, W, Hh, max_bounce=8, n_frames=12)
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.upload(cornell_scene)
    for f in range(1, 10):
        pt.render_async(f, 1, 0 if f == 1 else 1)
    pt.set_camera(cam2)
    for f in range(1, 13):
        pt.render_async(f, 1, 0 if f == 1 else 1)
    got = pt.read_rgba32f()
    pt.close()
    assert_bitwise(got, want, "reset after camera move")


@pytest.mark.parametrize("slots", [2, 3, 4])
def test_overlap_slots_grow_and_switch(cornell_scene, slots):
    """Overlap slots whose colour scratch must grow while earlier renders are in flight
    (launches of 1, then 16, then 1 frames rotate over the slots: ensure_slot drains the slot's
    stream and the accumulate stream before reallocating), a counting render in between (never
    overlapped), and the slot count switched mid-sequence: the oracle's image."""
    W, Hh = 56, 36
    want, cnt = O.render(cornell_scene, W, Hh, max_bounce=6, n_frames=70, counters=True)
    pt = H.PathTracer(W, Hh, max_bounce=6)
    pt.set_key(9, slots)
    pt.upload(cornell_scene)
    f = 1
    for n in [1, 1, 16, 1, 16, 1, 1, 16]:           # frames 1..53
        pt.render_async(f, n, 0 if f == 1 else 1)
        f += n
    pt.set_counting(True)
    pt.render(f, 3, 1)                              # 54..56, counted, on the context stream
    pt.set_counting(False)
    f += 3
    pt.set_key(9, 2 if slots != 2 else 4)
    for n in [1, 2, 1, 4, 1, 5]:                    # 57..70
        pt.render_async(f, n, 1)
        f += n
    got = pt.read_rgba32f()
    pt.close()
    assert f == 71
    assert_bitwise(got, want, "%d slots" % slots)


@pytest.mark.parametrize("world,lag", [(1, 1), (1, 2), (3, 2), (1, 3)])
def test_present_pipelined(cornell_scene, world, lag):
    """pt_present_begin / _end: the reference's show-every-frame loop with the readback of
    frame f-lag overlapping the renders of the later frames (lag + 1 pinned buffers in
    rotation; the copies run on their own stream from a ring of three device views, which lag 3
    wraps while earlier copies may be in flight).  Every presented image equals the host ACES of the oracle's accumulation after
    that frame, byte for byte, for each row-split rank; a buffer begun twice holds the later
    image; misuse is refused."""
    W, Hh, n = 72, 40, 7
    want = [H.aces_rgba8_host(O.render(cornell_scene, W, Hh, max_bounce=6, n_frames=f)) for f in range(1, n + 1)]
    nb = lag + 1
    for rank in range(world):
        pt = H.PathTracer(W, Hh, max_bounce=6, rank=rank, world=world)
        pt.upload(cornell_scene)
        got = []
        for i in range(n):
            pt.render_async(i + 1, 1, 0 if i == 0 else 1)
            pt.present_begin(i % nb)
            if i >= lag:
                got.append(pt.present_end((i - lag) % nb))
        for j in range(n - lag, n):
            got.append(pt.present_end(j % nb))
        for f, img in enumerate(got, 1):
            assert np.array_equal(img, want[f - 1][rank::world]), (rank, f)
        assert np.array_equal(pt.read_rgba8(), want[-1][rank::world])
        # begun twice without an end: the later image
        pt.present_begin(0)
        pt.render(n + 1, 1, 1)
        pt.present_begin(0)
        last = H.aces_rgba8_host(O.render(cornell_scene, W, Hh, max_bounce=6, n_frames=n + 1))
        assert np.array_equal(pt.present_end(0, copy=False), last[rank::world])
        with pytest.raises(H.PTError):
            pt.present_end(0)          # no begin pending
        with pytest.raises(H.PTError):
            pt.present_begin(4)
        pt.close()


def test_present_fused_view_tracks_the_image(cornell_scene):
    """After a present, the next render's accumulate pass writes the ACES view itself and
    pt_present_begin only copies it.  Whatever changes the image in between -- a write of the
    accumulation, a long render, a progressive graph replay, a render with presentation paused --
    must still show the view of the current image, byte-equal to the host ACES."""
    W, Hh = 64, 36
    acc = lambda n: O.render(cornell_scene, W, Hh, max_bounce=6, n_frames=n)
    pt = H.PathTracer(W, Hh, max_bounce=6)
    pt.upload(cornell_scene)
    pt.render_async(1, 1, 0)
    pt.present_begin(0)
    pt.render_async(2, 1, 1)                       # fused: the view comes from this pass
    pt.present_begin(1)
    assert np.array_equal(pt.present_end(1), H.aces_rgba8_host(acc(2)))
    pt.render_async(3, 1, 1)                       # fused, then the image is overwritten
    seed = np.random.default_rng(3).random((Hh, W, 4), dtype=np.float32) * 2.0
    pt.write_rgba32f(seed)
    pt.present_begin(0)
    assert np.array_equal(pt.present_end(0), H.aces_rgba8_host(seed))
    pt.render_async(1, 1, 0)
    pt.present_begin(0)
    pt.render_async(2, 40, 1)                      # a long launch after a present
    pt.present_begin(1)
    assert np.array_equal(pt.present_end(1), H.aces_rgba8_host(acc(41)))
    pt.render_async(42, 1, 1)
    pt.render_async(43, 1, 1)                      # no present after 42: 43 is not fused
    pt.present_begin(2)
    pt.present_begin(3)                            # twice, nothing rendered between
    want = H.aces_rgba8_host(acc(43))
    assert np.array_equal(pt.present_end(2), want) and np.array_equal(pt.present_end(3), want)
    pt.progressive_setup(2, 1)                     # graph replays after a present
    pt.progressive_reset(44)
    pt.progressive_run(1)
    pt.present_begin(0)
    assert np.array_equal(pt.present_end(0), H.aces_rgba8_host(acc(45)))
    pt.close()


def test_read_rgba8_fused_view(cornell_scene):
    """pt_read_rgba8_aces after every render (the synchronous show-every-frame loop) takes the
    view from the accumulate pass from the second frame on: byte-equal to the host ACES, also
    when a present and a read follow the same render."""
    W, Hh = 48, 30
    pt = H.PathTracer(W, Hh, max_bounce=6)
    pt.upload(cornell_scene)
    for f in range(1, 5):
        pt.render(f, 1, int(f > 1))
        want = H.aces_rgba8_host(O.render(cornell_scene, W, Hh, max_bounce=6, n_frames=f))
        assert np.array_equal(pt.read_rgba8(), want), f
        pt.present_begin(f % 2)
        assert np.array_equal(pt.present_end(f % 2), want), f
        assert np.array_equal(pt.read_rgba8(), want), f
    pt.close()


@pytest.mark.parametrize("world", [1, 3, 8])
def test_tile_shapes_bitwise(cornell_scene, world):
    """Tuning key 20: the work queue's 64-pixel tiles as 8x8, 16x4, 32x2 or 64x1 (local rows of
    a row-split rank).  The tile shape changes only which lanes render which pixels together:
    every shape, switched between renders of one context (with a learned tile order, a captured
    graph and overlapped short launches), gives the oracle's image for every rank."""
    W, Hh = 100, 44                       # partial tiles on both edges for every shape
    want = O.render(cornell_scene, W, Hh, max_bounce=6, n_frames=5)
    for rank in range(world):
        pt = H.PathTracer(W, Hh, max_bounce=6, rank=rank, world=world)
        pt.upload(cornell_scene)
        for key in (4, 1, 3, 2, 0):
            pt.set_key(20, key)
            pt.render(1, 3, 0)
            pt.render_async(4, 1, 1)
            pt.render_async(5, 1, 1)
            assert_bitwise(pt.read_rgba32f(), want[rank::world], "world %d rank %d key 20 = %d" % (world, rank, key))
        pt.progressive_setup(frames_per_launch=1, launches_per_replay=5)
        pt.set_key(20, 3)                 # drops the graph; the next setup uses the new shape
        pt.progressive_setup(frames_per_launch=1, launches_per_replay=5)
        pt.progressive_run(replays=1)
        assert_bitwise(pt.read_rgba32f(), want[rank::world], "world %d rank %d graph" % (world, rank))
        with pytest.raises(H.PTError):
            pt.set_key(20, 5)
        pt.close()
