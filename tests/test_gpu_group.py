"""pt_group.h on one GPU: G row-split contexts of one image with the scene validated once and
broadcast, and the frame gathered over RCCL (a 1-rank communicator when every context shares
the device) -- bit-identical to one context's render and to the oracle (SURVEY.md §8(e);
replaces the single context's dispatch + blit, ogl_path_trace.h:183-192).  8-GPU runs are the
driver's; the gather code path (pack, ncclGather, interleave kernel) is the same."""
import numpy as np
import pytest

import oracle_lib as O
import pt_host as H
from test_gpu_parity import assert_bitwise

pytestmark = pytest.mark.gpu


def split_render(sc, W, Hh, world, frames, max_bounce=8, order=None):
    order = list(range(world)) if order is None else order
    trs = [H.PathTracer(W, Hh, max_bounce=max_bounce, rank=r, world=world) for r in order]
    g = H.Group(trs)
    g.upload(sc)
    for t in trs:
        t.render_async(1, frames, 0)
    return g, trs


@pytest.mark.parametrize("world", [1, 3, 8])
def test_group_gather_equals_one_context(cornell_scene, ship_scene, world):
    for sc in (cornell_scene, ship_scene):
        W, Hh = 80, 53
        want = O.render(sc, W, Hh, max_bounce=8, n_frames=4)
        g, trs = split_render(sc, W, Hh, world, 4, order=list(range(world))[::-1])
        got = g.gather()
        ms, nbytes = g.stats()
        g.close()
        for t in trs:
            t.close()
        assert_bitwise(got, want, "world %d" % world)
        assert nbytes == world * ((Hh + world - 1) // world) * W * 16 and ms >= 0.0


def test_group_gather_into_device_memory(cornell_scene):
    import torch
    W, Hh, world = 96, 40, 4
    want = O.render(cornell_scene, W, Hh, max_bounce=6, n_frames=3)
    g, trs = split_render(cornell_scene, W, Hh, world, 3, max_bounce=6)
    out = torch.full((Hh, W, 4), float("nan"), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    g.gather(device_ptr=out.data_ptr())
    got = out.cpu().numpy()
    one = H.gather_rgba32f(trs)                    # one-shot form, host destination
    g.close()
    for t in trs:
        t.close()
    assert_bitwise(got, want, "device destination")
    assert_bitwise(one, want, "pt_gather_rgba32f")


def test_group_broadcast_global_memory_scene(tmp_path):
    """A scene too large for LDS (the global-memory walk with its breadth-first top nodes):
    the broadcast copies every device buffer and the walk facts; 1080p split 8 ways."""
    import pt_scenes
    sc = H.setupBuffers(*pt_scenes.write_scene("bunny", str(tmp_path), target_tris=5000))
    W, Hh = 1920, 1080
    g, trs = split_render(sc, W, Hh, 8, 2)
    got = g.gather()
    g.close()
    for t in trs:
        t.close()
    rng = np.random.default_rng(9)
    xs = np.concatenate([rng.integers(0, W, 3000), np.arange(W)])
    ys = np.concatenate([rng.integers(0, Hh, 3000), np.full(W, Hh - 1)])
    want = O.render_pixels(sc, W, Hh, xs, ys, max_bounce=8, n_frames=2)
    assert_bitwise(got[ys, xs], want, "global scene, 8-way split")


def test_group_rejects_inconsistent_contexts(cornell_scene):
    a = H.PathTracer(32, 16, rank=0, world=2)
    b = H.PathTracer(40, 16, rank=1, world=2)
    c = H.PathTracer(32, 16, rank=0, world=2)
    # render-affecting settings must agree too: the gathered frame is one render
    d = H.PathTracer(32, 16, rank=1, world=2, max_bounce=3)
    e_ = H.PathTracer(32, 16, rank=1, world=2, display_mode=2)
    f = H.PathTracer(32, 16, rank=1, world=2, flags=H.PT_FLAG_NO_SKY)
    g = H.PathTracer(32, 16, rank=1, world=2, rays_per_pixel=2)
    for trs in ([a, b], [a, c], [a], [a, d], [a, e_], [a, f], [a, g]):
        with pytest.raises(H.PTError) as e:
            H.Group(trs)
        assert e.value.code == -1
    for t in (a, b, c, d, e_, f, g):
        t.close()


def test_group_gather_time_excludes_renders(cornell_scene):
    """pt_group_stats' gather time starts at the first pack copy, after the device streams
    have waited for the contexts' renders (pt_group.h): a long render queued just before the
    gather does not count."""
    W, Hh, world = 640, 360, 2
    g, trs = split_render(cornell_scene, W, Hh, world, 200)
    g.gather()
    ms, _ = g.stats()
    for t in trs:
        t.sync()
    render_ms = max(t.timing()[0] for t in trs)
    g.close()
    for t in trs:
        t.close()
    assert render_ms > 5.0 and ms < 0.5 * render_ms, (ms, render_ms)


@pytest.mark.parametrize("world", [1, 3, 8])
def test_group_gather_aces(cornell_scene, world):
    """pt_group_gather_rgba8_aces: the gathered frame through the reference's ACES view
    (screenQuadFrag.c:12-33) on the root device, byte-equal to the host ACES of the oracle's
    frame, to host memory and to device memory."""
    import torch
    W, Hh = 72, 45
    want = O.aces_rgba8(O.render(cornell_scene, W, Hh, max_bounce=8, n_frames=3))
    g, trs = split_render(cornell_scene, W, Hh, world, 3, order=list(range(world))[::-1])
    got = g.gather_rgba8()
    out = torch.zeros((Hh, W, 4), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    g.gather_rgba8(device_ptr=out.data_ptr())
    dev = out.cpu().numpy()
    g.close()
    for t in trs:
        t.close()
    assert np.array_equal(got, want) and np.array_equal(dev, want)
    assert np.all(got[..., 3] == 255)


def test_group_present_pipelined(cornell_scene):
    """pt_group_present_begin / _end with renders queued behind them: frame f shown while f+1
    and f+2 render (three buffers), each byte-equal to the ACES view of the oracle's
    accumulation after that frame."""
    W, Hh, world, n = 64, 40, 3, 6
    trs = [H.PathTracer(W, Hh, max_bounce=8, rank=r, world=world) for r in range(world)]
    g = H.Group(trs)
    g.upload(cornell_scene)
    shown = {}
    for f in range(1, n + 1):
        for t in trs:
            t.render_async(f, 1, 0 if f == 1 else 1)
        g.present_begin(f % 3)
        if f >= 3:
            shown[f - 2] = g.present_end((f - 2) % 3)
    for f in (n - 1, n):
        shown[f] = g.present_end(f % 3)
    g.close()
    for t in trs:
        t.close()
    acc = np.zeros((Hh, W, 4), np.float32)
    for f in range(1, n + 1):
        acc = O.render(cornell_scene, W, Hh, max_bounce=8, frame_first=f, n_frames=1, acc_first=int(f > 1), accum=acc)
        assert np.array_equal(shown[f], O.aces_rgba8(acc)), f


@pytest.mark.skipif(__import__("torch").cuda.device_count() < 2, reason="needs two GPUs")
@pytest.mark.parametrize("world", [3, 5])
def test_group_across_two_devices(cornell_scene, world):
    """Contexts spread unevenly over two devices (so the device with more contexts has several
    slots and the other padded ones): the cross-device branches -- ncclBroadcast of the scene,
    the on-device copies to a device's other contexts, ncclGather of the row blocks and the
    block table -- assemble the oracle's frame bit for bit."""
    W, Hh = 80, 53
    want = O.render(cornell_scene, W, Hh, max_bounce=8, n_frames=3)
    trs = [H.PathTracer(W, Hh, max_bounce=8, rank=r, world=world, device=0 if r % 3 == 0 else 1)
           for r in range(world)]
    g = H.Group(trs)
    g.upload(cornell_scene)
    for t in trs:
        t.render_async(1, 3, 0)
    got = g.gather()
    aces = g.gather_rgba8()
    g.close()
    for t in trs:
        t.close()
    assert_bitwise(got, want, "world %d over two devices" % world)
    assert np.array_equal(aces, O.aces_rgba8(want))
