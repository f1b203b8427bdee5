"""HIP path vs CPU oracle: bit-exact RGBA32F parity (SURVEY.md App. B ladder, step 1).

Tolerance: NONE -- every comparison is on the uint32 bit patterns (NaN payloads
included).  The kernels and the oracle pin every binary32 operation.
"""
import numpy as np
import pytest

import oracle_lib as O
import pt_host as H

pytestmark = pytest.mark.gpu

VARIANTS = [0, 3]   # 0 state machine (default), 3 the same kernel with the scene kept in global memory


@pytest.fixture(params=VARIANTS, ids=lambda v: "v%d" % v)
def V(request):
    return request.param


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def assert_bitwise(got, want, label=""):
    g, w = bits(got), bits(want)
    bad = np.argwhere(g != w)
    assert bad.size == 0, "%s: %d words differ; first %s got %r want %r" % (
        label, len(bad), bad[:3].tolist(), got[tuple(bad[0])], want[tuple(bad[0])])


def gpu_render(sc, W, H_, max_bounce=5, mode=1, frame_first=1, n_frames=1, acc_first=0,
               flags=0, rank=0, world=1, prior=None, counting=False, variant=0):
    pt = H.PathTracer(W, H_, max_bounce=max_bounce, display_mode=mode, flags=flags, rank=rank, world=world)
    pt.set_kernel(variant)
    pt.upload(sc)
    if prior is not None:
        pt.write_rgba32f(prior)
    if counting:
        pt.set_counting(True)
    pt.render(frame_first, n_frames, acc_first)
    img = pt.read_rgba32f()
    st = pt.stats()
    pt.close()
    return (img, st) if counting else img


@pytest.mark.parametrize("mode", [2, 3, 4])
def test_debug_modes_bitwise(cornell_scene, mode, V):
    want = O.render(cornell_scene, 64, 48, mode=mode)
    got = gpu_render(cornell_scene, 64, 48, mode=mode, variant=V)
    assert_bitwise(got, want, "mode %d" % mode)


@pytest.mark.parametrize("spp", [1, 4, 16])
def test_shaded_cornell_bitwise(cornell_scene, spp, V):
    want = O.render(cornell_scene, 64, 64, max_bounce=5, n_frames=spp)
    got = gpu_render(cornell_scene, 64, 64, max_bounce=5, n_frames=spp, variant=V)
    assert_bitwise(got, want, "cornell %d spp" % spp)


def test_shaded_ship_bitwise(ship_scene, V):
    want = O.render(ship_scene, 80, 60, max_bounce=5, n_frames=4)
    got = gpu_render(ship_scene, 80, 60, max_bounce=5, n_frames=4, variant=V)
    assert_bitwise(got, want, "ship")


def test_eight_bounces_and_frame_offset(cornell_scene, V):
    # frames 3000..3002 exercise the signed-overflow seed term (frame*719393 > 2^31)
    prior = np.random.default_rng(1).random((36, 64, 4), dtype=np.float32)
    want = O.render(cornell_scene, 64, 36, max_bounce=8, frame_first=3000, n_frames=3, acc_first=1,
                    accum=prior.copy())
    got = gpu_render(cornell_scene, 64, 36, max_bounce=8, frame_first=3000, n_frames=3, acc_first=1,
                     prior=prior, variant=V)
    assert_bitwise(got, want, "8 bounces")


def test_fused_equals_separate_dispatches(cornell_scene, V):
    pt = H.PathTracer(48, 32, max_bounce=8)
    pt.set_kernel(V)
    pt.upload(cornell_scene)
    for f in range(1, 6):
        pt.dispatch(f, 0 if f == 1 else 1)
    sep = pt.read_rgba32f()
    pt.render(1, 5, 0)
    fused = pt.read_rgba32f()
    pt.close()
    assert_bitwise(fused, sep, "fused vs separate")


@pytest.mark.parametrize("flags", [H.PT_FLAG_NO_AA, H.PT_FLAG_NO_SKY, H.PT_FLAG_NO_SPHERES,
                                   H.PT_FLAG_NO_TRIANGLES])
def test_toggles_bitwise(cornell_scene, flags, V):
    want = O.render(cornell_scene, 40, 30, n_frames=2, flags=flags)
    got = gpu_render(cornell_scene, 40, 30, n_frames=2, flags=flags, variant=V)
    assert_bitwise(got, want, "flags %d" % flags)


def test_ref_dispatch_footprint(cornell_scene, V):
    # glDispatchCompute(W/10, H/10) with 10x10 groups writes only the 250x250 block at 256^2
    got = gpu_render(cornell_scene, 256, 256, mode=2, flags=H.PT_FLAG_REF_DISPATCH, variant=V)
    assert np.all(got[250:] == 0) and np.all(got[:, 250:] == 0)
    want = O.render(cornell_scene, 256, 256, mode=2)
    assert_bitwise(got[:250, :250], want[:250, :250], "footprint")


def test_partition_invariance(cornell_scene, V):
    full = gpu_render(cornell_scene, 64, 50, max_bounce=8, n_frames=3, variant=V)
    parts = [gpu_render(cornell_scene, 64, 50, max_bounce=8, n_frames=3, rank=r, world=3, variant=V)
             for r in range(3)]
    assert_bitwise(H.assemble_rows(parts, 50), full, "3-way row split")


def test_counters_match_oracle(cornell_scene, V):
    want_img, want_cnt = O.render(cornell_scene, 48, 48, max_bounce=8, n_frames=4, counters=True)
    got_img, (ms, cnt) = gpu_render(cornell_scene, 48, 48, max_bounce=8, n_frames=4, counting=True, variant=V)
    assert_bitwise(got_img, want_img, "counting build")
    assert [cnt["segments"], cnt["node_visits"], cnt["tri_tests"], cnt["sphere_tests"], cnt["hits"]] == \
        [int(x) for x in want_cnt]


def test_full_hd_sampled_pixels(cornell_scene, V):
    """1920x1080, 8 bounces, 2 spp: the full-size GPU frame checked bit-exactly at 4000
    oracle-rendered pixels (plus every pixel of the first and last rows)."""
    W, Hh = 1920, 1080
    got = gpu_render(cornell_scene, W, Hh, max_bounce=8, n_frames=2, variant=V)
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.integers(0, W, 4000), np.arange(W), np.arange(W)])
    ys = np.concatenate([rng.integers(0, Hh, 4000), np.zeros(W, int), np.full(W, Hh - 1)])
    want = O.render_pixels(cornell_scene, W, Hh, xs, ys, max_bounce=8, n_frames=2)
    assert_bitwise(got[ys, xs], want, "1080p samples")


def test_golden_fixtures(cornell_scene, ship_scene, V):
    """Committed fixtures (oracle == numpy twin, tests/golden/make_golden.py)."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_images.npz"))
    for key in z.files:
        scene, W, Hh, mb, mode, spp = key.split("_")
        sc = cornell_scene if scene == "cornell" else ship_scene
        got = gpu_render(sc, int(W), int(Hh), max_bounce=int(mb), mode=int(mode), n_frames=int(spp), variant=V)
        assert_bitwise(got, z[key], key)


def test_exact_reciprocal_guard_fallback(cornell_scene, V):
    """Scene scaled by 2^-100: box coordinates fall outside the exact-reciprocal guard, so
    every slab test takes the IEEE-division chain; results must still be bit-exact."""
    sc = {k: np.array(v, copy=True) for k, v in cornell_scene.items()}
    s = np.float32(2.0 ** -100)
    sc["tris"][:, [0, 1, 2, 4, 5, 6, 8, 9, 10]] *= s
    sc["nodes"][:, [0, 1, 2, 4, 5, 6]] *= s
    sc["spheres"][:, :4] *= s
    sc["cam"][:3] *= s
    want = O.render(sc, 40, 30, max_bounce=5, n_frames=2)
    got = gpu_render(sc, 40, 30, max_bounce=5, n_frames=2, variant=V)
    assert_bitwise(got, want, "scaled scene")


def test_rays_per_pixel(cornell_scene, V):
    """raysPerPixel > 1 (computeShader.c:507-544): rays share the RNG stream of the frame."""
    want = O.render(cornell_scene, 32, 24, max_bounce=6, n_frames=2, rpp=3)
    pt = H.PathTracer(32, 24, max_bounce=6, rays_per_pixel=3)
    pt.set_kernel(V)
    pt.upload(cornell_scene)
    pt.render(1, 2, 0)
    got = pt.read_rgba32f()
    pt.close()
    assert_bitwise(got, want, "rpp 3")


@pytest.fixture(scope="module", params=["bunny", "sponza"])
def big_scene(request, tmp_path_factory):
    import pt_scenes
    d = str(tmp_path_factory.mktemp("scenes"))
    return H.setupBuffers(*pt_scenes.write_scene(request.param, d))


@pytest.mark.parametrize("variant", [0])
def test_large_scene_bitwise(big_scene, variant):
    """C3/C4 stand-ins (69k / 249k triangles): the scene no longer fits the LDS staging
    budget, so the kernels walk the BVH from global memory."""
    want = O.render(big_scene, 48, 27, max_bounce=8, n_frames=2)
    got = gpu_render(big_scene, 48, 27, max_bounce=8, n_frames=2, variant=variant)
    assert_bitwise(got, want, "large scene")


@pytest.mark.parametrize("target", [20, 80])
def test_mid_size_lds_scene_bitwise(target, tmp_path):
    """Scenes staged in LDS with more nodes than the padded walk image (kPadNodes = 67):
    the image planes are then n_nodes apart and the walk computes the hi-half address at run
    time (Cornell, 35 nodes, takes the padded compile-time path)."""
    import pt_scenes
    sc = H.setupBuffers(*pt_scenes.write_scene("bunny", str(tmp_path), target_tris=target))
    n_nodes = len(np.asarray(sc["nodes"]).reshape(-1, 12))
    assert 67 < n_nodes <= 160, n_nodes
    want = O.render(sc, 64, 48, max_bounce=8, n_frames=3)
    for waves in (6, 7):
        pt = H.PathTracer(64, 48, max_bounce=8)
        pt.set_tuning(waves_per_simd=waves)
        pt.upload(sc)
        pt.render(1, 3, 0)
        got = pt.read_rgba32f()
        pt.close()
        assert_bitwise(got, want, "mid-size LDS scene, %d tris, %d waves" % (target, waves))


def test_progressive_graph_replay(cornell_scene, V):
    """hipGraph-captured sample loop with a device frame counter == pt_render(1, N, 0)."""
    pt = H.PathTracer(40, 24, max_bounce=8)
    pt.set_kernel(V)
    pt.upload(cornell_scene)
    pt.render(1, 12, 0)
    want = pt.read_rgba32f()
    pt.write_rgba32f(np.full((24, 40, 4), np.nan, np.float32))   # frame 1 must overwrite
    pt.progressive_setup(frames_per_launch=2, launches_per_replay=3)
    pt.progressive_run(replays=2)
    got = pt.read_rgba32f()
    # a camera change drops the graph; re-setup and restart from frame 1
    pt.set_camera(cornell_scene["cam"])
    pt.progressive_setup(frames_per_launch=4, launches_per_replay=1)
    pt.progressive_run(replays=3)
    got2 = pt.read_rgba32f()
    pt.close()
    assert_bitwise(got, want, "graph replay")
    assert_bitwise(got2, want, "graph replay after re-setup")


def test_adaptive_tile_order_is_invisible(cornell_scene):
    """The longest-first tile order learnt from earlier renders changes only the schedule."""
    imgs = []
    for adaptive in (0, 1):
        pt = H.PathTracer(72, 40, max_bounce=8)
        pt.set_tuning(adaptive=adaptive)
        pt.upload(cornell_scene)
        for f0 in (1, 3, 5):
            pt.render(f0, 2, 0 if f0 == 1 else 1)
        imgs.append(pt.read_rgba32f())
        pt.close()
    assert_bitwise(imgs[1], imgs[0], "adaptive order")


@pytest.mark.parametrize("waves", [5, 6, 7, 8])
@pytest.mark.parametrize("variant", [0, 3])
@pytest.mark.parametrize("rpp", [1, 3])
def test_occupancy_builds_bitwise(cornell_scene, waves, variant, rpp):
    """Every compiled occupancy (tuning key 3) of the state-machine kernel, LDS and global
    scene, raysPerPixel 1 and 3, with a few scheduling thresholds and walk floors (64: every
    walk phase ends after one step batch)."""
    want = O.render(cornell_scene, 48, 40, max_bounce=8, n_frames=5, rpp=rpp)
    for leaf, shade, floor in ((0, 0, 0), (1, 64, 1), (64, 1, 1), (64, 64, 64), (40, 40, 24)):
        pt = H.PathTracer(48, 40, max_bounce=8, rays_per_pixel=rpp)
        pt.set_kernel(variant)
        pt.set_tuning(leaf, shade, waves_per_simd=waves, trav_floor=floor)
        pt.upload(cornell_scene)
        pt.render(1, 5, 0)
        got = pt.read_rgba32f()
        pt.close()
        assert_bitwise(got, want, "waves %d variant %d rpp %d tune %d:%d:%d" % (waves, variant, rpp, leaf, shade,
                                                                                  floor))


@pytest.mark.parametrize("compact_max", [0, 8, 63])
@pytest.mark.parametrize("variant", [0, 3])
def test_leaf_compaction_limits_bitwise(cornell_scene, compact_max, variant):
    """Leaf-phase edge tests packed over the wave (tuning key 7): never (0), only for small
    pair counts (8: most phases take the per-lane path), and up to 63 pairs (the default),
    with leaf phases of up to 64 lanes (leaf threshold 64): the same bits each way."""
    want = O.render(cornell_scene, 64, 40, max_bounce=8, n_frames=4)
    for leaf in (0, 64):
        pt = H.PathTracer(64, 40, max_bounce=8)
        pt.set_kernel(variant)
        pt.set_tuning(leaf, 0, compact_max=compact_max)
        pt.upload(cornell_scene)
        pt.render(1, 4, 0)
        got = pt.read_rgba32f()
        pt.close()
        assert_bitwise(got, want, "compaction limit %d, leaf threshold %d" % (compact_max, leaf))


def test_aces_epilogue(cornell_scene):
    pt = H.PathTracer(64, 64, max_bounce=5)
    pt.upload(cornell_scene)
    pt.render(1, 8, 0)
    img = pt.read_rgba32f()
    rgba8 = pt.read_rgba8()
    pt.close()
    assert np.array_equal(rgba8, O.aces_rgba8(img))


@pytest.mark.parametrize("group", [1, 3, 64])
@pytest.mark.parametrize("rpp", [1, 3])
@pytest.mark.parametrize("variant", [0, 3])
def test_frame_split_work_items(cornell_scene, group, rpp, variant):
    """Frame-split work items (tuning key 5): a pixel's frames spread over several lanes,
    per-frame colours stored and the running mean applied in frame order by k_accum_frames.
    Covers accumulate onto a prior image, a frame offset and 64 = the register mode."""
    prior = np.random.default_rng(3).random((30, 44, 4), dtype=np.float32)
    want = O.render(cornell_scene, 44, 30, max_bounce=8, frame_first=7, n_frames=7, acc_first=1,
                    accum=prior.copy(), rpp=rpp)
    pt = H.PathTracer(44, 30, max_bounce=8, rays_per_pixel=rpp)
    pt.set_kernel(variant)
    pt.set_tuning(group=group)
    pt.upload(cornell_scene)
    pt.write_rgba32f(prior)
    pt.render(7, 7, 1)
    got = pt.read_rgba32f()
    pt.close()
    assert_bitwise(got, want, "group %d rpp %d variant %d" % (group, rpp, variant))


@pytest.mark.parametrize("batch", [32, 128, 1024])
def test_queue_reservation_sizes_bitwise(cornell_scene, batch):
    """Queue ids reserved per atomic (tuning key 4) change only which lane renders what: one
    frame per launch (the interactive loop's shape) and a 3-frame launch, on a prior image."""
    W, Hh = 72, 40
    rng = np.random.default_rng(3)
    prior = rng.random((Hh, W, 4), dtype=np.float32)
    want = O.render(cornell_scene, W, Hh, max_bounce=8, frame_first=5, n_frames=4, acc_first=1, accum=prior.copy())
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.upload(cornell_scene)
    pt.set_key(4, batch)
    pt.write_rgba32f(prior)
    pt.render(5, 1, 1)
    pt.render(6, 3, 1)
    got = pt.read_rgba32f()
    pt.close()
    assert_bitwise(got, want, "pull batch %d" % batch)


def test_frame_split_footprint_and_graph(cornell_scene):
    """Frame-split mode with the REF_DISPATCH footprint (k_accum_frames must not touch
    pixels outside it) and inside a captured progressive graph."""
    got = gpu_render(cornell_scene, 256, 256, mode=1, n_frames=3, flags=H.PT_FLAG_REF_DISPATCH)
    assert np.all(got[250:] == 0) and np.all(got[:, 250:] == 0)
    want = O.render(cornell_scene, 256, 256, mode=1, n_frames=3)
    assert_bitwise(got[:250, :250], want[:250, :250], "footprint, split")
    want = O.render(cornell_scene, 40, 24, max_bounce=6, n_frames=12)
    pt = H.PathTracer(40, 24, max_bounce=6)
    pt.set_tuning(group=2)
    pt.upload(cornell_scene)
    pt.progressive_setup(frames_per_launch=4, launches_per_replay=3)
    pt.progressive_run(replays=1)
    got = pt.read_rgba32f()
    pt.close()
    assert_bitwise(got, want, "graph, split")


def test_nan_rays(cornell_scene, V):
    """A NaN camera position makes every camera ray NaN: it can never hit (the render
    kernels skip its walk), while the counting build still walks and counts every node the
    reference's walk visits (:393-431 with IEEE NaN compares)."""
    sc = {k: np.array(v, copy=True) for k, v in cornell_scene.items()}
    sc["cam"][0] = np.float32("nan")
    want, want_cnt = O.render(sc, 32, 24, max_bounce=4, n_frames=2, counters=True)
    got = gpu_render(sc, 32, 24, max_bounce=4, n_frames=2, variant=V)
    assert_bitwise(got, want, "NaN origin")
    got_img, (ms, cnt) = gpu_render(sc, 32, 24, max_bounce=4, n_frames=2, counting=True, variant=V)
    assert_bitwise(got_img, want, "NaN origin, counting build")
    assert [cnt["segments"], cnt["node_visits"], cnt["tri_tests"], cnt["sphere_tests"], cnt["hits"]] == \
        [int(x) for x in want_cnt]


@pytest.mark.parametrize("group", [1, 3, 64])
def test_counters_every_work_item_size(cornell_scene, group):
    """The counting build with frame-split items and with whole-pixel items (register mode)
    reports the oracle's reference-semantics counts and the same image."""
    want_img, want_cnt = O.render(cornell_scene, 40, 36, max_bounce=8, n_frames=6, counters=True)
    pt = H.PathTracer(40, 36, max_bounce=8)
    pt.set_tuning(group=group)
    pt.upload(cornell_scene)
    pt.set_counting(True)
    pt.render(1, 6, 0)
    img = pt.read_rgba32f()
    ms, cnt = pt.stats()
    pt.close()
    assert_bitwise(img, want_img, "counting, group %d" % group)
    assert [cnt["segments"], cnt["node_visits"], cnt["tri_tests"], cnt["sphere_tests"], cnt["hits"]] == \
        [int(x) for x in want_cnt]


def _tri(v0, v1, v2, m=0):
    t = np.zeros(16, np.float32)
    t[0:3], t[4:7], t[8:11], t[12] = v0, v1, v2, m
    return t


def test_edge_scenes(cornell_scene, V):
    """Scenes at the edges of the input space: no triangles (sphere only), one triangle (a
    single-triangle leaf, tri0 == tri1), and two coincident triangles (exact ties in the
    leaf's 2-way choice, :411-428)."""
    mats = cornell_scene["mats"][: cornell_scene["n_loaded_mats"]]
    one = _tri((-2, 2, 0), (2, 2, 0), (0, 2, 3), 1)[None]
    twin = np.stack([_tri((-2, 3, -1), (2, 3, -1), (0, 3, 4), 2), _tri((-2, 3, -1), (2, 3, -1), (0, 3, 4), 3)])
    for tris in (np.zeros((0, 16), np.float32), one, twin):
        sc = H.scene_from_arrays(tris, mats)
        want = O.render(sc, 24, 20, max_bounce=6, n_frames=3)
        got = gpu_render(sc, 24, 20, max_bounce=6, n_frames=3, variant=V)
        assert_bitwise(got, want, "%d triangles" % len(tris))


@pytest.mark.parametrize("W,Hh", [(1, 1), (1, 9), (13, 1), (9, 7)])
def test_tiny_and_ragged_images(cornell_scene, W, Hh, V):
    """Images smaller than one 8x8 tile and ragged tile edges."""
    want = O.render(cornell_scene, W, Hh, max_bounce=8, n_frames=4)
    got = gpu_render(cornell_scene, W, Hh, max_bounce=8, n_frames=4, variant=V)
    assert_bitwise(got, want, "%dx%d" % (W, Hh))


def test_zero_bounces_and_huge_frame_numbers(cornell_scene, V):
    """maxBounceCount = 0 (one segment per path) and frame numbers near 2^24 and 2^31, where
    float(frame) in the running mean rounds and the seed term wraps (:514-515, :548-551)."""
    want = O.render(cornell_scene, 20, 16, max_bounce=0, n_frames=2)
    got = gpu_render(cornell_scene, 20, 16, max_bounce=0, n_frames=2, variant=V)
    assert_bitwise(got, want, "0 bounces")
    prior = np.random.default_rng(5).random((16, 20, 4), dtype=np.float32)
    for f0 in ((1 << 24) - 1, (1 << 31) - 3):
        want = O.render(cornell_scene, 20, 16, max_bounce=3, frame_first=f0, n_frames=3, acc_first=1,
                        accum=prior.copy())
        got = gpu_render(cornell_scene, 20, 16, max_bounce=3, frame_first=f0, n_frames=3, acc_first=1,
                         prior=prior, variant=V)
        assert_bitwise(got, want, "frame %d" % f0)


def test_c1_config_counts_and_image(cornell_scene):
    """SURVEY.md §8(d) C1 in full: Cornell 256x256, 1 spp, maxBounceCount 4, the reference's
    glDispatchCompute(W/10, H/10) footprint -- image and reference-semantics counts equal the
    oracle's."""
    want, want_cnt = O.render(cornell_scene, 256, 256, max_bounce=4, n_frames=1, counters=True)
    got, (ms, cnt) = gpu_render(cornell_scene, 256, 256, max_bounce=4, n_frames=1,
                                flags=H.PT_FLAG_REF_DISPATCH, counting=True)
    assert_bitwise(got[:250, :250], want[:250, :250], "C1 footprint")
    assert np.all(got[250:] == 0) and np.all(got[:, 250:] == 0)
    # the oracle rendered every pixel; count the footprint's share with render_pixels
    ys, xs = np.mgrid[0:250, 0:250]
    _, fp_cnt = O.render_pixels(cornell_scene, 256, 256, xs.ravel(), ys.ravel(), max_bounce=4, n_frames=1,
                                counters=True)
    assert [cnt["segments"], cnt["node_visits"], cnt["tri_tests"], cnt["sphere_tests"], cnt["hits"]] == \
        [int(x) for x in fp_cnt]


def test_c3_stand_in_reduced_spp_counts(big_scene):
    """Reduced-spp C2/C3-style counts on a large scene (global-memory walk, frame-split items)."""
    want, want_cnt = O.render(big_scene, 40, 24, max_bounce=8, n_frames=3, counters=True)
    got, (ms, cnt) = gpu_render(big_scene, 40, 24, max_bounce=8, n_frames=3, counting=True)
    assert_bitwise(got, want, "large scene, counting")
    assert [cnt["segments"], cnt["node_visits"], cnt["tri_tests"], cnt["sphere_tests"], cnt["hits"]] == \
        [int(x) for x in want_cnt]


@pytest.mark.parametrize("extra", [0, H.PT_FLAG_NO_SPHERES])
def test_moller_trumbore_mode_bitwise(cornell_scene, ship_scene, V, extra):
    """Opt-in PT_FLAG_MOLLER_TRUMBORE (the reference's dead RayIntersectsTriangle, :228-272):
    bit-exact against the oracle's MT mode on every kernel variant."""
    flags = H.PT_FLAG_MOLLER_TRUMBORE | extra
    for sc in (cornell_scene, ship_scene):
        want = O.render(sc, 40, 30, max_bounce=8, n_frames=3, flags=flags)
        got = gpu_render(sc, 40, 30, max_bounce=8, n_frames=3, flags=flags, variant=V)
        assert_bitwise(got, want, "MT flags %d" % flags)


def test_moller_trumbore_mode_tolerance(cornell_scene):
    """MT vs the live hit_triangle: not the reference's image (t differs in the last bits, and
    MT accepts edge/degenerate cases hit_triangle rejects), but the same picture.  Stated
    tolerance after 64 frames at 96x72: relative mean |dRGB| <= 2% of the mean radiance and
    the mean images agree to 2% per channel."""
    ref = gpu_render(cornell_scene, 96, 72, max_bounce=8, n_frames=64)[..., :3]
    mt = gpu_render(cornell_scene, 96, 72, max_bounce=8, n_frames=64, flags=H.PT_FLAG_MOLLER_TRUMBORE)[..., :3]
    assert np.all(np.isfinite(mt))
    differ = float((mt.view(np.uint32) != ref.view(np.uint32)).any(-1).mean())
    assert differ > 0, "the MT flag did not reach the kernel"
    rel = float(np.abs(mt - ref).mean() / np.abs(ref).mean())
    print("MT: %.4f of pixels differ, relative mean |dRGB| = %.2e" % (differ, rel))
    assert rel <= 0.02
    assert np.allclose(mt.mean(axis=(0, 1)), ref.mean(axis=(0, 1)), rtol=0.02)


def test_cold_probe_launch_is_invisible(cornell_scene):
    """The first long render after an upload issues its first 2 frames as a probe launch whose
    tile costs are sorted before the remaining frames run: the image is the oracle's, and the
    same as with the adaptive order off."""
    want = O.render(cornell_scene, 48, 32, max_bounce=8, n_frames=70)
    imgs = []
    for adaptive in (1, 0):
        pt = H.PathTracer(48, 32, max_bounce=8)
        pt.set_tuning(adaptive=adaptive)
        pt.upload(cornell_scene)
        pt.render(1, 70, 0)
        imgs.append(pt.read_rgba32f())
        pt.close()
    assert_bitwise(imgs[0], want, "cold render with probe launch")
    assert_bitwise(imgs[1], want, "raster order")
