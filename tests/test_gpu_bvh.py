"""The GPU BVH builder (pt_bvh_build_gpu) against the host builder, whose
node arrays are themselves pinned to the oracle's literal restatement of buildSAHTree
(tests/test_scene.py): the same node numbering, bounds, leaf indices and links, word for
word, on the reference's shipped scenes, the benchmark stand-ins and edge cases."""
import time

import numpy as np
import pytest

import pt_host as H
import pt_scenes

pytestmark = pytest.mark.gpu


def same(tris):
    want = H.buildSAHTree(tris)
    got = H.buildSAHTree(tris, device=0)
    assert got.shape == want.shape
    bad = np.argwhere(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, "%d words differ, first at node %s" % (len(bad), bad[:3].tolist())
    return got


@pytest.mark.parametrize("name", ["cornell", "bunny", "sponza"])
def test_benchmark_scenes(name, tmp_path):
    sb = H.setupBuffers(*pt_scenes.write_scene(name, str(tmp_path)))
    got = same(sb["tris"])
    assert np.array_equal(got.view(np.uint32), np.asarray(sb["nodes"], np.float32).view(np.uint32))


def test_shipped_ship_scene(ship_scene):
    same(ship_scene["tris"])


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 61, 62, 121, 1000])
def test_sizes_and_duplicates(n):
    rng = np.random.default_rng(n)
    t = np.zeros((n, 16), np.float32)
    t[:, :12] = rng.normal(size=(n, 12)).astype(np.float32)
    t[:, [3, 7, 11]] = 0
    t[:, 12] = rng.integers(0, 4, n)
    if n >= 4:
        t[n // 2] = t[0]                      # duplicate triangle: leaf index = first occurrence
        t[1, :12] = np.round(t[1, :12])       # integer coordinates: centroid ties
        t[2, :12] = np.round(t[2, :12])
    same(t)


def test_ties_signed_zeros_and_degenerate_boxes():
    """Equal centroids everywhere (stable order decides), -0 coordinates, zero-area boxes
    (no finite split cost: the median fallback)."""
    n = 40
    t = np.zeros((n, 16), np.float32)
    t[:, 0:3] = [0.0, 1.0, 2.0]
    t[:, 4:7] = [0.0, 1.0, 2.0]
    t[:, 8:11] = [0.0, 1.0, 2.0]
    t[::3, 0] = -0.0
    t[:, 12] = np.arange(n)
    same(t)
    q = np.zeros((n, 16), np.float32)           # flat quads in z = 0 with -0 / +0 mixed
    rng = np.random.default_rng(5)
    q[:, [0, 1, 4, 5, 8, 9]] = rng.integers(-3, 4, (n, 6)).astype(np.float32)
    q[::2, [2, 6, 10]] = -0.0
    same(q)


def test_gpu_builder_is_faster_on_sponza(tmp_path):
    tris, _ = H.load_vertex_data(*pt_scenes.write_scene("sponza", str(tmp_path)))
    H.buildSAHTree(tris[:1000], device=0)                    # warm-up (module load)
    t0 = time.perf_counter()
    H.buildSAHTree(tris)
    cpu = time.perf_counter() - t0
    t0 = time.perf_counter()
    H.buildSAHTree(tris, device=0)
    gpu = time.perf_counter() - t0
    print("sponza stand-in (%d tris): host %.3f s, GPU %.3f s" % (len(tris), cpu, gpu))
    assert gpu < cpu


def test_cli_gpu_bvh_same_image(tmp_path):
    """ptrace --gpu-bvh renders the same image as the host-built tree."""
    import subprocess
    from test_gpu_cli import EXE, read_pfm
    obj, mtl = pt_scenes.write_scene("cornell", str(tmp_path))
    outs = []
    for extra in ([], ["--gpu-bvh"]):
        pfm = str(tmp_path / ("x%d.pfm" % len(outs)))
        r = subprocess.run([EXE, obj, mtl, "--width", "48", "--height", "32", "--spp", "3", "--bounces", "8",
                            "--pfm", pfm, "--ppm", str(tmp_path / "x.ppm")] + extra,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        outs.append(read_pfm(pfm))
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
