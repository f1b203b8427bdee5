"""bench.py's N>1 path with the HIP kernels: 2, 3 and 8 ranks on device 0 over
gloo (8 ranks on C4's 249k-triangle scene, the configuration BASELINE sends to 8 GPUs) run the bench's own pt_dist.broadcast_scene -> pt_copy_rows_device -> pt_dist.gather_image
path; rank 0's assembled frame must equal one context's render bit for bit (each pixel's RNG
stream depends only on (x, y, frame), computeShader.c:514-515).  RCCL cannot put two ranks on
one GPU, so the 8-GPU RCCL run stays the driver's; tests/test_dist.py checks the gather on CPU.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import pt_host as H
from test_gpu_parity import assert_bitwise

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,config", [(2, "C2"), (3, "C3"), (8, "C4")])
def test_bench_ranks_gloo_one_gpu(tmp_path, cornell_scene, world, config):
    W, Hh, spp, chunk = 160, 90, 6, 3
    out = str(tmp_path / "frame.npy")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(world),
           "--config", config, "--dist-backend", "gloo", "--width", str(W), "--height", str(Hh), "--spp", str(spp),
           "--chunk", str(chunk), "--steps", "1", "--warmup", "1", "--no-cold", "--no-cpu-baseline",
           "--dump-frame", out]
    tj = None
    if world == 2:
        # rank 0's share carries a roofline when a PMC summary of that share (same build, world
        # recorded) is given: a synthetic one here -- the plumbing, not the counters
        import hashlib
        import json
        with open(H.LIB_PATH, "rb") as fh:
            sha = hashlib.sha256(fh.read()).hexdigest()
        tj = str(tmp_path / "C2_w2.json")
        with open(tj, "w") as fh:
            json.dump({"scene": "cornell", "width": W, "height": Hh, "chunk": chunk, "world": 2, "lib_sha256": sha,
                       "clock_ghz": 2.4, "counters_per_launch": {"SQ_INSTS_VALU": 1e6, "GRBM_GUI_ACTIVE": 8e6,
                                                                 "SQ_WAVE_CYCLES": 1e6}}, fh)
        cmd += ["--traffic-json", tj]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    import json
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    # rank 0 checks the assembled frame of the timed steps against the oracle
    assert line["parity"]["mismatches"] == 0 and line["parity"]["words"] > 0, line["parity"]
    if tj:
        rf = line["roofline"]
        assert rf["frac"] is not None and rf["bound"] == "valu" and "rank 0" in rf["share"], rf
    img = np.load(out)
    import pt_scenes
    name = {"C3": "bunny", "C4": "sponza"}.get(config)
    sc = cornell_scene if name is None else H.setupBuffers(*pt_scenes.write_scene(name, os.path.join(REPO, "scenes")))
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.upload(sc)
    pt.render(1, spp, 0)
    want = pt.read_rgba32f()
    pt.close()
    assert img.shape == want.shape
    assert_bitwise(img, want, "%d-rank bench frame vs one context" % world)


def test_bench_share_proxy_line(tmp_path):
    """bench.py --share-of N: one process renders rank 0's share of an N-way row split with no
    collective (the per-GPU proxy of the configs BASELINE sends to 8 GPUs); the line says so
    and its frame rows are rank 0's (y = 0 mod N)."""
    import json
    W, Hh, spp = 96, 40, 4
    out = str(tmp_path / "frame.npy")
    cmd = [sys.executable, "bench.py", "--config", "C2", "--share-of", "4", "--width", str(W), "--height", str(Hh),
           "--spp", str(spp), "--chunk", "2", "--steps", "1", "--warmup", "1", "--no-cold", "--no-cpu-baseline",
           "--dump-frame", out]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["share_proxy"]["of"] == 4 and line["share_proxy"]["rows"] == 10
    assert line["value"] > 0 and "share proxy" in line["config"]["parallelism"]
    img = np.load(out)                          # rank 0's rows_local x W accumulation
    pt = H.PathTracer(W, Hh, max_bounce=8)
    import pt_scenes
    pt.upload(H.setupBuffers(*pt_scenes.write_scene("cornell", os.path.join(REPO, "scenes"))))
    pt.render(1, spp, 0)
    want = pt.read_rgba32f()
    pt.close()
    assert_bitwise(img, want[0::4], "share proxy rows vs one context")


@pytest.mark.parametrize("config", ["C2", "C4"])
def test_bench_rccl_leg_world_one(tmp_path, cornell_scene, config):
    """The RCCL leg of bench.py rehearsed on one GPU (--force-dist at world 1): the nccl
    process group with device_id, pt_dist.broadcast_scene on cuda tensors, pt_copy_rows_device
    into a cuda send buffer and all_gather_into_tensor -- the calls the driver's 8-GPU run
    makes.  The line names RCCL's backend, its timed-image parity check against the oracle
    passes, and the dumped frame equals one context's render bit for bit."""
    import json
    W, Hh, spp, chunk = 160, 90, 6, 3
    out = str(tmp_path / "frame.npy")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
           "--config", config, "--dist-backend", "nccl", "--force-dist", "--width", str(W), "--height", str(Hh),
           "--spp", str(spp), "--chunk", str(chunk), "--steps", "2", "--warmup", "1", "--no-cold",
           "--no-cpu-baseline", "--parity-pixels", "300", "--dump-frame", out]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    pg = line["config"]["process_group"]
    assert pg["backend"] == "nccl" and pg["world"] == 1 and pg["rehearsal"] is True, pg
    assert line["parity"]["mismatches"] == 0 and line["parity"]["words"] == 1200, line["parity"]
    assert line["value"] > 0
    img = np.load(out)
    import pt_scenes
    sc = cornell_scene if config == "C2" else H.setupBuffers(*pt_scenes.write_scene("sponza", os.path.join(REPO, "scenes")))
    pt = H.PathTracer(W, Hh, max_bounce=8)
    pt.upload(sc)
    pt.render(1, spp, 0)
    want = pt.read_rgba32f()
    pt.close()
    assert img.shape == want.shape
    assert_bitwise(img, want, "RCCL world-1 bench frame vs one context")
