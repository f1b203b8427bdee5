"""Multi-GPU path on CPU: world_size-2 gloo run of the row split + all-gather assembly
(pt_dist.gather_image, the code bench.py uses over RCCL).  Each rank renders its own rows
with the oracle (the GPU kernels are exercised for the same partition by the -m gpu
partition-invariance test); the gathered frame must equal the single-process render bit
for bit (any partition is bit-identical)."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

import oracle_lib as O
import pt_dist

W, H, SPP, MB = 40, 27, 2, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sc, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank 0 holds the scene; the others receive it (bench.py's broadcast)
    got = pt_dist.broadcast_scene(sc if rank == 0 else None)
    for k in ("tris", "nodes", "mats", "spheres", "cam"):
        assert np.array_equal(np.asarray(got[k]).view(np.uint32), np.asarray(sc[k], np.float32).view(np.uint32)), k
    assert got["n_loaded_mats"] == sc["n_loaded_mats"]
    sc = got
    rows = np.arange(rank, H, world)
    ys, xs = np.meshgrid(rows, np.arange(W), indexing="ij")
    px = O.render_pixels(sc, W, H, xs.reshape(-1), ys.reshape(-1), max_bounce=MB, n_frames=SPP, threads=2)
    rmax = pt_dist.rows_max(H, world)
    local = torch.zeros((rmax, W, 4), dtype=torch.float32)
    local[: len(rows)] = torch.from_numpy(px.reshape(len(rows), W, 4))
    img = pt_dist.gather_image(local, H, world)
    if rank == 0:
        out.put(img.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


def _run(world, sc):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sc, q)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return img


def test_gloo_two_rank_gather_is_bit_identical(cornell_scene):
    sc = {k: np.asarray(v) for k, v in cornell_scene.items()}
    sc["n_loaded_mats"] = int(cornell_scene["n_loaded_mats"])
    full = O.render(sc, W, H, max_bounce=MB, n_frames=SPP)
    img = _run(2, sc)
    assert np.array_equal(img.view(np.uint32), full.view(np.uint32))


def test_interleave_layout():
    g = torch.arange(3 * 4 * 2 * 4, dtype=torch.float32).view(3, 4, 2, 4)   # world 3, rows_max 4
    img = pt_dist.interleave(g, 10)
    for y in range(10):
        assert torch.equal(img[y], g[y % 3, y // 3])
