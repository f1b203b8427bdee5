"""Image-space tiling across GPUs: one process per GPU, rank r renders
rows y = r, r+G, r+2G, ... (row interleave balances sky-vs-geometry cost), and the frame
is assembled with one all-gather of the per-rank RGBA32F row blocks over RCCL/xGMI
(torch.distributed backend "nccl" is RCCL on ROCm; "gloo" for CPU tests).

The reference has no multi-GPU path; this is the build's only collective.  The gather is
bit-transparent: the assembled image equals the single-GPU render word for word, because
each pixel's RNG stream depends only on (x, y, frame) (computeShader.c:514-515).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def rows_max(height, world):
    return (height + world - 1) // world


def interleave(gathered, height):
    """gathered: (world, rows_max, W, 4) -> (height, W, 4) with row y = r + world*k."""
    world, rmax, W, C = gathered.shape
    return gathered.permute(1, 0, 2, 3).reshape(world * rmax, W, C)[:height]


def gather_image(local_rows, height, world, group=None):
    """All-gather each rank's local rows (rows_local <= rows_max, padded) and interleave.

    local_rows: tensor (rows_max, W, 4) on this rank's device (rows beyond rows_local are
    padding).  Returns the full (height, W, 4) frame on every rank.
    """
    rmax, W, C = local_rows.shape
    out = torch.empty((world * rmax, W, C), dtype=local_rows.dtype, device=local_rows.device)
    dist.all_gather_into_tensor(out, local_rows.contiguous(), group=group)
    return interleave(out.view(world, rmax, W, C), height)


_SCENE_KEYS = (("tris", 16), ("nodes", 12), ("mats", 16), ("spheres", 8))


def broadcast_scene(sb, device="cpu", src=0, group=None):
    """The scene of setupBuffers() from rank `src` to every rank (the OBJ is parsed and the
    BVH built once, not per rank).  sb: the SceneBuffers on `src`, ignored
    elsewhere.  Returns the scene dict (tris, nodes, mats, spheres, cam, n_loaded_mats) on every
    rank; tensors travel on `device` ("cuda" for RCCL, "cpu" for gloo)."""
    import numpy as np
    rank = dist.get_rank(group)
    counts = torch.zeros(5, dtype=torch.int64, device=device)
    if rank == src:
        counts[:] = torch.tensor([len(np.asarray(sb[k]).reshape(-1, c)) for k, c in _SCENE_KEYS] +
                                 [int(sb["n_loaded_mats"])], dtype=torch.int64)
    dist.broadcast(counts, src, group=group)
    n = [int(v) for v in counts.cpu()]
    out = {}
    for (k, c), m in zip(_SCENE_KEYS + (("cam", 12),), n[:4] + [1]):
        t = torch.empty((m, c), dtype=torch.float32, device=device)
        if rank == src:
            t.copy_(torch.from_numpy(np.ascontiguousarray(sb[k], np.float32).reshape(m, c)))
        if m:
            dist.broadcast(t, src, group=group)
        out[k] = t.cpu().numpy()
    out["cam"] = out["cam"].reshape(12)
    out["n_loaded_mats"] = n[4]
    return out
