"""pt_group's multi-device planning on the CPU (include/pt_group.h: pt_group_plan,
pt_group_interleave_host).  A one-GPU box can never run pt_group_create's cross-device
branches (several devices, slots per device, the block table of ncclGather), so this suite
assembles frames on the host exactly as the gather does: each context's rows (y = rank +
k*world) are packed into its device's send buffer at its slot, the send buffers are
concatenated in device order (what ncclGather delivers on the root), and the host interleave
-- the index function the device kernel k_interleave_rows runs (csrc/pt_group_plan.h) --
must give back the untiled frame.  The reference has one GL context (ogl_path_trace.h:183-192)."""
import numpy as np
import pytest

import pt_host as H


def gather_on_host(frame, devices, ranks):
    """Pack, 'ncclGather' and interleave a frame split over contexts (devices[i], ranks[i])."""
    Hh, W, _ = frame.shape
    n = len(devices)
    plan = H.group_plan(devices, ranks)
    rmax = -(-Hh // n)
    nd, ms = len(plan["devices"]), plan["max_slots"]
    send = np.full((nd, ms, rmax, W, 4), np.nan, np.float32)      # padding stays NaN
    for i in range(n):
        rows = frame[ranks[i]::n]                                   # the context's accumulator
        assert rows.shape[0] == max(0, (Hh - ranks[i] + n - 1) // n)
        send[plan["dev_idx"][i], plan["slot"][i], :rows.shape[0]] = rows
    recv = send.reshape(nd * ms, rmax, W, 4)                        # ncclGather: device order
    return plan, H.group_interleave_host(recv, plan["table"], n, W, Hh)


@pytest.mark.parametrize("devices,ranks", [
    ([0, 1, 0], [2, 0, 1]),                         # 2 devices x 3 ranks, scrambled
    ([1, 0, 1, 0, 1], [4, 1, 0, 3, 2]),             # 2 devices x 5 ranks, root is device 1
    ([0, 1, 2, 3, 4, 5, 6, 7], [0, 1, 2, 3, 4, 5, 6, 7]),   # 8 devices x 1
    ([7, 6, 5, 4, 3, 2, 1, 0], [3, 7, 1, 5, 0, 2, 6, 4]),   # 8 devices, any order
    ([3, 3, 3, 3], [3, 2, 1, 0]),                   # one device, 4 contexts
    ([0, 1, 1, 1, 2, 0, 2], [6, 5, 4, 3, 2, 1, 0]), # uneven slots per device
])
@pytest.mark.parametrize("Hh", [1, 7, 53, 1080])
def test_gather_plan_reassembles_frame(devices, ranks, Hh):
    W = 24
    rng = np.random.default_rng(Hh * 31 + len(devices))
    frame = rng.random((Hh, W, 4), dtype=np.float32)
    plan, got = gather_on_host(frame, devices, ranks)
    assert plan["devices"][0] == devices[0]                         # ctxs[0]'s device is the root
    assert sorted(plan["devices"]) == sorted(set(devices))
    per_dev = [sum(1 for d in devices if d == x) for x in plan["devices"]]
    assert plan["max_slots"] == max(per_dev)
    assert np.array_equal(got.view(np.uint32), frame.view(np.uint32))


def test_plan_fields():
    p = H.group_plan([5, 9, 5, 9, 5], [1, 3, 0, 4, 2])
    assert p["devices"] == [5, 9] and p["max_slots"] == 3
    assert p["dev_idx"].tolist() == [0, 1, 0, 1, 0] and p["slot"].tolist() == [0, 0, 1, 1, 2]
    # table[rank] = dev_idx * max_slots + slot
    assert p["table"].tolist() == [1, 0, 2, 3, 4]


@pytest.mark.parametrize("ranks", [[0, 0], [0, 2], [-1, 0]])
def test_plan_refuses_bad_ranks(ranks):
    with pytest.raises(H.PTError):
        H.group_plan([0, 1], ranks)


def test_interleave_refuses_table_outside_blocks():
    with pytest.raises(H.PTError):
        H.group_interleave_host(np.zeros((2, 1, 4, 4), np.float32), np.array([0, 5], np.int32), 2, 4, 2)


def test_world8_1080p_row_blocks_match_pt_dist():
    """bench.py's torch.distributed path (pt_dist.gather_image) and the C++ group share the
    row-interleave: the same padded blocks in rank order give the same frame."""
    import torch
    import pt_dist
    Hh, W, n = 1080, 16, 8
    frame = np.random.default_rng(3).random((Hh, W, 4), dtype=np.float32)
    _, got = gather_on_host(frame, list(range(n)), list(range(n)))
    rmax = pt_dist.rows_max(Hh, n)
    blocks = torch.zeros((n, rmax, W, 4))
    for r in range(n):
        rows = torch.from_numpy(frame[r::n].copy())
        blocks[r, :rows.shape[0]] = rows
    ref = pt_dist.interleave(blocks, Hh).numpy()
    assert np.array_equal(ref.view(np.uint32), got.view(np.uint32))
    assert np.array_equal(got.view(np.uint32), frame.view(np.uint32))
