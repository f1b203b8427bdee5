#!/usr/bin/env python3
"""Benchmark of the MI355X path-tracing hot path (BASELINE.json metric:
"Mrays/sec + ms/frame @1920x1080, 8 bounces, 1/2/4/8 MI355X").

Default workload = config C2: the Cornell box (36 tris + the reference's
metal sphere), 1920x1080, 8 bounces (loop i <= 8), frames 1..1024 with accumulate=0 on
frame 1.  One *step* = one full progressive render of `spp` frames, issued as
ceil(spp/chunk) fused launches (C5: replays of a captured hipGraph), plus for N>1 the
RCCL all-gather that assembles the row-interleaved frame.  Scene and accumulator are
resident in HBM before timing starts.

value = ray segments (calculateRayCollision calls, computeShader.c:450) of all ranks /
max-over-ranks wall time, in Mrays/s.  Segment counts come from an untimed counting pass
over the same frames (reference traversal semantics; identical image).

The default run (C2 on one GPU) also times the global-memory configs C3 and C4 (2 steps each)
and reports them under "secondary", each with its own roofline.

Every line carries its own parity check (`parity`): after the timed region rank 0 renders
sampled pixels of the timed image (frames 1..spp, the assembled frame at N > 1) with the CPU
oracle (test infrastructure, never timed) and counts the words that differ; on one GPU the
frames of the cpu_baseline sample are also re-rendered on the timed context and compared in
full with the oracle image that leg computes.  --force-dist takes the N > 1 path (process
group, scene broadcast, device row copy, all-gather) at world size 1.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5]
N>1:   python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "opengl-path-tracing_amd")
sys.path.insert(0, PKG)

METRIC = "Mrays/sec + ms/frame @1920×1080, 8 bounces, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
N_SIMD = 1024           # 256 CUs x 4 SIMDs; a wave64 VALU instruction holds a SIMD-32 for 2 cycles
N_CU = 256
WAVES_PER_SIMD_PEAK = 8  # wave slots per SIMD (the occupancy peak)
PMC_DIR = os.path.join(REPO, "profiles", "pmc")

# scene, W, H, spp, bounces, frames per launch, graph launches/replay
CONFIGS = {
    "C2": ("cornell", 1920, 1080, 1024, 8, 1024, 0),
    "C3": ("bunny", 1920, 1080, 256, 8, 256, 0),
    "C4": ("sponza", 1920, 1080, 256, 8, 256, 0),
    "C5": ("cornell", 3840, 2160, 4096, 8, 256, 8),     # 2 replays of 8 x 256 frames
}


def algorithmic_bytes(cnt, pixels, first_launch_plain):
    """40 B/node visit + 36 B/tri test + 16 B/sphere test + 52 B/hit,
    plus 32 B per pixel per launch for the accumulator read+write (16 B when the launch
    starts with accumulate=0 and only writes)."""
    b = 40 * cnt["node_visits"] + 36 * cnt["tri_tests"] + 16 * cnt["sphere_tests"] + 52 * cnt["hits"]
    return b + pixels * (16 if first_launch_plain else 32)


def cpu_share():
    """-> (threads, description): the CPUs this process may run on -- its affinity mask, capped
    by a cgroup v2 cpu.max quota when one is set (os.cpu_count() counts the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    desc = "affinity %d" % n
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            lim = max(1, int(int(q) // int(per)))
            desc += ", cgroup quota %s/%s = %d" % (q, per, lim)
            n = min(n, lim)
    except (OSError, ValueError):
        pass
    return n, desc


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_path(config, world):
    """The PMC summary bench.py reads for a workload: tools/pmc_traffic.py writes
    profiles/pmc/<config>[_w<N>].json (per-rank share at N > 1) beside its per-round copy."""
    return os.path.join(PMC_DIR, "%s%s.json" % (config, "" if world == 1 else "_w%d" % world))


def pmc_for(traffic_json, lib_path, W, H, chunk, scene, world):
    """-> (PMC summary or None, why not, sha256 of the library).  The PMC figures count only
    for this exact build and workload: the pass records the sha256 of the library it
    profiled (tools/pmc_traffic.py), and a rebuilt kernel without a fresh pass gets frac =
    null -- dividing an old instruction count by a new time would not be a roofline.  At
    N > 1 the workload is one rank's share (rank 0 of the row split, frames per launch as
    launched), so rank 0's line carries the roofline of its own share."""
    with open(lib_path, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()
    try:
        with open(traffic_json) as fh:
            tj = json.load(fh)
    except (OSError, ValueError) as e:
        return None, "no PMC pass (%s)" % e, lib_sha
    if (tj.get("width"), tj.get("height"), tj.get("chunk"), tj.get("scene"), tj.get("world", 1)) != (W, H, chunk, scene,
                                                                                                      world):
        return None, "PMC pass is of another workload (%s %sx%s, %s frames per launch, world %s)" % (
            tj.get("scene"), tj.get("width"), tj.get("height"), tj.get("chunk"), tj.get("world", 1)), lib_sha
    if tj.get("lib_sha256") != lib_sha:
        return None, "PMC pass profiled another build (lib sha256 %s, this build %s)" % (
            str(tj.get("lib_sha256"))[:12], lib_sha[:12]), lib_sha
    return tj, None, lib_sha


def roofline_from(pmc, stale, lib_sha, avg_launch_ms, n_launch, segments_per_launch, alg_bytes_per_launch):
    """Roofline of the render launch from a PMC summary of the same build and workload.
    Two issue-side bounds, both utilisations of a unit every CU has one of (per SIMD for VALU):
      valu    achieved = SQ_INSTS_VALU per launch / live launch time; peak = 1024 SIMDs x clock / 2
              (a wave64 VALU instruction holds a SIMD-32 for 2 cycles)
      texture achieved = TD_TD_BUSY cycles per launch (summed over CUs) / live launch time;
              peak = 256 CUs x clock (the texture-data unit that returns every vector-memory
              load; the global-memory walk's scattered gathers keep it busy).  Busy includes
              cycles stalled on L1 (TD_TC_STALL): `stall_frac` and `unstalled_frac` say how much
    `bound` is the one with the larger fraction, the texture unit ranked by its unstalled
    fraction (its busy figure is mostly stall on the global walk).  HBM stays a secondary field: the scene is
    LDS / L2 / MALL-resident, and the algorithmic bytes are mostly LDS and
    L1 reads.  Occupancy: resident waves per SIMD (SQ_WAVE_CYCLES is counted in quad-cycles on
    gfx950) against the 8 wave slots."""
    t = avg_launch_ms * 1e-3
    hbm = {"algorithmic_gbs": round(alg_bytes_per_launch / t / 1e9, 1),
           "algorithmic_frac": round(alg_bytes_per_launch / t / 1e9 / HBM_PEAK_GBS, 4),
           "algorithmic_bytes_per_launch": int(alg_bytes_per_launch), "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    r = {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
         "avg_launch_ms": round(avg_launch_ms, 3), "n_launches": n_launch, "lib_sha256": lib_sha[:16]}
    if stale:
        r["pmc_stale"] = stale
    if pmc is not None:
        c = pmc["counters_per_launch"]
        clk = pmc.get("clock_ghz")     # None when no pass recorded GRBM_GUI_ACTIVE: no peaks
        cands = {}
        if c.get("SQ_INSTS_VALU") and clk:
            a = c["SQ_INSTS_VALU"] / t / 1e9
            cands["valu"] = {"achieved": round(a, 2), "peak": round(N_SIMD * clk / 2.0, 2), "unit": "G wave-VALU instr/s",
                             "per_segment": round(c["SQ_INSTS_VALU"] / segments_per_launch, 2)}
        if c.get("TD_TD_BUSY_sum") and clk:
            a = c["TD_TD_BUSY_sum"] / t / 1e9
            cands["texture"] = {"achieved": round(a, 2), "peak": round(N_CU * clk, 2), "unit": "G TD-busy cycles/s",
                                "per_segment": round(c["TD_TD_BUSY_sum"] / segments_per_launch, 2)}
        for k, v in cands.items():
            v["frac"] = round(v["achieved"] / v["peak"], 4)
        # TD busy cycles include the cycles the unit sits stalled on L1 (TD_TC_STALL): only the
        # rest is data-return work, and that unstalled share is what the bound is chosen on
        rank_frac = {k: v["frac"] for k, v in cands.items()}
        if "texture" in cands and c.get("TD_TC_STALL_sum"):
            stall = c["TD_TC_STALL_sum"] / c["TD_TD_BUSY_sum"]
            cands["texture"]["stall_frac"] = round(stall, 4)
            cands["texture"]["unstalled_frac"] = round(cands["texture"]["frac"] * (1.0 - stall), 4)
            rank_frac["texture"] = cands["texture"]["unstalled_frac"]
        if cands:
            b = max(cands, key=lambda k: rank_frac[k])
            r.update(bound=b, achieved=cands[b]["achieved"], peak=cands[b]["peak"], unit=cands[b]["unit"],
                     frac=cands[b]["frac"])
            r["bounds"] = cands
        r["clock_ghz_pmc"] = round(clk, 3) if clk else None
        if c.get("SQ_WAVE_CYCLES") and c.get("GRBM_GUI_ACTIVE"):
            w = 4.0 * c["SQ_WAVE_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8.0 * N_SIMD)
            r["occupancy"] = {"waves_per_simd": round(w, 2), "peak": WAVES_PER_SIMD_PEAK,
                              "frac": round(w / WAVES_PER_SIMD_PEAK, 4)}
        if c.get("SQ_ACTIVE_INST_VALU") and c.get("SQ_THREAD_CYCLES_VALU"):
            r["active_lanes_per_valu"] = round(c["SQ_THREAD_CYCLES_VALU"] / c["SQ_ACTIVE_INST_VALU"], 2)
        mem = {}
        if c.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
            mem["l1_accesses_per_segment"] = round(c["TCP_TOTAL_CACHE_ACCESSES_sum"] / segments_per_launch, 2)
        if c.get("TCP_TCC_READ_REQ_sum"):
            mem["l1_to_l2_per_segment"] = round(c["TCP_TCC_READ_REQ_sum"] / segments_per_launch, 2)
        if c.get("SQ_INSTS_VMEM_RD"):
            mem["vmem_load_instr_per_segment"] = round(c["SQ_INSTS_VMEM_RD"] / segments_per_launch, 3)
            if c.get("TD_TD_BUSY_sum"):
                mem["td_cycles_per_vmem_instr"] = round(c["TD_TD_BUSY_sum"] / c["SQ_INSTS_VMEM_RD"], 1)
        if c.get("TD_TC_STALL_sum") and c.get("TD_TD_BUSY_sum"):
            mem["td_stalled_on_l1_frac"] = round(c["TD_TC_STALL_sum"] / c["TD_TD_BUSY_sum"], 3)
        if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
            mem["l2_hit_rate"] = round(c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1.0), 4)
        if mem:
            r["memory_pipe"] = mem
        if pmc.get("hbm_bytes_per_launch"):
            tb = pmc["hbm_bytes_per_launch"]
            r["traffic"] = int(tb)
            hbm.update(traffic_bytes_per_launch=int(tb), measured_gbs=round(tb / t / 1e9, 1),
                       measured_frac=round(tb / t / 1e9 / HBM_PEAK_GBS, 4),
                       traffic_over_algorithmic=round(tb / alg_bytes_per_launch, 2))
        r["source"] = pmc.get("source")
        if pmc.get("pmc_launch_ms"):   # the PMC pass's own launch time beside the live one
            r["pmc_launch_ms"] = round(pmc["pmc_launch_ms"], 3)
    r["hbm"] = hbm
    r["basis"] = ("achieved = PMC count per launch (SQ_INSTS_VALU or TD_TD_BUSY_sum) / live avg launch time "
                  "(HIP events on the render stream); peak = 1024 SIMDs x clock / 2 (VALU) or 256 CUs x clock "
                  "(texture-data unit), clock held in the PMC pass; HBM kept as a secondary field")
    return r


def parity_pixels_for(spp, requested):
    """Pixels of the timed image checked against the oracle: about 16 M oracle pixel-frames
    (C2: 16384 pixels x 1024 frames, about 1.5 s on a 16-CPU share), 1024..16384."""
    if requested is not None:
        return max(0, int(requested))
    return int(min(16384, max(1024, (1 << 24) // max(spp, 1))))


def check_timed_image(img, sb, W, H, spp, bounces, row0, stride, n_pix, seed, threads):
    """Parity of the image the timed steps left in the accumulator: every step renders frames
    1..spp with accumulate = 0 on frame 1 (computeShader.c:505-554, :548-551), so the image is
    that of spp reference dispatches.  n_pix pixels drawn (seeded) from the rows this image
    holds (global row y = row0 + k * stride for local row k) are rendered by the CPU oracle
    (test infrastructure, after the timed region) and compared word for word."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    rows = img.shape[0]
    rng = np.random.default_rng(seed)
    n_pix = min(n_pix, rows * W)
    flat = rng.choice(rows * W, size=n_pix, replace=False)
    ky, xs = flat // W, flat % W
    ys = row0 + ky * stride
    t0 = time.perf_counter()
    want = oracle_lib.render_pixels(sb, W, H, xs, ys, max_bounce=bounces, n_frames=spp, threads=threads)
    dt = time.perf_counter() - t0
    got = np.ascontiguousarray(img[ky, xs], np.float32)
    mism = int(np.count_nonzero(got.view(np.uint32) != want.view(np.uint32)))
    return {"kind": "timed image, sampled pixels vs CPU oracle", "frames": "1..%d" % spp, "pixels": int(n_pix),
            "words": int(4 * n_pix), "mismatches": mism, "seed": int(seed), "oracle_s": round(dt, 2)}


def measure(cfg, args, ctx, steps, warmup, cold=True, W=None, H=None, spp=None, bounces=None, chunk=None,
            dump=False, parity_pixels=0, full_frames=0):
    """One configuration on this rank: scene (rank 0 builds it, N > 1 broadcasts), optional
    cold first render, `warmup` untimed steps, `steps` timed steps (barrier + synchronize on
    both sides, max over ranks), an untimed counting pass over the same frames, and the
    roofline from the PMC summary of this build and per-rank workload.  After the timed
    region, rank 0 checks `parity_pixels` sampled pixels of the timed image against the CPU
    oracle, and with `full_frames` re-renders frames 1..full_frames on the same context for a
    full-frame comparison with the cpu_baseline leg's oracle image."""
    import torch
    import pt_host
    import pt_scenes
    world, rank, device, distributed = ctx["world"], ctx["rank"], ctx["device"], ctx["distributed"]
    dist, backend = ctx.get("dist"), args.dist_backend
    scene, W0, H0, spp0, b0, chunk0, graph_launches = CONFIGS[cfg]
    W, H, spp = W or W0, H or H0, spp or spp0
    bounces = b0 if bounces is None else bounces
    # frames per launch: the per-GPU share of the image shrinks with N, so launches get N times
    # more frames, capped at spp (one launch tail per launch; measured: C2 on one GPU runs 2.5%
    # faster as one 1024-frame launch than as 8 of 128, and a 1080p/8 share runs at the
    # single-GPU rate with 1024-frame launches, 13% slower with 128).  The graph config (C5)
    # keeps its captured launch shape.
    if not chunk:
        chunk = chunk0 * world if graph_launches == 0 else chunk0
    chunk = min(chunk, spp)
    coll_dev = "cuda" if backend == "nccl" else "cpu"

    def barrier():
        if distributed:
            dist.barrier()

    # the scene is generated, parsed and its BVH built once, on rank 0, then broadcast
    # (pt_dist.broadcast_scene; RCCL for nccl) -- every rank renders the same arrays
    sb = None
    if rank == 0:
        sb = pt_host.setupBuffers(*pt_scenes.write_scene(scene, os.path.join(REPO, "scenes")))
    if distributed:
        import pt_dist
        sb = pt_dist.broadcast_scene(sb, device=coll_dev)
    cold_ms = None
    if cold and graph_launches == 0:
        # cold first render: a fresh context right after pt_upload_scene (raster tile order
        # until the probe launch's costs are sorted), after a tiny render on a throw-away
        # context has loaded the code object -- what one render of a new scene costs
        warm = pt_host.PathTracer(64, 32, max_bounce=bounces, device=device)
        warm.upload(sb)
        warm.render(1, 2, 0)
        warm.close()
        c0 = pt_host.PathTracer(W, H, max_bounce=bounces, display_mode=1, device=device, rank=rank, world=world)
        c0.set_kernel(args.variant)
        c0.upload(sb)
        barrier()
        tc = time.perf_counter()
        for f0 in range(1, spp + 1, chunk):
            c0.render_async(f0, min(chunk, spp - (f0 - 1)), 0 if f0 == 1 else 1)
        c0.sync()
        cold_ms = (time.perf_counter() - tc) * 1e3
        c0.close()
        if distributed:
            t = torch.tensor([cold_ms], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            cold_ms = float(t.item())
    pt = pt_host.PathTracer(W, H, max_bounce=bounces, display_mode=1, device=device, rank=rank, world=world)
    pt.set_kernel(args.variant)
    pt.upload(sb)
    launches = [(f0, min(chunk, spp - (f0 - 1))) for f0 in range(1, spp + 1, chunk)]
    use_graph = graph_launches > 0 and spp % (chunk * graph_launches) == 0
    if use_graph:
        pt.progressive_setup(chunk, graph_launches)
        replays = spp // (chunk * graph_launches)

    if distributed:
        import pt_dist
        rmax = pt_dist.rows_max(H, world)
        send = torch.zeros((rmax, W, 4), dtype=torch.float32, device=coll_dev)
        # the rows leave the render context by a device copy in both modes (the RCCL path's
        # pt_copy_rows_device); the gloo rehearsal then stages them through host memory
        dsend = send if coll_dev == "cuda" else torch.zeros((rmax, W, 4), dtype=torch.float32, device="cuda")

    def step():
        if use_graph:
            pt.progressive_reset(1)
            pt.progressive_run(replays, sync=False)
        else:
            for f0, n in launches:
                pt.render_async(f0, n, 0 if f0 == 1 else 1)
        pt.sync()
        if distributed:
            pt.copy_rows_device(dsend.data_ptr(), pt.rows_local * W * 16)
            if backend != "nccl":
                send.copy_(dsend)
            img = pt_dist.gather_image(send, H, world)
            if backend == "nccl":
                torch.cuda.synchronize()
            return img
        return None

    for _ in range(warmup):
        step()
    pt.timing(reset=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    img = None
    for _ in range(steps):
        img = step()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    kern_ms, n_launch = pt.timing(reset=True)
    if use_graph:
        n_launch = steps * replays * graph_launches      # events bracket whole replays
    if distributed:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # the image the timed steps produced (N > 1: the assembled frame; otherwise this
    # context's rows, y = rank + k * world), kept for the parity check and --dump-frame
    timed_img = None
    if rank == 0 and (parity_pixels or dump):
        timed_img = img.cpu().numpy() if img is not None else pt.read_rgba32f()
    parity = None
    if rank == 0 and parity_pixels and steps > 0:
        full = img is not None
        parity = check_timed_image(timed_img, sb, W, H, spp, bounces, 0 if full else pt.row0,
                                   1 if full else pt.row_stride, parity_pixels,
                                   0x5EED + sum(map(ord, cfg)), cpu_share()[0])

    # untimed counting pass over the same frames: exact reference-semantics work counts
    pt.set_counting(True)
    tot = dict(segments=0, node_visits=0, tri_tests=0, sphere_tests=0, hits=0)
    alg_bytes = 0
    for f0, n in launches:
        pt.render(f0, n, 0 if f0 == 1 else 1)
        _, cnt = pt.stats()
        for k in tot:
            tot[k] += cnt[k]
        alg_bytes += algorithmic_bytes(cnt, pt.rows_local * W, f0 == 1)
    pt.set_counting(False)
    seg_rank = float(tot["segments"])
    if distributed:
        v = torch.tensor([tot["segments"], alg_bytes], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        seg_all = float(v[0])
    else:
        seg_all = seg_rank
    avg_launch_ms = kern_ms / max(n_launch, 1)
    pmc_json = args.traffic_json if (args.traffic_json and cfg == args.config) else pmc_path(cfg, world)
    pmc, stale, lib_sha = pmc_for(pmc_json, pt_host.LIB_PATH, W, H, chunk, scene, world)
    roofline = roofline_from(pmc, stale, lib_sha, avg_launch_ms, n_launch, seg_rank / len(launches),
                             alg_bytes / len(launches))
    frame = timed_img if dump else None
    full_img = None
    if full_frames and rank == 0 and world == 1:
        # frames 1..full_frames on the timed context (its tuning, learned tile order and
        # scratch), for the word-for-word comparison with the cpu_baseline leg's oracle image
        pt.render(1, full_frames, 0)
        full_img = pt.read_rgba32f()
    rows_local = pt.rows_local
    pt.close()
    ms_per_step = dt / steps * 1e3
    return {
        "cfg": cfg, "scene": scene, "W": W, "H": H, "spp": spp, "bounces": bounces, "chunk": chunk,
        "use_graph": use_graph, "value": seg_all * steps / dt / 1e6, "ms_per_step": ms_per_step,
        "ms_per_frame": ms_per_step / spp, "cold_ms": cold_ms, "segments": seg_all, "roofline": roofline,
        "sb": sb, "frame": frame, "rows_local": rows_local, "parity": parity, "full_img": full_img,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--chunk", type=int, default=None, help="frames fused per kernel launch")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--bounces", type=int, default=None)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--cpu-spp", type=int, default=20,
                    help="spp of the bounded CPU-baseline sample (20: about 10 s on a 16-CPU share)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold first-render measurement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--secondary", default=None,
                    help="comma list of configs timed after the headline (default: C3,C4 for a one-GPU C2 "
                         "run, none otherwise; 'none' to skip)")
    ap.add_argument("--secondary-steps", type=int, default=2)
    ap.add_argument("--share-of", type=int, default=0,
                    help="one process renders rank 0's share of an N-way row split (its frames per launch "
                         "too) with no collective: the per-GPU share proxy of an N-GPU run (not a scaling "
                         "measurement)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo = CPU rehearsal of the N>1 path")
    ap.add_argument("--dump-frame", default=None,
                    help="rank 0 saves the last step's assembled RGBA32F frame here (np.save; tests)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary for the headline config (default profiles/pmc/<config>[_wN].json, "
                         "tools/pmc_traffic.py)")
    ap.add_argument("--parity-pixels", type=int, default=None,
                    help="pixels of each timed image checked against the CPU oracle after the timed region "
                         "(default: about 4 M oracle pixel-frames, 512..4096; 0 = skip)")
    ap.add_argument("--force-dist", action="store_true",
                    help="take the N>1 path (process group, scene broadcast, device row copy, all-gather) "
                         "even at world size 1: a one-GPU rehearsal of the RCCL leg")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1 or args.force_dist
    if distributed and args.share_of > 1:
        raise SystemExit("--share-of is a one-process proxy; do not combine it with torch.distributed.run")
    if distributed and world == 1:
        # a world-1 process group launched without torch.distributed.run: a loopback rendezvous
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            import socket
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
            s.close()
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    ndev = max(1, torch.cuda.device_count())
    device = local_rank % ndev
    if args.share_of > 1:
        world = args.share_of
    ctx = dict(world=world, rank=rank, device=device, distributed=distributed)
    if distributed:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
        ctx["dist"] = dist
        ctx["backend"] = dist.get_backend()

    spp_head = args.spp or CONFIGS[args.config][3]
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
    m = measure(args.config, args, ctx, args.steps, args.warmup, cold=not args.no_cold, W=args.width,
                H=args.height, spp=args.spp, bounces=args.bounces, chunk=args.chunk, dump=bool(args.dump_frame),
                parity_pixels=parity_pixels_for(spp_head, args.parity_pixels),
                full_frames=args.cpu_spp if want_cpu and args.parity_pixels != 0 else 0)
    W, H, spp, bounces, scene = m["W"], m["H"], m["spp"], m["bounces"], m["scene"]

    sec_cfgs = []
    if args.secondary is None:
        if args.config == "C2" and world == 1 and not any((args.width, args.height, args.spp, args.chunk)):
            sec_cfgs = ["C3", "C4"]
    elif args.secondary != "none":
        sec_cfgs = [c for c in args.secondary.split(",") if c]
    secondary = []
    for c in sec_cfgs:
        s = measure(c, args, ctx, args.secondary_steps, 1, cold=False,
                    parity_pixels=parity_pixels_for(CONFIGS[c][3], args.parity_pixels))
        secondary.append({
            "config": c, "workload": "%s: %s %dx%d, %d spp in launches of %d frames, %d bounces" % (
                c, s["scene"], s["W"], s["H"], s["spp"], s["chunk"], s["bounces"]),
            "value": round(s["value"], 3), "unit": "Mrays/s", "steps": args.secondary_steps, "warmup": 1,
            "ms_per_step": round(s["ms_per_step"], 3), "ms_per_frame": round(s["ms_per_frame"], 4),
            "segments_per_step": int(s["segments"]), "roofline": s["roofline"], "parity": s["parity"]})

    cpu = None
    full_parity = None
    if want_cpu:
        import numpy as np
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_lib
        threads, share = cpu_share()
        if args.cpu_threads:
            threads = args.cpu_threads
        t1 = time.perf_counter()
        cimg, ccnt = oracle_lib.render(m["sb"], W, H, max_bounce=bounces, n_frames=args.cpu_spp, threads=threads,
                                       counters=True)
        cdt = time.perf_counter() - t1
        if m["full_img"] is not None:
            # the oracle image of the timed baseline sample, word for word against the GPU's
            # frames 1..cpu_spp on the timed context
            g = np.ascontiguousarray(m["full_img"], np.float32)
            full_parity = {"kind": "full frame vs the cpu_baseline leg's oracle image", "frames": "1..%d" % args.cpu_spp,
                           "pixels": int(W * H), "words": int(g.size),
                           "mismatches": int(np.count_nonzero(g.view(np.uint32) != cimg.view(np.uint32)))}
        cpu = {"value": round(float(ccnt[0]) / cdt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
               "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "cpu_share": share,
               "sample": "CPU restatement of computeShader.c semantics (oracle/pt_oracle.cpp, -O3, %d threads = this "
                         "process's CPU share), same scene/camera/bounces at %dx%d, frames 1..%d (%d segments, "
                         "%.2f s); ms/frame = %.1f" % (threads, W, H, args.cpu_spp, int(ccnt[0]), cdt,
                                                        cdt * 1e3 / args.cpu_spp)}

    if args.dump_frame and rank == 0:
        import numpy as np
        np.save(args.dump_frame, m["frame"])
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(m["value"], 3), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(m["ms_per_step"], 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": "%s: %s %dx%d, %d spp (frames 1..%d), %d bounces (i<=%d), AA+sky+sphere on%s"
                       % (args.config, scene, W, H, spp, spp, bounces, bounces,
                          ", hipGraph sample loop" if m["use_graph"] else ""),
                       "scene": scene, "width": W, "height": H, "spp": spp, "max_bounce": bounces,
                       "frames_per_launch": m["chunk"], "kernel_variant": args.variant,
                       "parallelism": ("row-interleaved image split x%d + %s all-gather"
                                       % (world, "RCCL" if args.dist_backend == "nccl" else "gloo"))
                       if world > 1 else "single GPU"},
            "ms_per_frame": round(m["ms_per_frame"], 4),
            "cold_ms_per_step": None if m["cold_ms"] is None else round(m["cold_ms"], 3),
            "segments_per_step": int(m["segments"]),
            "roofline": m["roofline"],
            "cpu_baseline": cpu,
            "parity": None,
            "secondary": secondary,
        }
        checks = [p for p in (m["parity"], full_parity) if p]
        if checks:
            line["parity"] = {"words": sum(p["words"] for p in checks),
                              "mismatches": sum(p["mismatches"] for p in checks),
                              "checks": checks, "oracle": "oracle/pt_oracle.cpp (CPU restatement, test infrastructure)"}
        if distributed:
            line["config"]["process_group"] = {"backend": ctx["backend"], "world": world,
                                               "rehearsal": bool(args.force_dist and world == 1)}
        if world > 1:
            line["roofline"]["share"] = "rank 0's share: rows y = 0 mod %d, %d rows" % (world, m["rows_local"])
        if args.share_of > 1:   # a proxy line: this GPU's rate on rank 0's share, n_gpus stays 1
            line["n_gpus"] = 1
            line["share_proxy"] = {"of": world, "rows": m["rows_local"], "note": (
                "one GPU rendering rank 0's share of a %d-way row split (frames per launch x%d); value is this "
                "GPU's rate, not an N-GPU measurement" % (world, world))}
            line["config"]["parallelism"] = "share proxy: rank 0 of %d, no collective" % world
        print(json.dumps(line), flush=True)
    if distributed:
        ctx["dist"].destroy_process_group()


if __name__ == "__main__":
    main()
