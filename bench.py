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


def pmc_for(traffic_json, lib_path, W, H, chunk, scene, world):
    """-> (PMC summary or None, why not, sha256 of the library).  The PMC figures count only
    for this exact build and workload: the pass records the sha256 of the library it
    profiled (tools/pmc_traffic.py), and a rebuilt kernel without a fresh pass gets frac =
    null -- dividing an old instruction count by a new time would not be a roofline."""
    with open(lib_path, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()
    try:
        with open(traffic_json) as fh:
            tj = json.load(fh)
    except (OSError, ValueError) as e:
        return None, "no PMC pass (%s)" % e, lib_sha
    if (tj.get("width"), tj.get("height"), tj.get("chunk"), tj.get("scene")) != (W, H, chunk, scene) or world != 1:
        return None, "PMC pass is of another workload (%s %sx%s, %s frames per launch)" % (
            tj.get("scene"), tj.get("width"), tj.get("height"), tj.get("chunk")), lib_sha
    if tj.get("lib_sha256") != lib_sha:
        return None, "PMC pass profiled another build (lib sha256 %s, this build %s)" % (
            str(tj.get("lib_sha256"))[:12], lib_sha[:12]), lib_sha
    return tj, None, lib_sha


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
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo = CPU rehearsal of the N>1 path")
    ap.add_argument("--dump-frame", default=None,
                    help="rank 0 saves the last step's assembled RGBA32F frame here (np.save; tests)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_latest.json"),
                    help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py)")
    args = ap.parse_args()

    import torch

    import pt_host
    import pt_scenes

    scene, W, H, spp, bounces, chunk, graph_launches = CONFIGS[args.config]
    W = args.width or W
    H = args.height or H
    spp = args.spp or spp
    bounces = args.bounces if args.bounces is not None else bounces
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # frames per launch: the per-GPU share of the image shrinks with N, so launches get
    # N times more frames, capped at spp (one launch tail per launch; measured: C2 on one
    # GPU runs 2.5% faster as one 1024-frame launch than as 8 of 128, and a 1080p/8 share
    # runs at the single-GPU rate with 1024-frame launches, 13% slower with 128).  The graph
    # config (C5) keeps its captured launch shape.
    if args.chunk:
        chunk = args.chunk
    elif graph_launches == 0:
        chunk = chunk * world
    chunk = min(chunk, spp)

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    ndev = max(1, torch.cuda.device_count())
    device = local_rank % ndev
    if distributed:
        import torch.distributed as dist
        import pt_dist
        if args.dist_backend == "nccl":
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")

    def barrier():
        if distributed:
            dist.barrier()

    # the scene is generated, parsed and its BVH built once, on rank 0, then broadcast
    # (pt_dist.broadcast_scene; RCCL for nccl) -- every rank renders the same arrays
    scene_dir = os.path.join(REPO, "scenes")
    sb = None
    if rank == 0:
        sb = pt_host.setupBuffers(*pt_scenes.write_scene(scene, scene_dir))
    if distributed:
        sb = pt_dist.broadcast_scene(sb, device="cuda" if args.dist_backend == "nccl" else "cpu")
    cold_ms = None
    if not args.no_cold and graph_launches == 0:
        # cold first render: a fresh context right after pt_upload_scene (raster tile order
        # until the probe launch's costs are sorted), after a tiny render on a throw-away
        # context has loaded the code object -- what one render of a new scene costs
        warm = pt_host.PathTracer(64, 32, max_bounce=bounces, device=device)
        warm.upload(sb)
        warm.render(1, 2, 0)
        warm.close()
        cold = pt_host.PathTracer(W, H, max_bounce=bounces, display_mode=1, device=device, rank=rank, world=world)
        cold.set_kernel(args.variant)
        cold.upload(sb)
        barrier()
        tc = time.perf_counter()
        for f0 in range(1, spp + 1, chunk):
            cold.render_async(f0, min(chunk, spp - (f0 - 1)), 0 if f0 == 1 else 1)
        cold.sync()
        cold_ms = (time.perf_counter() - tc) * 1e3
        cold.close()
        if distributed:
            t = torch.tensor([cold_ms], dtype=torch.float64,
                             device="cuda" if args.dist_backend == "nccl" else "cpu")
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
        rmax = pt_dist.rows_max(H, world)
        dev = "cuda" if args.dist_backend == "nccl" else "cpu"
        send = torch.zeros((rmax, W, 4), dtype=torch.float32, device=dev)
        # the rows leave the render context by a device copy in both modes (the RCCL path's
        # pt_copy_rows_device); the gloo rehearsal then stages them through host memory
        dsend = send if dev == "cuda" else torch.zeros((rmax, W, 4), dtype=torch.float32, device="cuda")

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
            if args.dist_backend != "nccl":
                send.copy_(dsend)
            img = pt_dist.gather_image(send, H, world)
            if args.dist_backend == "nccl":
                torch.cuda.synchronize()
            return img
        return None

    for _ in range(args.warmup):
        step()
    pt.timing(reset=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        img = step()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    kern_ms, n_launch = pt.timing(reset=True)
    if use_graph:
        n_launch = args.steps * replays * graph_launches      # events bracket whole replays
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    if distributed:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

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
    if distributed:
        v = torch.tensor([tot["segments"], alg_bytes], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        seg_all = float(v[0])
    else:
        seg_all = float(tot["segments"])

    ms_per_step = dt / args.steps * 1e3
    value = seg_all * args.steps / dt / 1e6
    avg_launch_ms = kern_ms / max(n_launch, 1)
    bytes_per_launch = alg_bytes / len(launches)       # this rank's launches
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9

    # Roofline.  The scene is LDS/L2-resident, so HBM does not bound the kernel (the algorithmic
    # bytes exceed the HBM peak); the bound that binds is VALU issue.  Its per-launch
    # instruction count and held clock come from a PMC pass of the same build and workload
    # (tools/gpu_pmc.sh -> tools/pmc_traffic.py -> profiles/traffic_latest.json):
    #   achieved = SQ_INSTS_VALU per launch / the live launch time (HIP events, this run)
    #   peak     = 1024 SIMDs x held clock / 2 cycles per wave64 VALU instruction
    #   busy_frac_pmc = SQ_INSTS_VALU x 2 / (1024 x GRBM_GUI_ACTIVE / 8), all from the PMC pass
    pmc, stale, lib_sha = pmc_for(args.traffic_json, pt_host.LIB_PATH, W, H, chunk, scene, world)
    hbm = {"algorithmic_gbs": round(achieved, 1), "algorithmic_frac": round(achieved / HBM_PEAK_GBS, 4),
           "algorithmic_bytes_per_launch": int(bytes_per_launch), "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    roofline = {"bound": "valu", "achieved": None, "peak": None, "unit": "G wave-VALU instr/s", "frac": None,
                "traffic": None, "avg_launch_ms": round(avg_launch_ms, 3), "n_launches": n_launch,
                "lib_sha256": lib_sha[:16]}
    if stale:
        roofline["pmc_stale"] = stale
    if pmc is not None and pmc.get("valu_instr_per_launch"):
        cnt = pmc["counters_per_launch"]
        vi = pmc["valu_instr_per_launch"]
        clk = pmc["clock_ghz"]
        roofline.update(achieved=round(vi / (avg_launch_ms * 1e-3) / 1e9, 2), peak=round(N_SIMD * clk / 2.0, 2))
        roofline["frac"] = round(roofline["achieved"] / roofline["peak"], 4)
        roofline["busy_frac_pmc"] = round(pmc["valu_busy_frac"], 4)
        roofline["clock_ghz_pmc"] = round(clk, 3)
        roofline["valu_instr_per_launch"] = vi
        roofline["valu_instr_per_segment"] = round(vi / (seg_all / len(launches)), 2)
        roofline["active_lanes_per_valu"] = round(pmc.get("valu_active_lanes_per_instr", 0.0), 2)
        if pmc.get("hbm_bytes_per_launch"):
            tb = pmc["hbm_bytes_per_launch"]
            roofline["traffic"] = int(tb)
            hbm.update(traffic_bytes_per_launch=int(tb), measured_gbs=round(tb / (avg_launch_ms * 1e-3) / 1e9, 1),
                       measured_frac=round(tb / (avg_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                       traffic_over_algorithmic=round(tb / bytes_per_launch, 2))
        roofline["source"] = pmc.get("source", "profiles/traffic_latest.json")
        if pmc.get("pmc_launch_ms"):   # the PMC pass's own launch time beside the live one
            roofline["pmc_launch_ms"] = round(pmc["pmc_launch_ms"], 3)
    roofline["hbm"] = hbm
    roofline["basis"] = ("VALU issue: achieved = PMC SQ_INSTS_VALU per launch / live avg launch time (HIP events on "
                         "the render stream); peak = 1024 SIMDs x PMC-held clock / 2; HBM kept as a secondary "
                         "field (algorithmic bytes, SURVEY.md §8(d), and PMC-measured traffic)")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_lib
        threads, share = cpu_share()
        if args.cpu_threads:
            threads = args.cpu_threads
        t1 = time.perf_counter()
        _, ccnt = oracle_lib.render(sb, W, H, max_bounce=bounces, n_frames=args.cpu_spp, threads=threads,
                                    counters=True)
        cdt = time.perf_counter() - t1
        cpu = {"value": round(float(ccnt[0]) / cdt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
               "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "cpu_share": share,
               "sample": "CPU restatement of computeShader.c semantics (oracle/pt_oracle.cpp, -O3, %d threads = this "
                         "process's CPU share), same scene/camera/bounces at %dx%d, frames 1..%d (%d segments, "
                         "%.2f s); ms/frame = %.1f" % (threads, W, H, args.cpu_spp, int(ccnt[0]), cdt,
                                                        cdt * 1e3 / args.cpu_spp)}

    if args.dump_frame and rank == 0:
        import numpy as np
        np.save(args.dump_frame, img.cpu().numpy() if img is not None else pt.read_rgba32f())
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": "%s: %s %dx%d, %d spp (frames 1..%d), %d bounces (i<=%d), AA+sky+sphere on%s"
                       % (args.config, scene, W, H, spp, spp, bounces, bounces,
                          ", hipGraph sample loop" if use_graph else ""),
                       "scene": scene, "width": W, "height": H, "spp": spp, "max_bounce": bounces,
                       "frames_per_launch": chunk, "kernel_variant": args.variant,
                       "parallelism": ("row-interleaved image split x%d + %s all-gather"
                                       % (world, "RCCL" if args.dist_backend == "nccl" else "gloo"))
                       if world > 1 else "single GPU"},
            "ms_per_frame": round(ms_per_step / spp, 4),
            "cold_ms_per_step": None if cold_ms is None else round(cold_ms, 3),
            "segments_per_step": int(seg_all),
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    pt.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
