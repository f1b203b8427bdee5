"""Reduce rocprofv3 PMC passes (tools/gpu_pmc.sh output) for the render launch of one bench
configuration.

python tools/pmc_traffic.py gpurun_out/pmc/C3 r05a C3 [world=N]

A render launch is the state-machine kernel plus, in the frame-split mode, the k_accum_frames
pass that follows it; counters are summed over both and averaged over launches (the first,
warm-up launch dropped).  Writes profiles/pmc/<config>[_wN].json (what bench.py reads) and the
per-round copy profiles/<tag>_pmc_<config>[_wN].json:
  hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024, per render launch.
The factor 2 on FETCH_SIZE is the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE
reports half the bytes of wide 16-B/lane reads; the accumulator and colour-buffer reads are
float4 per lane); WRITE_SIZE is exact for 16-B/lane stores.  Raw values are kept alongside.
The summary records the sha256 of the library it profiled: bench.py uses it only for that
build and workload (bench.pmc_for).
"""
import collections
import csv
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def load(d):
    """-> list of launches: (summed counters, {kernel kind: duration ms})."""
    path = os.path.join(d, "run_counter_collection.csv")
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        kind = "render" if "k_render" in name else ("accum" if "k_accum_frames" in name else None)
        if kind is None:
            continue
        key = int(r["Dispatch_Id"])
        e = disp.setdefault(key, {"kind": kind, "ctr": collections.defaultdict(float), "ms": 0.0})
        e["ctr"][r["Counter_Name"]] += float(r["Counter_Value"])
        e["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    launches = []
    for key in sorted(disp):
        e = disp[key]
        if e["kind"] == "render" or not launches:
            launches.append((collections.defaultdict(float), {}))
        ctr, ms = launches[-1]
        for cn, v in e["ctr"].items():
            ctr[cn] += v
        ms[e["kind"]] = ms.get(e["kind"], 0.0) + e["ms"]
    return launches


def reduce(pmc, meta):
    out = dict(meta)
    per = collections.defaultdict(list)
    for name in sorted(os.listdir(pmc)):
        d = os.path.join(pmc, name)
        if not os.path.isdir(d) or not os.path.exists(os.path.join(d, "run_counter_collection.csv")):
            continue
        launches = load(d)
        # full-size launches only, then drop the warm-up render when possible
        top = max(sum(ms.values()) for _, ms in launches)
        launches = [(ctr, ms) for ctr, ms in launches if sum(ms.values()) >= 0.5 * top]
        for ctr, ms in (launches[1:] or launches):
            for cn, v in ctr.items():
                per[cn].append(v)
            per["launch_ms_" + name].append(sum(ms.values()))
            if "GRBM_GUI_ACTIVE" in ctr:       # this pass's own clock (its counters, its launch time)
                per["clock_ghz_" + name].append(ctr["GRBM_GUI_ACTIVE"] / 8.0 / (sum(ms.values()) * 1e6))
            for kind, v in ms.items():
                per["%s_ms_%s" % (kind, name)].append(v)
    avg = {k: sum(v) / len(v) for k, v in per.items()}
    out["counters_per_launch"] = avg
    lib = os.path.join(REPO, "opengl-path-tracing_amd", "build", "libptrace.so")
    with open(lib, "rb") as fh:
        out["lib_sha256"] = hashlib.sha256(fh.read()).hexdigest()
    ms = [v for k, v in avg.items() if k.startswith("launch_ms_")]
    if ms:
        out["pmc_launch_ms"] = sum(ms) / len(ms)
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        out["fetch_bytes_raw"] = avg["FETCH_SIZE"] * 1024
        out["write_bytes"] = avg["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = 2 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024
    # GRBM_GUI_ACTIVE sums the 8 XCDs' busy clocks; each pass that records it gives its own
    # clock (its cycles over its own launch time), and the passes' clocks are averaged
    clocks = [v for k, v in avg.items() if k.startswith("clock_ghz_")]
    if "GRBM_GUI_ACTIVE" in avg and not clocks:
        print("pmc_traffic: GRBM_GUI_ACTIVE without a launch time; no clock", file=sys.stderr)
    elif "GRBM_GUI_ACTIVE" not in avg:
        print("pmc_traffic: no pass recorded GRBM_GUI_ACTIVE; no clock, no busy fractions", file=sys.stderr)
    if clocks:
        out["clock_ghz"] = sum(clocks) / len(clocks)
        # cycles of one average launch at that clock
        cycles = out["clock_ghz"] * 1e6 * out.get("pmc_launch_ms", 0.0)
        if "SQ_INSTS_VALU" in avg:
            # a wave64 VALU op holds a SIMD-32 for 2 cycles (MI355X_MICROARCH.md); 1024 SIMDs
            out["valu_busy_frac"] = 2.0 * avg["SQ_INSTS_VALU"] / (1024.0 * cycles)
            out["valu_instr_per_launch"] = avg["SQ_INSTS_VALU"]
        if "TD_TD_BUSY_sum" in avg:
            out["td_busy_frac"] = avg["TD_TD_BUSY_sum"] / (256.0 * cycles)
        if "SQ_WAVE_CYCLES" in avg:
            out["waves_per_simd"] = 4.0 * avg["SQ_WAVE_CYCLES"] / (1024.0 * cycles)
    if "SQ_THREAD_CYCLES_VALU" in avg:
        out["valu_active_lanes_per_instr"] = avg["SQ_THREAD_CYCLES_VALU"] / max(avg["SQ_ACTIVE_INST_VALU"], 1)
    if "TCC_HIT_sum" in avg:
        out["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"], 1.0)
    if "SQ_WAVE_CYCLES" in avg and "SQ_WAIT_ANY" in avg:
        tot = avg["SQ_WAVE_CYCLES"]
        out["wave_cycle_split"] = {k: avg[k] / tot for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY") if k in avg}
    return out


def main():
    pmc, tag, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    import bench
    scene, W, H, spp, bounces, chunk0, graph = bench.CONFIGS[cfg]
    meta = dict(config=cfg, scene=scene, width=W, height=H, world=1)
    for a in sys.argv[4:]:
        k, v = a.split("=")
        meta[k] = int(v) if v.isdigit() else v
    meta["chunk"] = min(meta.get("chunk") or (chunk0 * meta["world"] if graph == 0 else chunk0), spp)
    out = reduce(pmc, meta)
    name = cfg if meta["world"] == 1 else "%s_w%d" % (cfg, meta["world"])
    out["source"] = "profiles/%s_pmc_%s.json (rocprofv3 --pmc passes of tools/pmc_run.py, same workload)" % (tag, name)
    os.makedirs(os.path.join(REPO, "profiles", "pmc"), exist_ok=True)
    for fn in (os.path.join("profiles", "%s_pmc_%s.json" % (tag, name)), os.path.join("profiles", "pmc", "%s.json" % name)):
        with open(os.path.join(REPO, fn), "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in out.items() if k != "counters_per_launch"}, indent=1))


if __name__ == "__main__":
    main()
