"""Reduce rocprofv3 PMC passes (tools/gpu_pmc.sh output) for the render launch.

A render launch is the state-machine kernel plus, in the frame-split mode, the k_accum_frames
pass that follows it; counters are summed over both and averaged over launches (the first,
warm-up launch dropped).  Writes profiles/<tag>_pmc.json and profiles/traffic_latest.json:
  hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024, per render launch.
The factor 2 on FETCH_SIZE is the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE
reports half the bytes of wide 16-B/lane reads; the accumulator and colour-buffer reads are
float4 per lane); WRITE_SIZE is exact for 16-B/lane stores.  Raw values are kept alongside.
"""
import collections
import csv
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


def main():
    pmc = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "pmc")
    tag = sys.argv[2] if len(sys.argv) > 2 else "latest"
    meta = dict(scene="cornell", width=1920, height=1080, chunk=1024)
    for a in sys.argv[3:]:
        k, v = a.split("=")
        meta[k] = int(v) if v.isdigit() else v
    out = dict(meta)
    per = collections.defaultdict(list)
    for name in sorted(os.listdir(pmc)):
        d = os.path.join(pmc, name)
        if not os.path.isdir(d) or not os.path.exists(os.path.join(d, "run_counter_collection.csv")):
            continue
        launches = load(d)
        # full-size launches only (a cold first render starts with a 2-frame probe launch),
        # then drop the warm-up render when possible
        top = max(sum(ms.values()) for _, ms in launches)
        launches = [(ctr, ms) for ctr, ms in launches if sum(ms.values()) >= 0.5 * top]
        for ctr, ms in (launches[1:] or launches):
            for cn, v in ctr.items():
                per[cn].append(v)
            per["launch_ms_" + name].append(sum(ms.values()))
            for kind, v in ms.items():
                per["%s_ms_%s" % (kind, name)].append(v)
    avg = {k: sum(v) / len(v) for k, v in per.items()}
    out["counters_per_launch"] = avg
    # the build these counters belong to: bench.py uses them only for this exact library
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
    if "SQ_THREAD_CYCLES_VALU" in avg:
        out["valu_active_lanes_per_instr"] = avg["SQ_THREAD_CYCLES_VALU"] / max(avg["SQ_ACTIVE_INST_VALU"], 1)
    if "SQ_INSTS_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
        # VALU pipe occupancy: a wave64 VALU op holds a SIMD-32 for 2 cycles (MI355X_MICROARCH.md);
        # GRBM_GUI_ACTIVE sums the 8 XCDs' busy clocks; 256 CUs x 4 SIMDs.
        cycles = avg["GRBM_GUI_ACTIVE"] / 8.0
        out["valu_busy_frac"] = 2.0 * avg["SQ_INSTS_VALU"] / (1024.0 * cycles)
        out["clock_ghz"] = cycles / (avg.get("launch_ms_sq2", avg.get("launch_ms_sq1", 1.0)) * 1e6)
        out["valu_instr_per_launch"] = avg["SQ_INSTS_VALU"]
        out["source"] = "profiles/%s_pmc.json (rocprofv3 --pmc passes of tools/pmc_run.py, same workload)" % tag
    if "SQ_WAVE_CYCLES" in avg and "SQ_WAIT_ANY" in avg:
        tot = avg["SQ_WAVE_CYCLES"]
        out["wave_cycle_split"] = {k: avg[k] / tot for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY") if k in avg}
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    for fn in ("%s_pmc.json" % tag, "traffic_latest.json"):
        with open(os.path.join(REPO, "profiles", fn), "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in out.items() if k != "counters_per_launch"}, indent=1))


if __name__ == "__main__":
    main()
