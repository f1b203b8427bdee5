"""Collect tools/gpu_configs.sh's bench lines into one JSON (profiles/<tag>_configs.json):
per config value / ms per frame, and for the share proxies the single-GPU rate on rank 0's
share beside the same config's full-image rate on one GPU (share / full = how well one GPU's
share of an N-way split keeps the chip busy; not a scaling measurement).
  python tools/configs_summary.py gpurun_out/cfg"""
import glob
import json
import os
import sys

d = sys.argv[1]
out = {"note": "bench.py lines on one MI355X; *_shareN = rank 0 of an N-way row split rendered alone on one GPU "
               "(bench.py --share-of N): a per-GPU proxy, not an N-GPU measurement"}
lines = {}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    name = os.path.basename(f)[:-5]
    if name == "configs":
        continue
    try:
        lines[name] = json.load(open(f))
    except ValueError:
        continue
for name, L in lines.items():
    e = {"value_mrays_s": L["value"], "ms_per_frame": L["ms_per_frame"], "ms_per_step": L["ms_per_step"],
         "workload": L["config"]["workload"], "frames_per_launch": L["config"]["frames_per_launch"],
         "roofline_frac": L["roofline"].get("frac"), "bound": L["roofline"].get("bound")}
    if "share_proxy" in L:
        e["share_of"] = L["share_proxy"]["of"]
        e["rows"] = L["share_proxy"]["rows"]
        base = name.split("_share")[0]
        full = lines.get(base) or (lines.get("C2") if base == "C2" else None)
        if full:
            e["share_over_full_image"] = round(L["value"] / full["value"], 4)
    out[name] = e
print(json.dumps(out, indent=1, sort_keys=True))
