"""Summary of tools/gpu_lds_attr.sh: LDS instructions, active cycles and bank-conflict cycles of
C2's render launch per diagnostic build, and by difference the share of the walk image (what
no build moves), the leaf phase's triangle quads (cur - dtri) and the shading records
(cur - dshade).  python3 tools/lds_attr.py [gpurun_out/ldsattr] > profiles/r06_lds_attribution.json
"""
import collections
import csv
import json
import os
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ldsattr"
KEYS = ("SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VALU")


def last_render(build):
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(os.path.join(D, build, "run_counter_collection.csv"))):
        if "k_render_sm" in r["Kernel_Name"]:
            disp[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    kt = [k for k in csv.DictReader(open(os.path.join(D, build, "run_kernel_trace.csv"))) if "k_render_sm" in k["Kernel_Name"]]
    v = {k: disp[max(disp)][k] for k in KEYS}
    v["ms"] = (int(kt[-1]["End_Timestamp"]) - int(kt[-1]["Start_Timestamp"])) / 1e6
    return v


b = {n: last_render(n) for n in ("cur", "dtri", "dshade", "dboth")}
cur = b["cur"]
parts = {"triangles (leaf phase)": {k: cur[k] - b["dtri"][k] for k in KEYS[:3]},
         "materials + spheres (shading)": {k: cur[k] - b["dshade"][k] for k in KEYS[:3]}}
parts["walk image and the rest"] = {k: b["dboth"][k] for k in KEYS[:3]}
for p in parts.values():
    p["conflict_frac_of_active"] = p["SQ_LDS_BANK_CONFLICT"] / p["SQ_LDS_IDX_ACTIVE"]
    p["share_of_conflicts"] = p["SQ_LDS_BANK_CONFLICT"] / cur["SQ_LDS_BANK_CONFLICT"]
    p["cycles_per_instr"] = p["SQ_LDS_IDX_ACTIVE"] / p["SQ_INSTS_LDS"]
json.dump({"workload": "C2 Cornell 1920x1080, one 1024-frame launch (tools/pmc_run.py --config C2 --launches 1)",
           "builds": b, "attribution": parts,
           "note": "dtri / dshade read those records from HBM instead of LDS; the differences attribute the "
                   "LDS counters (the dboth launch: 'walk image and the rest')"}, sys.stdout, indent=1)
print()
