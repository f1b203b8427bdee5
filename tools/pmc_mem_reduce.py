"""Reduce tools/gpu_pmc_mem.sh output (one dir per counter group) to the per-launch counters of
the LAST render launch and the derived vector-memory figures.
python tools/pmc_mem_reduce.py gpurun_out/pmcm [more dirs...]"""
import collections
import csv
import json
import os
import sys


def last_launch(d):
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if "k_render" not in r["Kernel_Name"]:
            continue
        e = disp.setdefault(int(r["Dispatch_Id"]), collections.defaultdict(float))
        e[r["Counter_Name"]] += float(r["Counter_Value"])
    return disp[max(disp)]


def reduce(root):
    c = {}
    for g in sorted(os.listdir(root)):
        p = os.path.join(root, g)
        if os.path.isdir(p) and os.path.exists(os.path.join(p, "run_counter_collection.csv")):
            c.update(last_launch(p))
    cu = 256.0
    gui = c.get("GRBM_GUI_ACTIVE", 1.0) / 8.0
    d = {}
    if "TD_TD_BUSY_sum" in c:
        d["td_busy_per_cu"] = c["TD_TD_BUSY_sum"] / (cu * gui)
        d["td_tc_stall_frac_of_td_busy"] = c["TD_TC_STALL_sum"] / c["TD_TD_BUSY_sum"]
    if "TA_TA_BUSY_sum" in c:
        d["ta_busy_per_cu"] = c["TA_TA_BUSY_sum"] / (cu * gui)
    if "SQ_INSTS_VMEM_RD" in c:
        d["valu_busy"] = 2.0 * c["SQ_INSTS_VALU"] / (1024.0 * gui)
        d["vmem_rd_instr"] = c["SQ_INSTS_VMEM_RD"]
        if "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
            d["l1_accesses_per_vmem_instr"] = c["TCP_TOTAL_CACHE_ACCESSES_sum"] / c["SQ_INSTS_VMEM_RD"]
            d["l1_to_l2_read_frac"] = c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"]
        if "TD_TD_BUSY_sum" in c:
            d["td_cycles_per_vmem_instr"] = c["TD_TD_BUSY_sum"] / c["SQ_INSTS_VMEM_RD"]
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        d["l2_hit_rate"] = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1.0)
    return {"counters": c, "derived": d}


if __name__ == "__main__":
    out = {r: reduce(r) for r in sys.argv[1:]}
    print(json.dumps(out, indent=1, sort_keys=True))
