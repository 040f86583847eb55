#!/usr/bin/env python3
"""Summary of bench/r06_t2counters.sh (measurement tool, round 6): per build, the T = 2 group
launch's registers and scratch (kernel trace), its mean duration, the SQ counters per wave
(SQ_WAVE_CYCLES and SQ_WAIT_INST_ANY count quad-cycles), and its HBM-side bytes per launch from
the request-size counters (32/64/128 x TCC_EA0_RDREQ_*B) and WRITE_SIZE (KiB).

  python t2_counter_summary.py OUTDIR > t2_counters.json      (OUTDIR/{ref,t2nopf4,t2pf4})
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

GROUP = "cells_atmos_group_kernel"


def dispatches(path):
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(path)):
        if GROUP not in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[r["Dispatch_Id"]] = r
    return per, meta


def mean(xs):
    return sum(xs) / len(xs) if xs else None


def build(d):
    tr = [r for r in csv.DictReader(open(glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))[0]))
          if GROUP in r["Kernel_Name"]]
    dur = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr)
    out = {"launches": len(tr), "vgprs": int(tr[0]["VGPR_Count"]), "sgprs": int(tr[0]["SGPR_Count"]),
           "scratch_bytes_per_lane": int(tr[0]["Scratch_Size"]), "lds_bytes": int(tr[0]["LDS_Block_Size"]),
           "median_us": round(dur[len(dur) // 2] / 1e3, 1), "mean_us": round(mean(dur) / 1e3, 1)}
    sq, _ = dispatches(os.path.join(d, "sq", "run_counter_collection.csv"))
    c = {k: mean([v[k] for v in sq.values()]) for k in next(iter(sq.values()))}
    w = c["SQ_WAVES"]
    out["sq"] = {"waves": round(w), "wave_cycles_per_wave": round(c["SQ_WAVE_CYCLES"] / w),
                 "frac_wait_inst_any": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3),
                 "busy_cycles": round(c["SQ_BUSY_CYCLES"]),
                 "per_wave": {k: round(c[k] / w, 1) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM")}}
    rd, _ = dispatches(os.path.join(d, "rdreq", "run_counter_collection.csv"))
    rb = mean([32 * v["TCC_EA0_RDREQ_32B_sum"] + 64 * v["TCC_EA0_RDREQ_64B_sum"] + 128 * v["TCC_EA0_RDREQ_128B_sum"]
               for v in rd.values()])
    wr, _ = dispatches(os.path.join(d, "write", "run_counter_collection.csv"))
    wb = mean([v["WRITE_SIZE"] * 1024 for v in wr.values()])
    out["hbm"] = {"read_bytes": round(rb), "write_bytes": round(wb), "total_bytes": round(rb + wb),
                  "read_frac_128B_requests": round(mean([128 * v["TCC_EA0_RDREQ_128B_sum"] for v in rd.values()]) / rb, 3)}
    out["group_ab"] = json.load(open(os.path.join(d, "group_ab.json")))["group"]
    return out


def main():
    top = sys.argv[1]
    res = {b: build(os.path.join(top, b)) for b in ("ref", "t2nopf4", "t2pf4") if os.path.isdir(os.path.join(top, b))}
    ref = res.get("ref")
    for b, r in res.items():
        if ref and b != "ref":
            r["vs_ref"] = {"duration": round(r["mean_us"] / ref["mean_us"] - 1, 4),
                           "hbm_bytes": round(r["hbm"]["total_bytes"] / ref["hbm"]["total_bytes"] - 1, 4),
                           "wave_cycles": round(r["sq"]["wave_cycles_per_wave"] / ref["sq"]["wave_cycles_per_wave"] - 1, 4),
                           "vmem_insts": round(r["sq"]["per_wave"]["SQ_INSTS_VMEM"] / ref["sq"]["per_wave"]["SQ_INSTS_VMEM"] - 1, 4)}
    res["_builds"] = {"ref": "the build: next-type prefetch, 3 blocks per CU (168 VGPRs)",
                      "t2nopf4": "FCX_T2_PREFETCH=0, FCX_RAVG_ATMOS_BLOCKS=4 (128 VGPRs, spills)",
                      "t2pf4": "prefetch kept, FCX_RAVG_ATMOS_BLOCKS=4 (128 VGPRs, more spills)"}
    res["_source"] = ("bench/r06_t2counters.sh: bench/group_ab.py --types 2 at 10M cells, random map, each build in "
                      "its own process; kernel trace + three --pmc passes (SQ, RDREQ sizes, WRITE_SIZE); means over "
                      "the group launches")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
