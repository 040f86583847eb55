#!/usr/bin/env python3
"""Per-wave SQ counters of the group launches from two rocprofv3 --pmc passes
(bench/r05_pmc.sh: <dir>/sq and <dir>/sq2), means over the group-kernel dispatches
(measurement tool; the same rule as profiles/r04/sq_counters.json).

  python sq_summary.py DIR [DIR ...] > sq_counters.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def passes(d):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, pass file, dispatch) -> counter -> value
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "cells_atmos_group_kernel" not in r["Kernel_Name"]:
                continue
            per[(r["Kernel_Name"].split("(")[0].replace("void ", ""), f, r["Dispatch_Id"])][r["Counter_Name"]] += \
                float(r["Counter_Value"])
    tot = defaultdict(lambda: defaultdict(list))
    for (k, f, _), c in per.items():
        for name, v in c.items():
            tot[k][name].append(v)
    return {k: {n: sum(v) / len(v) for n, v in c.items()} for k, c in tot.items()}


def main():
    out = {}
    for d in sys.argv[1:]:
        for k, c in passes(d).items():
            w = c.get("SQ_WAVES", 0) or 1
            cyc = c.get("SQ_WAVE_CYCLES", 0) or 1
            out[f"{os.path.basename(d.rstrip('/'))}: {k}"] = {
                "waves": round(c.get("SQ_WAVES", 0)),
                "wave_cycles_per_wave": round(cyc / w),
                "frac_wait_any": round(c.get("SQ_WAIT_ANY", 0) / cyc, 3),
                "frac_wait_inst_any": round(c.get("SQ_WAIT_INST_ANY", 0) / cyc, 3),
                "frac_active_any": round(c.get("SQ_ACTIVE_INST_ANY", 0) / cyc, 3),
                "frac_active_valu": round(c.get("SQ_ACTIVE_INST_VALU", 0) / cyc, 3),
                "frac_active_lds": round(c.get("SQ_ACTIVE_INST_LDS", 0) / cyc, 3),
                "per_wave": {n: round(c.get(n, 0) / w, 1) for n in (
                    "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                    "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS")}}
    out["_source"] = ("bench/r05_pmc.sh: rocprofv3 --pmc, two passes of 8 SQ counters per workload (bench.py "
                      "--steps 20 --warmup 5, main workload only); means over the group launches")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
