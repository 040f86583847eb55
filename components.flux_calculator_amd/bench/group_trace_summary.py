#!/usr/bin/env python3
"""Mean duration of the timed group launches of each bench.py workload in a rocprofv3 kernel
trace of `bench.py --no-cpu --e2e 0` (measurement tool).

The bench's workloads run one after the other: main (random map, 10M cells), other_map
(periodic), config5_fp32 (the fp32 engine, round 6), config4 (40M cells), each as build + cold + warm-up + event-timed per-engine
block + one more block + the timed steps, the timed ones being the LAST `steps` group
launches of the workload.  A workload's group launches are the run of consecutive
cells_atmos_group_kernel dispatches of one kernel name and grid size (the 0.5-s idle gap before the cold step
and the event-timed per-engine block stay inside it; building the next workload takes longer).

  python group_trace_summary.py TRACE_CSV BENCH_LINE_JSON [--steps 200] > summary.json
"""
import csv
import json
import sys


def main():
    trace, line = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 200
    rows = sorted((r for r in csv.DictReader(open(trace)) if "cells_atmos_group_kernel" in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    segs, key = [], None
    for r in rows:
        k = (r["Kernel_Name"], r["Grid_Size_X"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        gap = segs and (int(r["Start_Timestamp"]) - segs[-1]["end"]) / 1e6
        if k != key or gap > 1000.0:  # a new workload: other kernel or grid, or 1 s without group launches
            segs.append({"kernel": r["Kernel_Name"].split("(")[0].replace("void ", ""), "grid": int(r["Grid_Size_X"]),
                         "durs": []})
            key = k
        segs[-1]["durs"].append(dur)
        segs[-1]["end"] = int(r["End_Timestamp"])
    bench = json.loads([x for x in open(line) if x.startswith("{")][-1])
    names = ["main"] + [k for k in ("other_map", "config5_fp32", "config4") if k in bench]
    out = {"source": trace, "rule": f"mean of the last {steps} group launches of each workload (its timed steps)",
           "workloads": []}
    for i, s in enumerate(segs):
        t = s["durs"][-steps:]
        out["workloads"].append({"workload": names[i] if i < len(names) else f"w{i}", "kernel": s["kernel"],
                                 "grid_threads": s["grid"], "launches": len(s["durs"]), "timed": len(t),
                                 "mean_ms": round(sum(t) / len(t), 4)})
    out["bench_line_mean_kernel_ms"] = bench["roofline"]["mean_kernel_ms"]
    out["bench_line_alg_bytes"] = bench["roofline"]["alg_bytes_per_launch"]
    m = out["workloads"][0]["mean_ms"]
    out["main_GBps_from_trace"] = round(bench["roofline"]["alg_bytes_per_launch"] / (m * 1e-3) / 1e9, 1)
    out["main_frac_from_trace"] = round(out["main_GBps_from_trace"] / 8000.0, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
