#!/usr/bin/env python3
"""Per-phase kernel statistics of one `rocprofv3 --kernel-trace` run of bench.py.

A default bench line times three workloads one after the other: the main one (`value`,
`roofline`), the `other_map` sub-object and the `config4` sub-object.  rocprof's
`kernel_stats.csv` averages every dispatch of a kernel name over all three, so it cannot be
compared with the roofline's mean kernel time.  This tool splits the kernel trace of the same
run into the three phases (a phase ends where a kernel's dispatches pause for more than
--gap seconds: the next workload's construction; the bench's 0.5 s cold-step gap stays
inside a phase) and reports, per phase and kernel, the mean duration of the last `steps`
dispatches, the timed steps (bench.py measure(): plan step, cold step, warm-up, timed steps).

  stats_split.py RUN_DIR/run_kernel_trace.csv BENCH.json [--gap 1.0]
"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench_json")
    ap.add_argument("--gap", type=float, default=1.0)
    a = ap.parse_args()
    bench = json.load(open(a.bench_json))
    steps = int(bench["steps"])
    phases = ["main"] + (["other_map"] if "other_map" in bench else []) + (["config4"] if "config4" in bench else [])
    per = defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"]
        if "fcx::" not in name:
            continue
        per[name.split("(")[0]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = {"steps": steps, "phases": phases, "kernels": {}}
    for name, d in sorted(per.items()):
        d.sort()
        groups, cur = [], [d[0]]
        for x, y in zip(d, d[1:]):
            if (y[0] - x[1]) * 1e-9 > a.gap:
                groups.append(cur)
                cur = []
            cur.append(y)
        groups.append(cur)
        res = {}
        for i, g in enumerate(groups):
            label = phases[i] if len(groups) == len(phases) else f"phase{i}"
            timed = g[-steps:]
            res[label] = {"dispatches": len(g), "timed_mean_us": round(sum(e - s for s, e in timed) / len(timed) / 1e3, 2)}
        out["kernels"][name] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
