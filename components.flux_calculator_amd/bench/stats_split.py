#!/usr/bin/env python3
"""Per-phase kernel statistics of one `rocprofv3 --kernel-trace` run of bench.py.

A default bench line times three workloads one after the other: the main one (`value`,
`roofline`), the `other_map` sub-object and the `config4` sub-object.  rocprof's
`kernel_stats.csv` averages every dispatch of a kernel name over all three, so it cannot be
compared with the roofline's mean kernel time.  This tool splits the kernel trace of the same
run into the three phases (a phase ends where the dispatches of all libfcx kernels pause for more
than --gap seconds: the next workload's construction; the bench's 0.5 s cold-step gap stays
inside a phase; phases after the third, e.g. the e2e sub-object's, are labelled afterN) and reports, per phase and kernel, the mean duration of the last `steps`
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
    disp = []
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"]
        if "fcx::" in name:
            disp.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0]))
    disp.sort()
    # phases over ALL fcx dispatches (a map without crossings, a halo launch and the pipelined
    # e2e chunks run differently named kernels, so per-name pauses would not line up)
    group, gi = [], 0
    for i, (s0, _, _) in enumerate(disp):
        if i and (s0 - disp[i - 1][1]) * 1e-9 > a.gap:
            gi += 1
        group.append(gi)
    labels = {g: (phases[g] if g < len(phases) else f"after{g}") for g in set(group)}
    per = defaultdict(lambda: defaultdict(list))
    for (s0, e0, name), g in zip(disp, group):
        per[name][labels[g]].append(e0 - s0)
    out = {"steps": steps, "phases": phases, "gap_s": a.gap, "kernels": {}}
    for name, byp in sorted(per.items()):
        out["kernels"][name] = {lab: {"dispatches": len(d), "timed_mean_us": round(sum(d[-steps:]) / len(d[-steps:]) / 1e3, 2)}
                                for lab, d in byp.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
