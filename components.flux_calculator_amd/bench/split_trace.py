#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of bench/arm_ab.py by arm (measurement tool): the run's
grouped launches, in issue order, are assigned to the arms by the run's schedule (one
cells_atmos_group_kernel launch per fcx_run_group call); every other kernel launched between
two group launches (fix-ups) goes to the arm of the preceding group launch.

  python split_trace.py TRACE_CSV ARM_AB_JSON  -> per arm: mean group-kernel ms and the mean
  of each other kernel, over the timed blocks (warm-up launches excluded)
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    trace, res = sys.argv[1], sys.argv[2]
    line = [x for x in open(res) if x.startswith("{")][-1]
    ab = json.loads(line)
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "fcx::" in r["Kernel_Name"]]
    tags = []  # arm of every group launch, and whether it is in a timed block
    for name, n in ab["schedule"]:
        tags += [(name, n > 1)] * n
    per = defaultdict(lambda: defaultdict(list))
    gi, cur = -1, None
    for r in rows:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        kname = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "cells_atmos_group_kernel" in kname:
            gi += 1
            if gi >= len(tags):
                break
            cur = tags[gi]
            if cur[1]:
                per[cur[0]]["group: " + kname].append(dur)
        elif cur is not None and cur[1]:
            per[cur[0]][kname].append(dur)
    out = {"group_launches_in_trace": gi + 1, "group_launches_scheduled": len(tags), "arms": {}}
    for arm, ks in per.items():
        out["arms"][arm] = {k: {"mean_ms": round(sum(v) / len(v), 5), "launches": len(v)} for k, v in ks.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
