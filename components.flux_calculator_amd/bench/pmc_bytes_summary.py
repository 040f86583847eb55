#!/usr/bin/env python3
"""Summary of pmc_bytes.sh output: per kernel name, the mean read bytes per launch from the
request-size counters (32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B), the request mix,
and WRITE_SIZE bytes per launch.   pmc_bytes_summary.py OUTDIR [OUTDIR ...]"""
import collections
import csv
import json
import os
import sys


def per_dispatch(path):
    d = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        k = r["Dispatch_Id"]
        d[k][r["Counter_Name"]] = d[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
    return d, names


def summarize(out):
    res = {}
    rd, names = per_dispatch(os.path.join(out, "rdreq", "run_counter_collection.csv"))
    wr, wnames = per_dispatch(os.path.join(out, "write", "run_counter_collection.csv"))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for k, c in rd.items():
        n = names[k].split("(")[0][:90]
        b = 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0) + \
            128 * c.get("TCC_EA0_RDREQ_128B_sum", 0)
        agg[n]["read_bytes"].append(b)
        agg[n]["req"].append(c.get("TCC_EA0_RDREQ_sum", 0))
        for s in ("32B", "64B", "128B"):
            agg[n]["req_" + s].append(c.get(f"TCC_EA0_RDREQ_{s}_sum", 0))
    for k, c in wr.items():
        n = wnames[k].split("(")[0][:90]
        agg[n]["write_bytes"].append(c.get("WRITE_SIZE", 0) * 1024)
    for n, v in agg.items():
        res[n] = {k: round(sum(x) / len(x)) for k, x in v.items() if x}
        res[n]["launches"] = len(v["read_bytes"]) if v["read_bytes"] else len(v["write_bytes"])
    return res


if __name__ == "__main__":
    print(json.dumps({o: summarize(o) for o in sys.argv[1:]}, indent=1))
