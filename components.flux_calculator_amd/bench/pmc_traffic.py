#!/usr/bin/env python3
"""Per-launch HBM traffic of the cells kernels from rocprofv3 PMC passes.

Collect (separate passes, MI355X_MICROARCH.md 'rocprofv3 PMC slots'):
  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d D/fetch -o run -- python bench.py ...
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d D/write -o run -- python bench.py ...
then: python pmc_traffic.py D --cells N  -> profiles/traffic.json entries.

Units and gfx950 corrections (MI355X_MICROARCH.md section HBM): FETCH_SIZE and WRITE_SIZE
are KiB; on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide (16 B/lane)
coalesced streaming read, which is the access of the cells kernels, so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

VARIANTS = {"1": "CCLM", "2": "MOM5", "3": "RCO", "0": "generic"}


def read_counter(d, name):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r.get("Counter_Name") == name]
    per = defaultdict(list)
    for r in rows:
        m = re.search(r"cells_kernel<(\d), (true|false), (\d), (true|false)>", r["Kernel_Name"])
        if not m:
            continue
        per[VARIANTS[m.group(3)]].append(float(r["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--types", type=int, default=1)
    ap.add_argument("--bias", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.dirname(os.path.abspath(__file__)))), "profiles", "traffic.json"))
    a = ap.parse_args()
    fetch = read_counter(os.path.join(a.dir, "fetch"), "FETCH_SIZE")
    write = read_counter(os.path.join(a.dir, "write"), "WRITE_SIZE")
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    for v in sorted(set(fetch) & set(write)):
        f = sum(fetch[v]) / len(fetch[v]) * 1024 * 2  # KiB -> B, gfx950 x2 read correction
        w = sum(write[v]) / len(write[v]) * 1024
        key = f"{v}:{a.cells}:T{a.types}:bias{a.bias}"
        out[key] = round(f + w)
        print(key, "read", round(f / a.cells, 2), "B/cell", "write", round(w / a.cells, 2), "B/cell",
              "launches", len(fetch[v]))
    json.dump(out, open(a.out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
