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


def kernel_key(name):
    """(variant, atmos fused, dtype) of a cells kernel, or None for any other kernel."""
    m = re.search(r"cells_kernel<(\d), (true|false), (\d), (true|false), (double|float)", name)
    if m:
        return VARIANTS[m.group(3)], 0, "f64" if m.group(5) == "double" else "f32"
    m = re.search(r"cells_atmos_kernel<(\d), (double|float), (\d), (true|false)", name)
    if m:
        return VARIANTS[m.group(3)], 1, "f64" if m.group(2) == "double" else "f32"
    m = re.search(r"cells_atmos_group_kernel<(\d), (double|float)", name)
    if m:  # the variants' fused passes in one launch (fcx_run_group)
        return "GROUP", 1, "f64" if m.group(2) == "double" else "f32"
    return None


def read_counter(d, name):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r.get("Counter_Name") == name]
    per = defaultdict(list)
    for r in rows:
        k = kernel_key(r["Kernel_Name"])
        if k is not None:
            per[k].append(float(r["Counter_Value"]))
    return per


def read_request_bytes(d):
    """Read bytes per launch from the request-size counters (bench/pmc_bytes.sh):
    32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B, exact on gfx950 (no calibration)."""
    disp = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            disp[(f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            names[(f, r["Dispatch_Id"])] = r["Kernel_Name"]
    per = defaultdict(list)
    for key, c in disp.items():
        k = kernel_key(names[key])
        if k is not None and "TCC_EA0_RDREQ_128B_sum" in c:
            per[k].append(32 * c["TCC_EA0_RDREQ_32B_sum"] + 64 * c["TCC_EA0_RDREQ_64B_sum"]
                          + 128 * c["TCC_EA0_RDREQ_128B_sum"])
    return per


def traffic_key(variant, cells, types, bias, atmos, dtype):
    """profiles/traffic.json key (bench.py looks the dominant kernel up by it)."""
    return f"{variant}:{cells}:T{types}:bias{int(bias)}:atmos{int(atmos)}:{dtype}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--types", type=int, default=1)
    ap.add_argument("--bias", type=int, default=0)
    ap.add_argument("--source", default=None,
                    help="where the PMC run's outputs are kept (e.g. profiles/r02/pmc_t1), stamped per key")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.dirname(os.path.abspath(__file__)))), "profiles", "traffic.json"))
    a = ap.parse_args()
    rdreq = os.path.isdir(os.path.join(a.dir, "rdreq"))  # bench/pmc_bytes.sh layout
    if rdreq:
        fetch = read_request_bytes(os.path.join(a.dir, "rdreq"))
    else:
        fetch = read_counter(os.path.join(a.dir, "fetch"), "FETCH_SIZE")
    write = read_counter(os.path.join(a.dir, "write"), "WRITE_SIZE")
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    for k in sorted(set(fetch) & set(write)):
        v, atm, dt = k
        if rdreq:
            f = sum(fetch[k]) / len(fetch[k])
            how = ("rocprofv3 --pmc TCC_EA0_RDREQ_{32B,64B,128B}_sum and --pmc WRITE_SIZE passes "
                   "(separate runs), read bytes = 32/64/128 x requests of each size + WRITE_SIZE")
        else:
            # KiB -> B, gfx950 x2 read correction (calibrated for 16 B/lane streaming reads; the
            # fused kernel's 8 B/lane atmosphere-index reads are 4 of its ~150 B/cell)
            f = sum(fetch[k]) / len(fetch[k]) * 1024 * 2
            how = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (separate runs), "
                   "FETCH_SIZE x2 (gfx950) + WRITE_SIZE")
        w = sum(write[k]) / len(write[k]) * 1024
        key = traffic_key(v, a.cells, a.types, a.bias, atm, dt)
        out[key] = round(f + w)
        out.setdefault("_sources", {})[key] = f"{a.source or a.dir}: {how}, mean over {len(fetch[k])} launches"
        print(key, "read", round(f / a.cells, 2), "B/cell", "write", round(w / a.cells, 2), "B/cell",
              "launches", len(fetch[k]))
    json.dump(out, open(a.out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
