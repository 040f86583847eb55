#!/usr/bin/env python3
"""Baltic-size (32,768 cells) drop-in step from caller heap arrays (zero-copy transport: the
kernel reads and writes the page-locked arena over the host link) under grid caps
(FCX_OPT_MAX_BLOCKS): fewer waves, each looping over more cells, so that some waves read
while others write and the link carries both directions at once (measurement tool).

  python zc_cap_probe.py [--variant CCLM] [--caps 0,8,16,32,64,128] [--steps 300]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="CCLM")
    ap.add_argument("--cells", type=int, default=32_768)
    ap.add_argument("--caps", default="0,8,16,32,64,128")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.synthetic import build_case, inputs_for_bench

    data = inputs_for_bench(a.cells)
    caps = [int(c) for c in a.caps.split(",")]
    engines = {}
    for c in caps:
        case = build_case(a.variant, n=a.cells, T=1, data=data)
        opts = {"max_blocks": c} if c > 0 else {}
        engines[c] = (case, Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                                   averages=case.averages, options=opts or None))
    for c, (_, e) in engines.items():
        for k in range(50):
            e.step(PHASE_ALL, k * 3600)
    res = {c: [] for c in caps}
    for r in range(a.rounds):
        for c in (caps if r % 2 == 0 else caps[::-1]):
            e = engines[c][1]
            ts = []
            for k in range(a.steps):
                t0 = time.perf_counter()
                e.step(PHASE_ALL, k * 3600)
                ts.append(time.perf_counter() - t0)
            res[c] += ts
    ref = engines[caps[0]][0]
    out = {"variant": a.variant, "cells": a.cells, "steps": a.steps * a.rounds, "caps": {}}
    for c in caps:
        case = engines[c][0]
        same = all(np.array_equal(np.asarray(case.lf.field[k]), np.asarray(ref.lf.field[k])) for k in case.outputs)
        out["caps"][str(c)] = {"us_median": round(float(np.median(res[c])) * 1e6, 1),
                               "us_p90": round(float(np.percentile(res[c], 90)) * 1e6, 1), "same_bits_as_first": same}
        engines[c][1].close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
