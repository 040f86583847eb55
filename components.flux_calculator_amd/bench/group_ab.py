#!/usr/bin/env python3
"""fcx_run_group against one launch per engine, in ONE process over the SAME engines and
arrays (measurement tool): blocks of steps alternate between the two, each block timed with
a HIP event pair on the engines' stream, after a warm-up of device work.  Same placement and
clock state for both, so the difference is the launch structure.

  python group_ab.py [--cells 10000000] [--types 1] [--precision f64] [--rounds 8]
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
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--types", type=int, default=1)
    ap.add_argument("--precision", choices=("f64", "f32"), default="f64")
    ap.add_argument("--atmos-map", choices=("random", "periodic"), default="random")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20, help="steps per block")
    ap.add_argument("--variants", default="CCLM,MOM5,RCO")
    ap.add_argument("--lib", default=None, help="another libfcx build (A/B of the group kernel)")
    a = ap.parse_args()
    import torch
    if a.lib:
        os.environ["FCX_LIBRARY"] = a.lib
    from fcx.workload import Workload

    wl = Workload(a.cells, 0, 1, variants=tuple(a.variants.split(",")), types=a.types, precision=a.precision,
                  atmos=True, atmos_map=a.atmos_map)
    s = wl.stream
    runs = {"group": lambda t: wl.run_group(t), "per_engine": lambda t: wl.run(t)}
    t_w = time.perf_counter()
    k = 0
    while time.perf_counter() - t_w < 0.3:  # clocks to steady state
        for name in runs:
            runs[name](3600 * k)
        k += 1
        torch.cuda.synchronize()
    res = {name: [] for name in runs}
    for r in range(a.rounds):
        order = list(runs) if r % 2 == 0 else list(runs)[::-1]
        for name in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(a.steps):
                runs[name](3600 * i)
            e1.record(s)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / a.steps)
    total = sum(wl.alg_bytes)
    out = {"cells": a.cells, "types": a.types, "precision": a.precision, "atmos_map": a.atmos_map,
           "alg_bytes_per_step": total, "rounds": a.rounds, "steps_per_block": a.steps}
    for name, v in res.items():
        ms = float(np.mean(v))
        out[name] = {"ms_per_step": round(ms, 4), "ms_blocks": [round(x, 4) for x in v],
                     "Mcells_per_s": round(a.cells * len(wl.engines) / (ms * 1e-3) / 1e6, 1),
                     "TBps": round(total / (ms * 1e-3) / 1e12, 3)}
    out["group_gain"] = round(out["per_engine"]["ms_per_step"] / out["group"]["ms_per_step"] - 1, 4)
    wl.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
