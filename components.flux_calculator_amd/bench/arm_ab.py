#!/usr/bin/env python3
"""Several workload arms (atmosphere map + engine options) in ONE process, their grouped
steps (fcx_run_group) timed in alternating blocks with a HIP event pair per block on the
engines' stream (measurement tool).  Every arm keeps its own engines and arrays, all
resident together, so the arms see the same clocks and the same allocator state.

  python arm_ab.py --arms "halo:random;nohalo:random:atmos_halo=0;periodic:periodic" \
      [--cells 10000000] [--types 1] [--precision f64] [--rounds 8] [--steps 20]

The output JSON holds each arm's mean step time and the launch schedule (arm, group calls
per block, in issue order), so a rocprofv3 kernel trace of the same run can be split by arm
(bench/split_trace.py) into per-kernel times that exclude an arm's other launches.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))


def parse_arms(text):
    arms = []
    for spec in text.split(";"):
        parts = spec.split(":")
        name, amap = parts[0], parts[1]
        opts = {}
        for kv in (parts[2].split(",") if len(parts) > 2 and parts[2] else []):
            k, v = kv.split("=")
            opts[int(k) if k.isdigit() else k] = int(v)  # a raw option id: an A/B build's knob
        arms.append((name, amap, opts))
    return arms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", required=True)
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--types", type=int, default=1)
    ap.add_argument("--precision", choices=("f64", "f32"), default="f64")
    ap.add_argument("--variants", default="CCLM,MOM5,RCO")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20, help="grouped steps per block")
    a = ap.parse_args()
    import torch
    from fcx.workload import Workload

    arms = parse_arms(a.arms)
    wls = {}
    for name, amap, opts in arms:
        wls[name] = Workload(a.cells, 0, 1, variants=tuple(a.variants.split(",")), types=a.types,
                             precision=a.precision, atmos=True, atmos_map=amap, engine_options=opts)
    s = wls[arms[0][0]].stream
    schedule = []
    t_w = time.perf_counter()
    k = 0
    while time.perf_counter() - t_w < 0.3:  # clocks to steady state
        for name, _, _ in arms:
            wls[name].run_group(3600 * k)
            schedule.append([name, 1])
        k += 1
        torch.cuda.synchronize()
    res = {name: [] for name, _, _ in arms}
    for r in range(a.rounds):
        order = [x[0] for x in arms]
        order = order if r % 2 == 0 else order[::-1]
        for name in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(a.steps):
                wls[name].run_group(3600 * i)
            e1.record(s)
            torch.cuda.synchronize()
            schedule.append([name, a.steps])
            res[name].append(e0.elapsed_time(e1) / a.steps)
    out = {"cells": a.cells, "types": a.types, "precision": a.precision, "rounds": a.rounds,
           "steps_per_block": a.steps, "arms": {}}
    for name, amap, opts in arms:
        v = res[name]
        ms = float(np.mean(v))
        total = sum(wls[name].alg_bytes)
        out["arms"][name] = {"atmos_map": amap, "options": opts, "ms_per_step": round(ms, 4),
                             "ms_blocks": [round(x, 4) for x in v],
                             "alg_bytes_per_step": total,
                             "TBps_alg": round(total / (ms * 1e-3) / 1e12, 3)}
    base = arms[0][0]
    for name in out["arms"]:
        out["arms"][name]["vs_first"] = round(out["arms"][name]["ms_per_step"] / out["arms"][base]["ms_per_step"] - 1, 4)
    out["schedule"] = schedule
    for w in wls.values():
        w.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
