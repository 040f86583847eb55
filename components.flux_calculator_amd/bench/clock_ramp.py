#!/usr/bin/env python3
"""How long does the GPU take to reach its steady kernel rate after a pause?

The bench's coupling step (CCLM, MOM5, RCO fused kernels back-to-back, 10M cells, fields in
HBM) is run continuously for --ms milliseconds after (a) an idle pause of --idle-s seconds
and (b) a 2 GB allocation + first touch, with an event pair around every kernel.  Prints
each kernel's median duration per window of elapsed time, so a clock / power ramp shows
up as slow early windows.

  python components.flux_calculator_amd/bench/clock_ramp.py [--cells N] [--ms 600]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))
ATM = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))
WINDOWS_MS = (0, 5, 10, 20, 40, 80, 160, 320, 640, 1280)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--ms", type=float, default=600.0)
    ap.add_argument("--idle-s", type=float, default=1.0)
    a = ap.parse_args()
    import torch

    from fcx.basic import PHASE_ALL, PHASE_NORMAL
    from fcx.engine import Engine
    from fcx.parallel import PeriodicAtmosMap
    from fcx.synthetic import build_case, inputs_for_bench

    n = a.cells
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    data = {k: torch.as_tensor(v).to(dev) for k, v in inputs_for_bench(n).items()}
    la = PeriodicAtmosMap().local(0, n, 0, 1, n)
    engines = []
    for v in ("CCLM", "MOM5", "RCO", "CCLM"):  # the 4th: a duplicate CCLM engine, own outputs
        c = build_case(v, n=n, T=1, device=dev, data=data)
        outs = [torch.empty(la.n_atmos, dtype=torch.float64, device=dev) for _ in ATM]
        atmos = {"local": la, "fields": [(PHASE_NORMAL, 1, g, name, o) for (name, g), o in zip(ATM, outs)]}
        e = Engine(c.lf, 1, c.methods, device=0, stream=stream.cuda_stream, atmos=atmos,
                   options={"atmos_in_run": 1, "timing": 0})
        engines.append((v if len(engines) < 3 else v + "'", c, outs, e))
    step_engines = engines[:3]
    for _, _, _, e in engines:
        e.run(PHASE_ALL, 0)
    torch.cuda.synchronize()

    def burst():
        """Steps until --ms of GPU time has elapsed; (start_ms, kernel, duration_ms) rows."""
        evs = []
        t_end = time.perf_counter() + a.ms / 1e3 * 1.5
        k = 0
        while True:
            for i, (_, _, _, e) in enumerate(step_engines):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                e.run(PHASE_ALL, 0)
                e1.record(stream)
                evs.append((i, e0, e1))
            k += 1
            if k % 50 == 0:
                evs[-1][2].synchronize()
                if evs[0][1].elapsed_time(evs[-1][2]) >= a.ms or time.perf_counter() > t_end:
                    break
        torch.cuda.synchronize()
        t0 = evs[0][1]
        return [(t0.elapsed_time(e0), i, e0.elapsed_time(e1)) for i, e0, e1 in evs]

    def summarize(rows):
        out = {}
        for lo, hi in zip(WINDOWS_MS[:-1], WINDOWS_MS[1:]):
            sel = [(i, d) for t, i, d in rows if lo <= t < hi]
            if not sel:
                continue
            out[f"{lo}-{hi} ms"] = {engines[i][0]: round(float(np.median([d for j, d in sel if j == i])), 4)
                                    for i in range(len(step_engines)) if any(j == i for j, _ in sel)}
        return out

    res = {}
    time.sleep(a.idle_s)
    res[f"after {a.idle_s:g} s idle"] = summarize(burst())
    res["back-to-back (no pause)"] = summarize(burst())
    big = torch.empty(256 << 20, dtype=torch.float64, device=dev)  # 2 GB
    big.fill_(0.0)
    torch.cuda.synchronize()
    res["after a 2 GB allocation + fill"] = summarize(burst())
    del big

    # steady state (after >= 300 ms of load): event cost vs interleaving
    def warm(ms=300.0):
        t = time.perf_counter() + ms / 1e3
        while time.perf_counter() < t:
            for _, _, _, e in step_engines:
                e.run(PHASE_ALL, 0)
            torch.cuda.synchronize()

    def loop(seq, reps, bracket):
        """seq: engine indices per step; bracket: indices timed with an event pair.
        Returns (ms per step from one outer event pair, {index: median kernel ms})."""
        o0, o1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        evs = []
        o0.record(stream)
        for _ in range(reps):
            for i in seq:
                if i in bracket:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    engines[i][3].run(PHASE_ALL, 0)
                    e1.record(stream)
                    evs.append((i, e0, e1))
                else:
                    engines[i][3].run(PHASE_ALL, 0)
        o1.record(stream)
        torch.cuda.synchronize()
        per = {}
        for i in bracket:
            per[engines[i][0]] = round(float(np.median([e0.elapsed_time(e1) for j, e0, e1 in evs if j == i])), 4)
        return round(o0.elapsed_time(o1) / reps, 4), per

    steady = {}
    for label, seq, bracket in (("step, no events", (0, 1, 2), ()),
                                ("step, events on every kernel", (0, 1, 2), (0, 1, 2)),
                                ("step, events on MOM5 only", (0, 1, 2), (1,)),
                                ("MOM5 repeated, no events", (1,), ()),
                                ("MOM5 repeated, events on every kernel", (1,), (1,)),
                                ("CCLM repeated, events", (0,), (0,)),
                                ("RCO repeated, events", (2,), (2,))):
        warm()
        ms, per = loop(seq, 200, bracket)
        steady[label] = {"ms_per_iteration": ms, "kernel_ms": per}
    # Y after X at steady state: same code + own outputs (CCLM after CCLM') vs same engine
    pairs = {}
    for x, y in ((0, 0), (3, 0), (0, 3), (1, 0), (2, 0), (1, 1), (0, 1), (3, 1), (2, 2), (1, 2)):
        warm()
        _, per = loop((x, y) if x != y else (y,), 200, (y,))
        pairs[f"{engines[y][0]} after {engines[x][0]}"] = per[engines[y][0]]
    steady["pairs (events on Y only)"] = pairs

    # what persists: translation caches or the memory-side cache?  CCLM after CCLM with an
    # operation in between: a TLB sweep (one element per 2 MB page of 8 GB: 4096 pages,
    # ~0.5 MB of data), or 200 MB written / read contiguously (few pages, much cache)
    sweep = torch.empty(8 << 30, dtype=torch.uint8, device=dev)
    pages = sweep.view(-1, 2 << 20)[:, 0]
    w200 = torch.empty(25 << 20, dtype=torch.float64, device=dev)
    w200.fill_(1.0)
    ops = {"nothing": None, "TLB sweep 8 GB": lambda: pages.fill_(1),
           "200 MB write": lambda: w200.fill_(2.0), "200 MB read": lambda: w200.sum()}
    between = {}
    for label, op in ops.items():
        warm()
        ts = []
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(100):
            engines[0][3].run(PHASE_ALL, 0)
            if op is not None:
                op()
            e0.record(stream)
            engines[0][3].run(PHASE_ALL, 0)
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        between[f"CCLM after CCLM + {label}"] = round(float(np.median(ts)), 4)
    steady["same engine with an operation in between"] = between
    del sweep, w200
    print(json.dumps({"cells": n, "burst_ms": a.ms, "kernel_ms_by_window": res, "steady": steady}))


if __name__ == "__main__":
    main()
