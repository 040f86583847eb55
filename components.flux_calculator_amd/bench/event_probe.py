#!/usr/bin/env python3
"""Does timing perturb the step?  The bench's coupling step (CCLM, MOM5, RCO fused kernels
back-to-back, 10M cells, fields in HBM) timed by wall clock over many steps, with and
without HIP events recorded between the kernels, and with the engines' own per-run events
on or off (FCX_OPT_TIMING).  Interleaved rounds, medians.

  python components.flux_calculator_amd/bench/event_probe.py [--cells N] [--steps K]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--order", default="CCLM,MOM5,RCO", help="engine creation order")
    ap.add_argument("--atmos", type=int, default=1)
    ap.add_argument("--spacer-mb", type=int, default=0, help="allocation between inputs and engines")
    ap.add_argument("--pool", action="store_true",
                    help="repack every case's device arrays into one allocation before the engines")
    ap.add_argument("--pool-reverse", action="store_true",
                    help="with --pool: pack the cases in reverse order (case 0's arrays last)")
    ap.add_argument("--engines-reversed", action="store_true",
                    help="allocate all cases first, then create the engines in reverse order")
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
    spacer = torch.empty(a.spacer_mb << 20, dtype=torch.uint8, device=dev) if a.spacer_mb else None  # noqa: F841
    cases = []
    for v in a.order.split(","):
        c = build_case(v, n=n, T=1, device=dev, data=data)
        outs = [torch.empty(la.n_atmos, dtype=torch.float64, device=dev) for _ in ATM]
        atmos = {"local": la, "fields": [(PHASE_NORMAL, 1, g, name, o) for (name, g), o in zip(ATM, outs)]}
        cases.append((c, outs, atmos if a.atmos else None))
    if a.pool:  # one allocation for all fields of all cases (aliases kept)
        uniq = {}
        for c, _, _ in (cases[::-1] if a.pool_reverse else cases):
            for t in c.lf.field.values():
                uniq.setdefault(t.data_ptr(), t)
        total = sum(t.numel() for t in uniq.values())
        pool = torch.empty(total + 32 * len(uniq), dtype=torch.float64, device=dev)
        view, off = {}, 0
        for ptr, t in uniq.items():
            v = pool[off: off + t.numel()]
            v.copy_(t)
            view[ptr] = v
            off += (t.numel() + 31) // 32 * 32  # 256-B aligned sub-buffers
        for c, _, _ in cases:
            for k, t in list(c.lf.field.items()):
                c.lf.field[k] = view[t.data_ptr()]
        del uniq
    made = {}
    order = range(len(cases) - 1, -1, -1) if a.engines_reversed else range(len(cases))
    for i in order:
        c, outs, atmos = cases[i]
        made[i] = (c, outs, Engine(c.lf, 1, c.methods, device=0, stream=stream.cuda_stream,
                                   atmos=atmos, options={"atmos_in_run": 0}))
        made[i][2].run(PHASE_ALL, 0)  # plan + Params allocated now, in creation order
    engines = [made[i] for i in range(len(cases))]

    def run(mode):
        torch_events = mode in ("torch_events", "both")
        fcx_timing = mode in ("fcx_timing", "both")
        for _, _, e in engines:
            e.set_option("timing", int(fcx_timing))
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in engines]
        for _, _, e in engines:
            e.run(PHASE_ALL, 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            for i, (_, _, e) in enumerate(engines):
                if torch_events:
                    evs[i][0].record(stream)
                e.run(PHASE_ALL, k * 3600)
                if torch_events:
                    evs[i][1].record(stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    # predecessor effect: kernel Y timed right after kernel X (one event pair around Y only)
    pairs = {}
    for _, _, e in engines:
        e.set_option("timing", 0)
    names = tuple(f"{v}#{i}" for i, v in enumerate(a.order.split(",")))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for x in range(len(engines)):
        for y in range(len(engines)):
            ts = []
            for r in range(15):
                engines[x][2].run(PHASE_ALL, 0)
                ev0.record(stream)
                engines[y][2].run(PHASE_ALL, 0)
                ev1.record(stream)
                ev1.synchronize()
                ts.append(ev0.elapsed_time(ev1))
            pairs[f"{names[y]} after {names[x]}"] = round(float(np.median(ts)), 4)

    # dirty-cache hypothesis: a 512 MB read (torch sum) between X and Y -- if X leaves dirty
    # Infinity-Cache lines, the flush absorbs the write-back and Y runs at its clean speed
    flush_buf = torch.ones(64 << 20, dtype=torch.float64, device=dev)  # 512 MB
    ev2 = torch.cuda.Event(enable_timing=True)
    flushed = {}
    # a 512 MB read (sum) or write (fill) between X and Y: a write has to evict dirty
    # memory-side cache lines X left behind, a read need not
    for kind, op in (("read", lambda: flush_buf.sum()), ("write", lambda: flush_buf.fill_(1.0))):
        for x in range(len(engines)):
            y = 0
            tf, ty = [], []
            for r in range(15):
                engines[x][2].run(PHASE_ALL, 0)
                ev0.record(stream)
                op()
                ev2.record(stream)
                engines[y][2].run(PHASE_ALL, 0)
                ev1.record(stream)
                ev1.synchronize()
                tf.append(ev0.elapsed_time(ev2))
                ty.append(ev2.elapsed_time(ev1))
            flushed[f"{names[y]} after {names[x]} + 512 MB {kind}"] = {
                "flush_ms": round(float(np.median(tf)), 4), "kernel_ms": round(float(np.median(ty)), 4)}
    del flush_buf

    modes = ["none", "torch_events", "fcx_timing", "both"]
    res = {m: [] for m in modes}
    for r in range(a.rounds):
        order = list(modes)
        np.random.default_rng(r).shuffle(order)
        for m in order:
            res[m].append(run(m))
    out = {m: round(float(np.median(v)), 4) for m, v in res.items() if v}
    print(json.dumps({"ms_per_step_median": out, "kernel_ms_after": pairs, "flushed": flushed, "cells": n,
                      "steps": a.steps, "rounds": a.rounds}))


if __name__ == "__main__":
    main()
