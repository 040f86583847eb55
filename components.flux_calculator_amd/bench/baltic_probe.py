#!/usr/bin/env python3
"""The Baltic-size drop-in (32,768 cells, caller heap arrays) under several transports, to
find the one closest to the host-link bound (link_probe.py): median wall time of fcx_step
of each variant alone, and of the three variants started with fcx_step_async from one host
thread then synchronised.

  python components.flux_calculator_amd/bench/baltic_probe.py [--cells 32768] [--steps 400]
    [--mode NAME:opt=val,opt=val ...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))

VARIANTS = ("CCLM", "MOM5", "RCO")
MODES = [
    "default:",
    "zc_chunks4:zero_copy=1,pipeline_min_chunk=8192,pipeline_chunks=4",
    "zc_chunks8:zero_copy=1,pipeline_min_chunk=4096,pipeline_chunks=8",
    "dma_chunks4:zero_copy=0,pipeline_min_chunk=8192,pipeline_chunks=4",
    "dma_seq:zero_copy=0",
]


def parse_mode(m):
    name, _, rest = m.partition(":")
    opts = {}
    for kv in filter(None, rest.split(",")):
        k, v = kv.split("=")
        opts[k] = int(v)
    return name, opts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=32_768)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--mode", action="append", default=[])
    ap.add_argument("--handover", type=int, default=1, help="0: skip the hand-over comparison")
    ap.add_argument("--host-malloc", action="store_true",
                    help="the fields in fcx_host_malloc memory (a Fortran host's c_f_pointer arrays, "
                         "INTEGRATION.md) instead of caller heap arrays")
    ap.add_argument("--no-torch", action="store_true",
                    help="a process without torch, as a Fortran host: libfcx binds the system HIP "
                         "runtime and every engine creates its own stream")
    a = ap.parse_args()
    if a.no_torch:
        os.environ["FCX_NO_TORCH"] = "1"
    else:
        import torch
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.host_alloc import Arena
    from fcx.synthetic import build_case, inputs_for_bench

    n = a.cells
    data = inputs_for_bench(n)
    out = {"cells": n, "steps": a.steps, "host_malloc": a.host_malloc, "modes": {}}
    for m in a.mode or MODES:
        name, opts = parse_mode(m)
        cases = [build_case(v, n=n, T=1, bias=True, data=data) for v in VARIANTS]
        arena = Arena() if a.host_malloc else None
        if arena:
            for c in cases:
                arena.adopt(c.lf)
        # own_stream=1: every engine creates its own non-blocking stream (as for a Fortran host)
        # instead of running on a torch stream
        own = bool(opts.pop("own_stream", 0)) or a.no_torch
        streams = [None if own else torch.cuda.Stream().cuda_stream for _ in cases]
        engines = [Engine(c.lf, 1, c.methods, corrections=c.corrections, stream=s, options=opts)
                   for c, s in zip(cases, streams)]
        if own:
            opts["own_stream"] = 1
        res = {"options": opts}
        for v, e in zip(VARIANTS, engines):
            for k in range(50):
                e.step(PHASE_ALL, k * 3600)
            ts = []
            for k in range(a.steps):
                t0 = time.perf_counter()
                e.step(PHASE_ALL, k * 3600)
                ts.append(time.perf_counter() - t0)
            res[v] = round(float(np.median(ts)) * 1e6, 1)
        res["sequential_sum_us"] = round(sum(res[v] for v in VARIANTS), 1)
        ts = []
        for k in range(50 + a.steps):
            t0 = time.perf_counter()
            for e in engines:
                e.step_async(PHASE_ALL, k * 3600)
            for e in engines:
                e.synchronize()
            if k >= 50:
                ts.append(time.perf_counter() - t0)
        res["async_three_us"] = round(float(np.median(ts)) * 1e6, 1)
        for e in engines:
            e.close()
        if arena:
            arena.close()
        out["modes"][name] = res
        print(name, json.dumps(res), flush=True)
    if a.handover:
        out["handover"] = handover(n, a.steps)
        print("handover", json.dumps(out["handover"]), flush=True)
    print(json.dumps(out), flush=True)


def handover(n, steps):
    """The coupled host's step with OASIS's receives in it: every input field arrives by an
    oasis_get, played here by a copy from a receive buffer into the field array (256 KB at
    32,768 cells).  'after' = all receives, then fcx_step; 'handed' = each receive followed
    by fcx_upload_field (the engine's thread stages the field while the next one arrives),
    then fcx_step.  Median wall time per step of the three variants one after the other."""
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.synthetic import build_case

    def wait_us(us):  # a receive's wait for the sender (MPI progress), no memory traffic
        t_end = time.perf_counter() + us * 1e-6
        while time.perf_counter() < t_end:
            pass

    res = {}
    cases = [build_case(v, n=n, T=1, bias=True) for v in VARIANTS]
    per = []
    for c in cases:
        outs = {id(c.lf.field[k]) for k in c.outputs}
        slots, seen = [], set()
        for key, arr in c.lf.field.items():
            if id(arr) not in outs and id(arr) not in seen:
                seen.add(id(arr))
                slots.append((key, arr, arr.copy()))  # (slot, field array, "received" data)
        per.append(slots)
    for recv_model in ("copy", "wait20"):
        for mode in ("after", "handed"):
            engines = [Engine(c.lf, 1, c.methods, corrections=c.corrections) for c in cases]
            ts = []
            for k in range(50 + steps):
                t0 = time.perf_counter()
                for e, slots in zip(engines, per):
                    for key, arr, recv in slots:
                        if recv_model == "copy":
                            np.copyto(arr, recv)  # oasis_get: the message copied into the field
                        else:
                            wait_us(20)  # oasis_get: waiting 20 us for the sender
                        if mode == "handed":
                            e.upload_field(*key)
                    e.step(PHASE_ALL, k * 3600)
                if k >= 50:
                    ts.append(time.perf_counter() - t0)
            for e in engines:
                e.close()
            res[f"{recv_model}_{mode}_us"] = round(float(np.median(ts)) * 1e6, 1)
    res["rule"] = ("three variants one after the other; each input field received (copy: a copy from a receive "
                   "buffer into the field array; wait20: 20 us of waiting for the sender), then fcx_step ('after') or "
                   "each receive followed by fcx_upload_field ('handed')")
    return res


if __name__ == "__main__":
    main()
