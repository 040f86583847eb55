#!/usr/bin/env python3
"""A/B of libfcx builds in ONE process over the SAME device arrays (measurement tool).

Physical placement of the field arrays moves the HBM rate of a many-stream kernel by up to
~10 % from one allocation to the next (profiles/r01/alloc_probe.txt), which swamps small
kernel differences between separate bench runs.  Here every build's engines are bound to
the same LocalFields (inputs, outputs, atmosphere map and outputs), and the builds take
turns, step by step, so they see the same placement and the same clock state.

  FCX_LIBRARY is the reference build (load()); the others come from --lib NAME=PATH.
  python inproc_ab.py --lib ho=ab/ho/libfcx.so --lib triv=ab/triv/libfcx.so [--types 1]

Output: one JSON object, per build the mean step time and per-variant kernel times and
GB/s (algorithmic bytes, bench.py's definition).
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
FIELDS = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", default=[],
                    help="NAME=PATH[:atmos0][@key=val,...] of another build (PATH 'ref': the main build; "
                         ":atmos0 = that build's engines without the accumulation; @: fcx_set_option values)")
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--types", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--steps", type=int, default=40, help="steps per build and round")
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--atmos", type=int, default=1, help="0: flux pass only (no accumulation)")
    ap.add_argument("--opts", action="append", default=[],
                    help="NAME:key=val[,key=val] -- another engine set of the main build with these "
                         "fcx_set_option values (e.g. split0:type_split=0)")
    ap.add_argument("--precision", choices=("f64", "f32"), default="f64")
    ap.add_argument("--streams", action="append", default=[],
                    help="NAME: another engine set of the main build with every variant's engine on its "
                         "own stream (forked from and joined back into the main stream every step)")
    ap.add_argument("--atmos-map", choices=("periodic", "random"), default="random",
                    help="exchange->atmosphere map (bench.py's default: random runs crossing the wave tiles)")
    ap.add_argument("--group", action="store_true",
                    help="every build's step is ONE fcx_run_group of its engines (the bench step), "
                         "timed with one event pair around it (reported as the first variant's kernel)")
    ap.add_argument("--host", action="store_true",
                    help="bind host arrays: every build's engines own their (tile-blocked) device "
                         "mirrors, uploaded once -- the bench's layout; builds then differ in placement")
    a = ap.parse_args()

    import torch
    from fcx import _lib
    from fcx.basic import PHASE_ALL, PHASE_NORMAL
    from fcx.engine import Engine
    from fcx.parallel import BlockedRandomAtmosMap, PeriodicAtmosMap
    from fcx.synthetic import as_dtype, build_case, inputs_for_bench

    libs, no_atmos, extra_opts = {"ref": None}, set(), {}
    for name in a.streams:
        libs[name] = None
    for spec in a.opts:
        name, kv = spec.split(":", 1)
        libs[name] = None
        extra_opts[name] = {k: int(v) for k, v in (x.split("=") for x in kv.split(","))}
    for spec in a.lib:
        name, path = spec.split("=", 1)
        if "@" in path:
            path, kv = path.split("@", 1)
            extra_opts[name] = {k: int(v) for k, v in (x.split("=") for x in kv.split(","))}
        if path.endswith(":atmos0"):
            path = path[: -len(":atmos0")]
            no_atmos.add(name)
        libs[name] = None if path == "ref" else _lib.load_path(path)
    variants = [v for v in a.variants.split(",") if v]
    n = a.cells
    dev = torch.device("cuda", 0)
    host = inputs_for_bench(n)
    if a.host:
        data, cdev = host, None
    else:
        data, cdev = {k: torch.as_tensor(v).to(dev) for k, v in host.items()}, dev
        del host
    stream = torch.cuda.current_stream(dev)
    la = (BlockedRandomAtmosMap() if a.atmos_map == "random" else PeriodicAtmosMap()).local(0, n, 0, 1, n)
    cases, outs = [], []
    f32 = a.precision == "f32"
    for v in variants:
        c = build_case(v, n=n, T=a.types, device=cdev, data=data if a.types == 1 else None)
        cases.append(as_dtype(c, "float32") if f32 else c)
        outs.append({name: (np.empty(max(la.n_atmos, 1), dtype=np.float32 if f32 else np.float64) if a.host else
                            torch.empty(max(la.n_atmos, 1), dtype=torch.float32 if f32 else torch.float64,
                                        device=dev))
                     for name, _ in FIELDS})
    s0 = 0 if a.types >= 2 else 1
    engines, estreams = {}, {}
    for lname, lib in libs.items():
        estreams[lname] = ([torch.cuda.Stream(dev) for _ in variants] if lname in a.streams else
                           [stream] * len(variants))
        engines[lname] = [
            Engine(c.lf, c.num_surface_types, c.methods, corrections=c.corrections, averages=c.averages,
                   device=0, stream=st.cuda_stream,
                   atmos=({"local": la, "fields": [(PHASE_NORMAL, s0, g, name, o[name]) for name, g in FIELDS]}
                          if a.atmos and lname not in no_atmos else None),
                   options={"atmos_in_run": 0, "timing": 0, "host_staging": 0, **extra_opts.get(lname, {})}, lib=lib)
            for c, o, st in zip(cases, outs, estreams[lname])]
        if a.host:
            for e in engines[lname]:
                e.upload(PHASE_ALL)
    alg = {k: [es[i].algorithmic_bytes(PHASE_ALL) for i in range(len(variants))] for k, es in engines.items()}

    from fcx.engine import run_group

    def step(es, t, ev=None, sts=None):
        if a.group:
            if ev is not None:
                ev[0][0].record(stream)
            run_group(es, PHASE_ALL, t)
            if ev is not None:
                ev[0][1].record(stream)
                for i in range(1, len(es)):  # (one launch: the other variants' pairs are empty)
                    ev[i][0].record(stream)
                    ev[i][1].record(stream)
            return
        fork = None
        if sts is not None and sts[0] is not stream:
            fork = torch.cuda.Event()
            fork.record(stream)
        for i, e in enumerate(es):
            st = stream if sts is None else sts[i]
            if fork is not None:
                st.wait_event(fork)
            if ev is not None:
                ev[i][0].record(st)
            e.run(PHASE_ALL, t)
            if ev is not None:
                ev[i][1].record(st)
        if fork is not None:
            for st in sts:
                stream.wait_stream(st)

    names = list(libs)
    for w in range(a.warmup):
        for lname in names:
            step(engines[lname], w * 3600, sts=estreams[lname])
    torch.cuda.synchronize()
    kern = {k: [] for k in names}
    wall = {k: [] for k in names}
    for r in range(a.rounds):
        order = names[r % len(names):] + names[: r % len(names)]  # rotate who goes first
        for lname in order:
            ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in variants] for _ in range(a.steps)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.steps):
                step(engines[lname], k * 3600, ev[k], sts=estreams[lname])
            torch.cuda.synchronize()
            wall[lname].append((time.perf_counter() - t0) / a.steps * 1e3)
            kern[lname].append([[x.elapsed_time(y) for x, y in row] for row in ev])
    out = {"cells": n, "types": a.types, "precision": a.precision, "atmos": a.atmos, "atmos_map": a.atmos_map, "rounds": a.rounds,
           "steps": a.steps, "builds": {}}
    for lname in names:
        km = np.array(kern[lname]).reshape(-1, len(variants)).mean(axis=0)
        if a.group:
            out["builds"].setdefault(lname, {})["group_ms"] = round(float(km[0]), 4)
            out["builds"][lname]["group_GBps"] = round(sum(alg[lname]) / (km[0] * 1e-3) / 1e9, 1)
        out["builds"].setdefault(lname, {}).update({
            "ms_per_step": round(float(np.mean(wall[lname])), 4),
            "ms_per_step_rounds": [round(x, 4) for x in wall[lname]],
            "kernels": {v: {"ms": round(float(km[i]), 4), "GBps": round(alg[lname][i] / (km[i] * 1e-3) / 1e9, 1)}
                        for i, v in enumerate(variants)},
        })
    for es in engines.values():
        for e in es:
            e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
