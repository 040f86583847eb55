#!/usr/bin/env python3
"""Config 2 of SURVEY.md 8d: the Baltic-size exchange grid (N = 32,768 cells, T = 1, all
fluxes fused) on one MI355X.  The working set (~4.5 MB per variant) is LLC-resident, so the
step is latency-bound: report microseconds per step, not an HBM fraction.

  device   fields HBM-resident (torch tensors): fcx_run of CCLM, MOM5 and RCO back-to-back,
           wall time per step over many steps (host launch cost included) and the kernels'
           HIP-event time
  host     fields in host arrays (the Fortran host's view): fcx_step per variant, through
           device mirrors (H2D, kernel, D2H, synchronise) and zero-copy (the kernel reads and
           writes the page-locked host arrays in place; the default at this size)
  cpu      the reference flux_lib (oracle/_ref, else the C port) on one core, same cells

  python components.flux_calculator_amd/bench/latency.py [--cells 32768] [--steps 2000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

VARIANTS = ("CCLM", "MOM5", "RCO")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=32_768)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--bias", type=int, default=1)
    ap.add_argument("--mode", action="append", default=[],
                    help="NAME:key=val[,key=val] -- another host-heap mode with these fcx_set_option values (A/B)")
    a = ap.parse_args()

    import torch
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.synthetic import build_case, inputs_for_bench

    n = a.cells
    host = inputs_for_bench(n)
    out = {"cells": n, "steps": a.steps, "bias": bool(a.bias)}

    # ---- device-resident: the three variants back-to-back per step
    data = {k: torch.as_tensor(v).to("cuda:0") for k, v in host.items()}
    stream = torch.cuda.current_stream()
    engines = []
    for v in VARIANTS:
        c = build_case(v, n=n, T=1, bias=bool(a.bias), device="cuda:0", data=data)
        engines.append(Engine(c.lf, 1, c.methods, corrections=c.corrections, stream=stream.cuda_stream,
                              options={"timing": 1}))
    for k in range(50):
        for e in engines:
            e.run(PHASE_ALL, k * 3600)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        for e in engines:
            e.run(PHASE_ALL, k * 3600)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e6
    kern = {}
    for v, e in zip(VARIANTS, engines):
        ts = []
        for k in range(200):
            e.run(PHASE_ALL, k * 3600)
            ts.append(e.last_kernel_ms() * 1e3)
        kern[v] = round(float(np.median(ts)), 2)
    out["device"] = {"us_per_step_3_variants": round(wall, 2), "kernel_us_median": kern,
                     "Mcells_per_s": round(3 * n / wall, 1)}

    # ---- same step without the engines' timing events, and captured into one HIP graph
    # (the engines launch on the capture stream; the replay reuses the captured month's
    # bias slice, fine for timing)
    for e in engines:
        e.set_option("timing", 0)

    def timed(fn, steps):
        for k in range(50):
            fn(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            fn(k)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e6

    def plain(k):
        for e in engines:
            e.run(PHASE_ALL, 0)
    wall_ne = timed(plain, a.steps)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream().cuda_stream
        for e in engines:
            e.set_stream(cap)
        for e in engines:
            e.run(PHASE_ALL, 0)
    for e in engines:
        e.set_stream(stream.cuda_stream)
    wall_g = timed(lambda k: g.replay(), a.steps)
    out["device"]["us_per_step_no_events"] = round(wall_ne, 2)
    out["device"]["us_per_step_one_graph"] = round(wall_g, 2)
    for e in engines:
        e.close()

    # ---- device-resident with the fused exchange -> atmosphere accumulation (6 fluxes), on
    # the periodic map (no segment crosses a wave tile) and the random-run map (carries
    # completed by the fix-up launch)
    from fcx.parallel import BlockedRandomAtmosMap, PeriodicAtmosMap
    atm_fields = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))
    acc = {}
    for mname, mk in (("periodic", PeriodicAtmosMap()), ("random", BlockedRandomAtmosMap())):
        la = mk.local(0, n, 0, 1, n)
        engs = []
        for v in VARIANTS:
            c = build_case(v, n=n, T=1, bias=bool(a.bias), device="cuda:0", data=data)
            outs = {k: torch.empty(la.n_atmos, dtype=torch.float64, device="cuda:0") for k, _ in atm_fields}
            engs.append(Engine(c.lf, 1, c.methods, corrections=c.corrections, stream=stream.cuda_stream,
                               atmos={"local": la, "fields": [(2, 1, g, k, outs[k]) for k, g in atm_fields]},
                               options={"timing": 0}))

        def step_atm(k, engs=engs):
            for e in engs:
                e.run(PHASE_ALL, 0)
        acc[mname] = round(timed(step_atm, a.steps), 2)
        for e in engs:
            e.close()
    out["device"]["us_per_step_with_atmos_accumulation"] = acc

    # ---- host-bound: fcx_step per variant (upload, run, download, synchronise)
    # host_heap_staged: caller heap arrays (a Fortran host's ALLOCATEd fields) through the
    # engine's staging arena, which the kernels use in place at this size (the default);
    # host_heap_staged_dma: the arena moved by one DMA per pool and direction
    # (FCX_OPT_ZERO_COPY=0); host_heap_runtime_copies: one runtime copy per array
    # (FCX_OPT_HOST_STAGING=0, round 2's default);
    # host_library_arrays: arrays from fcx_host_malloc, used in place by default (auto
    # zero-copy); host_library_mirrors: the same arrays through mirrors (FCX_OPT_ZERO_COPY=0)
    from fcx.host_alloc import Arena

    for mode, opts, lib_arrays in (("host_heap_staged", {}, False),
                                   ("host_heap_staged_dma", {"zero_copy": 0}, False),
                                   ("host_heap_runtime_copies", {"host_staging": 0}, False),
                                   ("host_library_arrays", {}, True),
                                   ("host_library_mirrors", {"zero_copy": 0}, True),
                                   *[(m.split(":", 1)[0], {k: int(v) for k, v in (x.split("=") for x in m.split(":", 1)[1].split(","))},
                                      False) for m in a.mode]):
        hb = {}
        for v in VARIANTS:
            c = build_case(v, n=n, T=1, bias=bool(a.bias), data=host)
            arena = Arena()
            if lib_arrays:
                arena.adopt(c.lf)
            e = Engine(c.lf, 1, c.methods, corrections=c.corrections, options=opts)
            e.set_option("timing", 0)
            for k in range(50):
                e.step(PHASE_ALL, k * 3600)
            ts = []
            for k in range(min(a.steps, 1000)):
                t0 = time.perf_counter()
                e.step(PHASE_ALL, k * 3600)
                ts.append(time.perf_counter() - t0)
            e.set_option("timing", 1)
            e.run(PHASE_ALL, 0)
            e.synchronize()
            kms = e.last_kernel_ms()
            zc = e.zero_copy_bytes()
            e.close()
            arena.close()
            hb[v] = {"zero_copy_bytes": zc,"us_per_step_median": round(float(np.median(ts)) * 1e6, 1),
                     "us_per_step_p90": round(float(np.percentile(ts, 90)) * 1e6, 1),
                     "kernel_us": round(kms * 1e3, 1)}
        out[mode] = hb

    # ---- the reference on one core, same cells
    import oracle_lib

    kind = "ref" if oracle_lib.load("ref") is not None else "c"
    cpu = {}
    for v in VARIANTS:
        c = build_case(v, n=n, T=1, bias=bool(a.bias), data=host)
        st = oracle_lib.OracleState(c, 0)
        oracle_lib.run_state(st, kind)
        ts = []
        for _ in range(20):
            t0 = time.perf_counter()
            oracle_lib.run_state(st, kind)
            ts.append(time.perf_counter() - t0)
        cpu[v] = round(float(np.median(ts)) * 1e6, 1)
    out["cpu_1core_us_per_step"] = cpu
    out["cpu_kind"] = "reference" if kind == "ref" else "port"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
