#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) rate of the drop-in path: the fields live in host arrays, as
the Fortran host owns them, and every coupling step is fcx_step = H2D of the inputs, the
fused kernels, D2H of the outputs ("kernel-only and end-to-end with H2D/D2H,
reported separately"; 8f rank 1).  bench.py's `value` is the HBM-resident rate; this is the
rate a host that hands over host buffers sees.

Sweeps: caller heap arrays through the engine's staging arena (FCX_OPT_HOST_STAGING, the
default) or one runtime copy per array, library arrays (fcx_host_malloc: direct DMA or
zero-copy), and sequential vs pipelined steps (FCX_OPT_PIPELINE_CHUNKS).  The ceiling is the host link: the same bytes as
one pinned hipMemcpy per direction, measured here with torch, H2D and D2H concurrently.

  python components.flux_calculator_amd/bench/e2e_host.py [--cells N] [--steps K]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))


def link_ceiling(h2d_bytes, d2h_bytes, reps=5):
    """Pinned copies of the step's byte counts: H2D alone, D2H alone, both concurrently."""
    import torch

    hi = torch.empty(h2d_bytes, dtype=torch.uint8, pin_memory=True)
    ho = torch.empty(d2h_bytes, dtype=torch.uint8, pin_memory=True)
    di = torch.empty(h2d_bytes, dtype=torch.uint8, device="cuda")
    do = torch.empty(d2h_bytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        return float(np.median(t))

    def both():
        with torch.cuda.stream(s1):
            di.copy_(hi, non_blocking=True)
        with torch.cuda.stream(s2):
            ho.copy_(do, non_blocking=True)

    t_in = timed(lambda: di.copy_(hi, non_blocking=True))
    t_out = timed(lambda: ho.copy_(do, non_blocking=True))
    t_both = timed(both)
    return {"h2d_GBps": h2d_bytes / t_in / 1e9, "d2h_GBps": d2h_bytes / t_out / 1e9,
            "concurrent_s": t_both, "concurrent_GBps": (h2d_bytes + d2h_bytes) / t_both / 1e9}


SWEEP = [("heap, runtime copies, sequential", {"host_staging": 0, "pipeline_chunks": 1}),
         ("heap, runtime copies, 8 chunks", {"host_staging": 0, "pipeline_chunks": 8}),
         ("heap, staged, sequential", {"pipeline_chunks": 1}),
         ("heap, staged, 4 chunks", {"pipeline_chunks": 4}),
         ("heap, staged, 8 chunks", {"pipeline_chunks": 8}),   # the default transport
         ("heap, staged, 16 chunks", {"pipeline_chunks": 16}),
         ("heap, staged, 32 chunks", {"pipeline_chunks": 32}),
         ("heap, arena in place, 8 chunks", {"zero_copy": 1, "pipeline_chunks": 8}),
         ("heap, arena in place, 16 chunks", {"zero_copy": 1, "pipeline_chunks": 16}),
         ("zero-copy", {"zero_copy": 1}),                       # arrays from fcx_host_malloc
         ("library arrays, 8 chunks", {"zero_copy": 0, "pipeline_chunks": 8})]
LIBRARY_ARRAYS = ("zero-copy", "library arrays, 8 chunks")
N_IN = {"CCLM": 10, "MOM5": 11, "RCO": 5}
N_OUT = {"CCLM": 7, "MOM5": 7, "RCO": 6}


def child(a):
    """One (variant, sweep entry) in this process: an engine created once, as a host would."""
    import torch  # noqa: F401  (one HIP runtime per process: torch first, fcx/_lib.py)
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.synthetic import build_case, inputs_for_bench

    n = a.cells
    if a.only == "link":
        print(json.dumps(link_ceiling(N_IN[a.variants] * 8 * n, N_OUT[a.variants] * 8 * n)))
        return
    case = build_case(a.variants, n=n, T=1, data=inputs_for_bench(n))
    if a.only in LIBRARY_ARRAYS:  # the host allocated its arrays with fcx_host_malloc
        from fcx.host_alloc import Arena

        arena = Arena()
        arena.adopt(case.lf)
    opts = {**dict(SWEEP)[a.only], "timing": 1}  # device_timeline_ms / kernel_ms below
    eng = Engine(case.lf, 1, case.methods, options=opts)
    staging = eng.staging_bytes()
    eng.step(PHASE_ALL, 0)  # warm-up (first touch, plan, code objects)
    t = []
    for k in range(a.steps):
        t0 = time.perf_counter()
        eng.step(PHASE_ALL, k * 3600)
        t.append(time.perf_counter() - t0)
    ms = float(np.median(t)) * 1e3
    dev_ms = eng.last_kernel_ms()  # s_in start -> s_out end of the last step
    eng.run(PHASE_ALL, 0)  # kernel alone, fields already resident
    eng.synchronize()
    kern_ms = eng.last_kernel_ms()
    eng.close()
    print(json.dumps({"ms_per_step": round(ms, 3), "Mcells_per_s": round(n / ms / 1e3, 1),
                      "device_timeline_ms": round(dev_ms, 3), "kernel_ms": round(kern_ms, 4),
                      "staging_MB": round(staging / 1e6, 1)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--variants", default="CCLM,MOM5,RCO")
    ap.add_argument("--only", default=None, help="child: one sweep entry label, or 'link'")
    a = ap.parse_args()
    if a.only:
        child(a)
        return
    import subprocess

    def run(v, label):
        cmd = [sys.executable, os.path.abspath(__file__), "--cells", str(a.cells), "--steps", str(a.steps),
               "--variants", v, "--only", label]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f"{v} / {label}: exit {r.returncode}\n{r.stderr[-2000:]}")
        return json.loads(r.stdout.strip().splitlines()[-1])

    out = {"cells": a.cells, "steps": a.steps, "process_per_entry": True, "variants": {}}
    for v in a.variants.split(","):
        rows = {label: run(v, label) for label, _ in SWEEP}
        ceil = run(v, "link")
        best = min(r["ms_per_step"] for r in rows.values())
        out["variants"][v] = {"steps": rows, "h2d_bytes": N_IN[v] * 8 * a.cells,
                              "d2h_bytes": N_OUT[v] * 8 * a.cells, "link": ceil,
                              "best_vs_link_concurrent": round(ceil["concurrent_s"] * 1e3 / best, 3)}
        print(v, json.dumps(out["variants"][v]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
