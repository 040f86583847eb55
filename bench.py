#!/usr/bin/env python3
"""Benchmark of the exchange-grid flux path on MI355X (BASELINE.json configs[2]).

Workload (per GPU): the synthetic 10M-cell exchange grid of SURVEY.md 8d, one coupling
step = the fused flux kernel of each of the CCLM, MOM5 and RCO variants back-to-back (T=1,
u/v grids = t grid, outputs QSUR MEVA HLAT HSEN RBBR UMOM VMOM; RCO has no QSUR).  Inputs
are resident in HBM before the timed region.  value = exchange-grid cells processed per
second over the whole job, one variant over N cells counting N cells.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one rank
per GPU, each owns a contiguous APPLE cell range of its own 10M cells (decomp_def.F90:23-31,
weak scaling); the one cross-rank exchange is the all-reduce of the atmosphere cells shared
by neighbouring ranks (libfcx's RCCL communicator), once per step.

Also reported:
  roofline      algorithmic bytes of the step's one launch (fcx_run_group) / its mean device
                time per timed step (one HIP event pair around the timed steps; --group 0: an
                event pair per step around the dominant engine's launch)
  cpu_baseline  the reference path on this box's host cores (rank 0, N=1 only; cpu_legs.py):
                the reference flux_lib compiled from source (oracle/_ref, kind "reference";
                the C restatement oracle/fco.c, kind "port", where it was not built) on one
                core and on the box's CPU share as APPLE-range ranks, at 32,768 cells
                (configs 1/2) and at this workload's size, on the same inputs
  baltic_size   the drop-in from host arrays (e2e) against those host cores at 32,768 cells,
                from caller heap arrays and from fcx_host_malloc arrays
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "exchange-grid Mcells/s per coupling step; achieved HBM GB/s vs MI355X peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip-level parameters)
VARIANTS = ("CCLM", "MOM5", "RCO")
MIN_WARMUP_S = 0.15  # back-to-back device work before the timed steps, whatever --warmup says
WARMUP_BLOCK = 10    # warm-up steps between two synchronisations
COLD_IDLE_S = 0.5    # idle gap before the cold step


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks (one per GPU); without a launcher bench.py starts torch.distributed.run itself")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--cells", type=int, default=10_000_000, help="exchange-grid cells per GPU (weak scaling)")
    p.add_argument("--global-cells", type=int, default=0,
                   help="fixed global grid sharded over the ranks by APPLE ranges (strong scaling, "
                        "config 4: 40000000); overrides --cells")
    p.add_argument("--variants", default=",".join(VARIANTS))
    p.add_argument("--types", type=int, default=1, help="surface types")
    p.add_argument("--bias", action="store_true", help="monthly evaporation bias corrections")
    p.add_argument("--cpu-seconds", type=float, default=3.0,
                   help="CPU baselines: seconds per leg (1 core and all cores, at 32,768 cells and --cells)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--e2e", type=int, default=1,
                   help="N=1: also time the end-to-end host-array step at 10M and 32,768 cells (an 'e2e' "
                        "sub-object; never the `value`)")
    p.add_argument("--atmos", type=int, default=1,
                   help="exchange->atmosphere accumulation (+ one RCCL all-reduce when N>1)")
    p.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    p.add_argument("--collective", choices=("rccl", "torch"), default="rccl",
                   help="N > 1: the boundary all-reduce through libfcx's RCCL communicator (default) or "
                        "torch.distributed (rehearsals)")
    p.add_argument("--config5", type=int, default=1,
                   help="N = 1, fp64 line: also time the fp32 variant of the same workload (BASELINE config 5's "
                        "fp32 kernels, a 'config5_fp32' sub-object; never the `value`)")
    p.add_argument("--config4", type=int, default=40_000_000,
                   help="also time config 4's fixed grid of this many cells sharded over the ranks "
                        "(strong scaling, a 'config4' sub-object); 0 = off")
    p.add_argument("--same-device", action="store_true",
                   help="rehearsal only: every rank on GPU 0 (with --backend gloo on a 1-GPU box)")
    p.add_argument("--max-blocks", type=int, default=None,
                   help="A/B only: FCX_OPT_MAX_BLOCKS of every engine (default: the engine's)")
    p.add_argument("--atmos-map", choices=("periodic", "random"), default="random",
                   help="exchange->atmosphere map: runs of 3..5 cells at random (default: segments cross "
                        "the kernel's 128-cell wave tiles, as on a real intersection grid), or periodic runs "
                        "of 3,4,5,4 cells (no segment crosses a tile; the round-1 bench map)")
    p.add_argument("--other-map", type=int, default=1,
                   help="also time the same workload on the other atmosphere map (an 'other_map' sub-object)")
    p.add_argument("--caller-device", action="store_true",
                   help="bind the caller's device arrays (contiguous torch tensors, the inputs shared "
                        "by the variants) instead of host arrays whose engine-owned device mirrors "
                        "(tile-blocked, FCX_OPT_TILED_LAYOUT) are uploaded once before the timed region")
    p.add_argument("--tiled", type=int, default=1, help="FCX_OPT_TILED_LAYOUT of the engines (A/B)")
    p.add_argument("--nontemporal", type=int, default=1, help="FCX_OPT_NONTEMPORAL of the engines (A/B)")
    p.add_argument("--precision", choices=("f64", "f32"), default="f64",
                   help="f32: the fp32 variant (config 5): fp32 cell pass with the accumulation fused in "
                        "(fp32 fluxes, fp64 weights, products and sums, fp32 outputs)")
    p.add_argument("--group", type=int, default=1,
                   help="1: every step runs the variants' engines through fcx_run_group, their fused flux "
                        "passes as ONE launch (one event pair around the timed steps); 0: one launch "
                        "per engine")
    p.add_argument("--kernel-events", choices=("dominant", "all"), default="dominant",
                   help="HIP event pairs inside the timed steps: around the dominant engine's launch only "
                        "(picked in an event-timed warm-up block), or around every engine's")
    return p.parse_args()


def host_cpu():
    """lscpu-style model name and the CPUs this process may use (SURVEY.md 8d CPU timing)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"model": model, "nproc": len(os.sched_getaffinity(0)), "machine_cpus": os.cpu_count()}


def multi_gpu_check(wl, world, rank, dist, samples=2000):
    """After the timed steps (outside the timed region): the atmosphere cells of the last step
    checked against the sequential SCRIP sum (fcx.parallel maps, oracle/fco.c order).

    * shared cells (a rank's first / last atmosphere cell, completed by the one all-reduce):
      every rank sends its partial cells (weights, fluxes) and its finished values to rank 0,
      which sums each boundary's cells in global exchange order from 0.0 and compares both
      neighbours' finished values (mixed error; association differs from the sequential sum
      only by the split into two partial sums);
    * a sample of interior cells of every rank: bit-identical to the sequential sum of the
      rank's own fluxes.
    The sequential sum is restated here (the oracle serves only the CPU baseline leg of this
    file): acc = acc + w * x from 0.0 in link order, in IEEE double without contraction.
    Returns the JSON sub-object on rank 0 (None elsewhere)."""
    from fcx.workload import ATM_FIELDS

    def seq_sum(w, x):
        acc = 0.0
        for wk, xk in zip(w, x):
            acc = acc + float(wk) * float(xk)
        return acc

    wl.download()
    la = wl.la
    rng = np.random.default_rng(7 + rank)
    idx = la.atmos_index
    starts = np.searchsorted(idx, np.arange(la.n_atmos + 1))  # CSR of the local map
    lo = 1 if la.left >= 0 else 0
    hi = la.n_atmos - (1 if la.right >= 0 else 0)
    pick = np.unique(rng.integers(lo, max(hi, lo + 1), min(samples, max(hi - lo, 0)))) if hi > lo else np.zeros(0, int)
    interior_bad, edge = 0, []
    for i, (case, outs) in enumerate(zip(wl.cases, wl.atm_outs)):
        for name, g in ATM_FIELDS:
            flux = np.asarray(case.lf.field[(1 if wl.types == 1 else 0, g, name)])
            got = np.asarray(outs[name])
            for a in pick:
                x0, x1 = starts[a], starts[a + 1]
                interior_bad += int(got[a] != seq_sum(la.weight[x0:x1], flux[x0:x1]))
            for side, a, slot in (("left", 0, la.left), ("right", la.n_atmos - 1, la.right)):
                if side == "right" and la.n_atmos == 1 and la.right == la.left:
                    continue  # one cell shared on both sides: one slot, its part sent once
                if slot >= 0:
                    x0, x1 = starts[a], starts[a + 1]
                    edge.append({"variant": i, "field": name, "slot": int(slot), "side": side, "rank": rank,
                                 "x0": int(wl.offset + x0), "w": la.weight[x0:x1].tolist(),
                                 "x": flux[x0:x1].tolist(), "got": float(got[a])})
    mine = {"rank": rank, "interior": int(pick.size) * len(wl.cases) * len(ATM_FIELDS),
            "interior_bad": interior_bad, "edge": edge}
    if world > 1:
        allv = [None] * world
        dist.all_gather_object(allv, mine)
    else:
        allv = [mine]
    if rank != 0:
        return None
    by = {}
    for r in allv:
        for e in r["edge"]:
            by.setdefault((e["variant"], e["field"], e["slot"]), []).append(e)
    worst, cells = 0.0, 0
    for key, parts in by.items():
        parts.sort(key=lambda e: e["x0"])  # the boundary's exchange cells in global order
        w = np.concatenate([np.asarray(e["w"]) for e in parts])
        x = np.concatenate([np.asarray(e["x"]) for e in parts])
        want = seq_sum(w, x)
        for e in parts:
            err = abs(e["got"] - want) / max(abs(want), 1e-300)
            worst = max(worst, err)
        cells += 1
    return {"max_mixed_err": worst, "shared_cells": cells, "ranks_seen": len(allv),
            "interior_sampled": sum(r["interior"] for r in allv),
            "interior_bit_identical": all(r["interior_bad"] == 0 for r in allv),
            "rule": "shared boundary cells vs the sequential sum over both neighbours' exchange cells "
                    "(relative error); sampled interior cells bit-identical to the rank's own sequential sum"}


def allreduce_cost(comm, wl, world, dist, iters=100):
    """N > 1: the step's one collective alone -- an all-reduce (sum, fp64) of as many doubles
    as the step's boundary slots (every variant's, wl.shared), through the same libfcx
    communicator on the workload's stream, timed with one HIP event pair around `iters` of
    them after a barrier; max over ranks.  None at N = 1 or without the libfcx communicator."""
    import torch

    if world <= 1 or comm is None or not hasattr(comm, "allreduce_sum"):
        return None
    buf = torch.zeros(wl.shared.numel(), dtype=torch.float64, device=wl.dev)
    s = wl.stream
    for _ in range(10):
        comm.allreduce_sum(buf, s.cuda_stream)
    torch.cuda.synchronize()
    dist.barrier()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(iters):
        comm.allreduce_sum(buf, s.cuda_stream)
    b.record(s)
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / iters
    t = torch.tensor([us], dtype=torch.float64, device=wl.dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"us_per_allreduce": round(float(t.item()), 2), "doubles": int(buf.numel()), "iters": iters,
            "rule": "the step's boundary all-reduce alone (same count, same communicator, the workload's stream): "
                    "one HIP event pair around the iterations, max over ranks"}


def e2e_host(args, variants, sizes=(10_000_000, 32_768)):
    """SURVEY.md 8d end-to-end rate (never `value`): the fields in caller heap arrays (numpy,
    as a Fortran host's ALLOCATEd local_field arrays), every coupling step fcx_step = inputs
    host -> device, the fused kernels, outputs device -> host, synchronised, with the default
    transport (the engine's staging arena, pipelined over chunks on large grids).  Wall time
    per step, one engine per variant at a time."""
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.synthetic import build_case, inputs_for_bench

    out = {"transport": "default: caller heap arrays through the engine's page-locked staging arena "
                        "(FCX_OPT_HOST_STAGING), pipelined H2D/kernel/D2H chunks from 2 x 256K cells",
           "unit": "Mcells/s", "sizes": {}}
    for n in sizes:
        data = inputs_for_bench(n)
        steps = 10 if n >= 1_000_000 else 500
        per = {}
        for v in variants:
            case = build_case(v, n=n, T=args.types, bias=args.bias, data=data if args.types == 1 else None)
            eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                         averages=case.averages)
            for k in range(3 if n >= 1_000_000 else 50):  # first touch, plans, arena, clocks
                eng.step(PHASE_ALL, k * 3600)
            ts = []
            for k in range(steps):
                t0 = time.perf_counter()
                eng.step(PHASE_ALL, k * 3600)
                ts.append(time.perf_counter() - t0)
            staging = eng.staging_bytes()
            eng.close()
            med = float(np.median(ts))
            per[v] = {"us_per_step_median": round(med * 1e6, 1),
                      "us_per_step_p90": round(float(np.percentile(ts, 90)) * 1e6, 1),
                      "Mcells_per_s": round(n / med / 1e6, 1), "staging_MB": round(staging / 1e6, 1)}
            del case
        tot = sum(x["us_per_step_median"] for x in per.values()) * 1e-6
        out["sizes"][str(n)] = {"variants": per, "steps": steps,
                                "value": round(n * len(per) / tot / 1e6, 1),
                                "value_rule": "cells x variants / sum of the variants' median step times"}
    return out


def e2e_concurrent(args, variants, n=32_768, steps=500):
    """The drop-in as the reference deploys it: every bottom model's flux_calculator is its
    own MPI task (flux_calculator.F90:275-298), so the variants' steps run side by side.  One
    engine per variant on its own HIP stream, driven by its own host thread (ctypes releases
    the GIL in fcx_step); a step = all of them from a common start to the last one done, each
    from its caller heap arrays with the default transport.  Wall time per step."""
    import threading

    import torch
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.synthetic import build_case, inputs_for_bench

    data = inputs_for_bench(n)
    streams = [torch.cuda.Stream() for _ in variants]
    cases = [build_case(v, n=n, T=args.types, bias=args.bias, data=data if args.types == 1 else None)
             for v in variants]
    engines = [Engine(c.lf, c.num_surface_types, c.methods, corrections=c.corrections, averages=c.averages,
                      stream=st.cuda_stream) for c, st in zip(cases, streams)]
    total = 50 + steps
    start, done = threading.Barrier(len(engines) + 1), threading.Barrier(len(engines) + 1)
    errors = []

    def worker(e):
        try:
            for k in range(total):
                start.wait()
                e.step(PHASE_ALL, k * 3600)
                done.wait()
        except Exception as ex:  # noqa: BLE001 -- reported by the main thread
            errors.append(ex)
            start.abort()
            done.abort()

    threads = [threading.Thread(target=worker, args=(e,)) for e in engines]
    for t in threads:
        t.start()
    ts = []
    try:
        for k in range(total):
            start.wait()
            t0 = time.perf_counter()
            done.wait()
            if k >= 50:  # first touch, plans, arenas, clocks
                ts.append(time.perf_counter() - t0)
    except threading.BrokenBarrierError:
        pass
    for t in threads:
        t.join()
    for e in engines:
        e.close()
    if errors:
        raise errors[0]
    med = float(np.median(ts))
    return {"us_per_step_median": round(med * 1e6, 1), "us_per_step_p90": round(float(np.percentile(ts, 90)) * 1e6, 1),
            "steps": steps, "engines": len(engines),
            "rule": "every variant's engine on its own stream and host thread, side by side as the reference's "
                    "per-bottom-model MPI tasks; a step = common start to the last engine done"}


def e2e_async(args, variants, n=32_768, steps=500):
    """The variants' steps started one after the other from ONE host thread with
    fcx_step_async (each engine on its own stream), then every engine synchronised: the
    asynchronous phase, no host threads of the caller's.  Transport: the staging arena with
    DMA (FCX_OPT_ZERO_COPY 0) -- one engine's host copies then overlap the others' DMAs;
    with the kernels reading the arena over the link (zero-copy, the one-engine default)
    the three steps take 320 us instead of 258 (bench/baltic_probe.py,
    profiles/r05/baltic_probe.json).  Wall time per step."""
    import torch
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.synthetic import build_case, inputs_for_bench

    data = inputs_for_bench(n)
    streams = [torch.cuda.Stream() for _ in variants]
    cases = [build_case(v, n=n, T=args.types, bias=args.bias, data=data if args.types == 1 else None)
             for v in variants]
    engines = [Engine(c.lf, c.num_surface_types, c.methods, corrections=c.corrections, averages=c.averages,
                      stream=st.cuda_stream, options={"zero_copy": 0}) for c, st in zip(cases, streams)]
    ts = []
    for k in range(50 + steps):
        t0 = time.perf_counter()
        for e in engines:
            e.step_async(PHASE_ALL, k * 3600)
        for e in engines:
            e.synchronize()
        if k >= 50:
            ts.append(time.perf_counter() - t0)
    for e in engines:
        e.close()
    med = float(np.median(ts))
    return {"us_per_step_median": round(med * 1e6, 1), "us_per_step_p90": round(float(np.percentile(ts, 90)) * 1e6, 1),
            "steps": steps, "engines": len(engines),
            "transport": "staging arena + DMA (FCX_OPT_ZERO_COPY 0)",
            "rule": "fcx_step_async of every variant's engine (own stream) from one host thread, then fcx_synchronize "
                    "of each; a step = first start to the last engine synchronised"}


def e2e_library_memory(args, variants, n=32_768, steps=500):
    """The Baltic-size step with the fields in fcx_host_malloc memory -- a host that allocates
    its local_field arrays from the library (c_f_pointer) instead of
    its own heap, inputs first and outputs after them as the reference allocates them
    (flux_calculator.F90:436-560, then prepare:36-42).  Two transports: zero-copy (the default
    at this size: the kernels read and write the arrays in place over the link) and the span
    transport (FCX_OPT_ZERO_COPY 0: device mirrors laid out like the host memory, one or two
    uploads and ONE download per engine and step).  Median wall time per step of the variants one after the other
    (fcx_step) and started together (fcx_step_async from one thread, each engine on its own
    stream, then fcx_synchronize of each)."""
    import torch
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.host_alloc import Arena
    from fcx.synthetic import build_case, inputs_for_bench

    data = inputs_for_bench(n)
    res = {}
    for transport, opts in (("zero_copy", {}), ("spans", {"zero_copy": 0})):
        streams = [torch.cuda.Stream() for _ in variants]
        cases = [build_case(v, n=n, T=args.types, bias=args.bias, data=data if args.types == 1 else None)
                 for v in variants]
        with Arena() as arena:
            for c in cases:
                arena.adopt(c.lf)
            engines = [Engine(c.lf, c.num_surface_types, c.methods, corrections=c.corrections, averages=c.averages,
                              stream=st.cuda_stream, options=opts) for c, st in zip(cases, streams)]
            out = {}
            if transport == "spans":
                out["copies_per_step"] = [list(e.span_runs()) for e in engines]
            for mode in ("sequential", "async"):
                ts = []
                for k in range(50 + steps):
                    t0 = time.perf_counter()
                    if mode == "sequential":
                        for e in engines:
                            e.step(PHASE_ALL, k * 3600)
                    else:
                        for e in engines:
                            e.step_async(PHASE_ALL, k * 3600)
                        for e in engines:
                            e.synchronize()
                    if k >= 50:
                        ts.append(time.perf_counter() - t0)
                out[f"{mode}_us_per_step_median"] = round(float(np.median(ts)) * 1e6, 1)
                out[f"{mode}_us_per_step_p90"] = round(float(np.percentile(ts, 90)) * 1e6, 1)
            for e in engines:
                e.close()
        res[transport] = out
    res.update(steps=steps, engines=len(variants),
               transports="zero_copy: the kernels use the arrays in place (the default at this size); spans: "
                          "device mirrors laid out like the host memory, one copy per run of adjacent arrays "
                          "(FCX_OPT_ZERO_COPY 0)",
               rule="sequential: fcx_step of each variant in turn; async: fcx_step_async of each from one host "
                    "thread, then fcx_synchronize of each; a step = first start to the last engine done")
    return res


def link_bytes(variants, n, args):
    """Bytes one coupling step of the variants moves over the host link from host arrays:
    every distinct input array up, every output array down (the staged transfers)."""
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.synthetic import build_case

    b_in = b_out = 0
    for v in variants:
        c = build_case(v, n=n, T=args.types, bias=args.bias)
        e = Engine(c.lf, c.num_surface_types, c.methods, corrections=c.corrections, averages=c.averages)
        total = e.algorithmic_bytes(PHASE_ALL)  # the plan's distinct arrays read once, written once
        e.close()
        outs = sum(c.lf.field[k].nbytes for k in dict.fromkeys(c.outputs))
        b_in += total - outs - (8 * n if args.bias else 0)  # (the month slice stays on the device)
        b_out += outs
    return b_in, b_out


def relaunch(n):
    """`python bench.py --gpus N` outside a launcher: run this same command under
    torch.distributed.run (one rank per GPU, rendezvous on 127.0.0.1) as a child process,
    before anything touches the GPU, and return its exit code."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def measure(wl, args, world, dist, comm, steps, warmup, t_base=0, cold=False):
    """Warm-up (at least `warmup` steps and MIN_WARMUP_S of device work), then EXACTLY
    `steps` timed steps bracketed by barrier + synchronize, max over ranks.  A step is
    fcx_run of every variant's engine plus, for N > 1, the ONE all-reduce of the boundary
    slots of all variants (libfcx's RCCL communicator) and their finish."""
    import torch

    stream = wl.stream
    group = bool(args.group)

    def step(t, events=None, grouped=group):
        if grouped:  # fcx_run_group: the variants' flux passes as one launch
            wl.run_group(t, events)
        else:
            wl.run(t, events)
        if comm is not None:
            comm.atmos_allreduce(wl.engines)  # the one collective of the step (RCCL over xGMI)

    def pairs(k):
        return [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                 for _ in wl.engines] for _ in range(k)]

    nv = len(wl.engines)
    # event-timed warm-up block: every engine's launch, to pick the dominant one (and report
    # the others); the timed steps then carry ONE event pair, around the dominant launch --
    # each pair in the step costs ~2.5 % of it (bench/event_probe.py)
    probe_steps = max(WARMUP_BLOCK, min(steps, 200))
    ev_probe = pairs(probe_steps)
    # the timed steps' events exist before the warm-up starts: nothing host-side sits between
    # the warm-up and the timed region (an idle GPU drops its clocks)
    ev = pairs(steps)
    # the grouped step's one launch: ONE event pair around the whole timed region, not a pair per
    # step -- an event recorded between two launches on a stream holds the next launch back
    # ~10.5 us (the kernel trace of round 5: 10.5 us between timed launches with per-step
    # pairs, none between the warm-up's, profiles/r05/ev/), 1.4 % of the step
    ev_region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    step(t_base)  # builds the engines' plans
    torch.cuda.synchronize()
    cold_ms = None
    if cold:
        # cold step: one step after an idle gap, as a coupled model runs its flux step
        # between the other components' steps
        if world > 1:
            dist.barrier()
        time.sleep(COLD_IDLE_S)
        t_c = time.perf_counter()
        step(t_base)
        torch.cuda.synchronize()
        cold_ms = (time.perf_counter() - t_c) * 1e3
    def all_ranks(flag):
        """A loop exit every rank takes together: each warm-up step issues the step's
        collective, so a rank-local exit test (wall time) would let the ranks run different
        numbers of all-reduces -- the N > 1 abort of GPUTEST_r04 (a hang under real RCCL).
        MIN over the ranks of the local flag, on the torch group."""
        if world == 1:
            return flag
        t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64, device=wl.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item() > 0.5)

    # warm-up: the clocks reach steady state after ~40 ms of load; a short warm-up timed the
    # ramp (34.7 Gcells/s with 5 steps against 37.5 at steady state, round 1)
    warm, t_w = 0, time.perf_counter()
    while True:
        for _ in range(WARMUP_BLOCK):
            step(t_base + warm * 3600)
            warm += 1
        torch.cuda.synchronize()
        if all_ranks(warm >= warmup and time.perf_counter() - t_w >= MIN_WARMUP_S):
            break
    for k in range(probe_steps):  # still warm-up: the event-timed block, one launch per engine
        step(t_base + (warm + k) * 3600, ev_probe[k], grouped=False)
    torch.cuda.synchronize()
    probe_ms = np.array([[a.elapsed_time(b) for (a, b) in row] for row in ev_probe])  # [steps][variant]
    dom = int(np.argmax(probe_ms.mean(axis=0)))
    if args.kernel_events == "dominant":
        ev = [[p if i == dom else None for i, p in enumerate(row)] for row in ev]
    for k in range(WARMUP_BLOCK):  # back under load after the host read the probe events
        step(t_base + (warm + probe_steps + k) * 3600)
    torch.cuda.synchronize()
    warm += probe_steps + WARMUP_BLOCK
    warmup_s = time.perf_counter() - t_w
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if group:
        ev_region[0].record(stream)
    for k in range(steps):
        step(t_base + k * 3600, None if group else ev[k])
    if group:
        ev_region[1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # per-variant mean kernel time: the timed steps where they carry events (the dominant
    # engine; every engine with --kernel-events all), the event-timed warm-up block otherwise
    kern_mean = probe_ms.mean(axis=0)
    timed = {} if group else {i: np.array([row[i][0].elapsed_time(row[i][1]) for row in ev])
                              for i in range(nv) if ev and ev[0][i] is not None}
    # device time per grouped step: the launch plus the kernel boundary to the next (~0-1.5 us;
    # the rocprof trace's mean launch duration is the cross-check)
    group_ms = ev_region[0].elapsed_time(ev_region[1]) / steps if group and steps else None
    for i, x in timed.items():
        kern_mean[i] = x.mean()
    t_max = elapsed
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=wl.dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
    del stream
    return {"t_max": t_max, "kern_mean": kern_mean, "dom": dom, "timed_events": sorted(timed),
            "cold_ms": cold_ms, "warm": warm, "warmup_s": warmup_s, "group_ms": group_ms}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args.gpus))
    variants = tuple(v for v in args.variants.split(",") if v)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    gpu = 0 if args.same_device else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    from fcx.workload import Workload
    sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "bench"))
    from pmc_traffic import traffic_key

    f32 = args.precision == "f32"
    # the library's own RCCL communicator for the boundary exchange (N > 1); the unique id is
    # broadcast over torch.distributed.  Same-device rehearsals on one GPU (RCCL refuses two
    # ranks per device) keep torch's all-reduce of the slots, unless FCX_RCCL_LIBRARY names a
    # stand-in that allows it (tests/cpp/mock_rccl.cpp: the libfcx exchange code itself runs)
    comm = None
    if world > 1 and args.collective == "rccl" and (not args.same_device or os.environ.get("FCX_RCCL_LIBRARY")):
        from fcx.comm import Comm

        comm = Comm.from_torch(gpu)

    class TorchCollective:  # rehearsal only
        def atmos_allreduce(self, engines):
            dist.all_reduce(wl.shared)
            wl.finish()

    coll = comm if comm is not None else (TorchCollective() if world > 1 else None)

    engine_options = {"tiled_layout": args.tiled, "nontemporal": args.nontemporal}
    if args.max_blocks is not None:
        engine_options["max_blocks"] = args.max_blocks
    # this rank's APPLE range (decomp_def.F90:23-31): weak scaling (every rank owns args.cells
    # cells of a grid of world * cells) or a fixed global grid (--global-cells, strong)
    n_global = args.global_cells if args.global_cells else args.cells * world
    wl = Workload(n_global, rank, world, variants, types=args.types, bias=args.bias, precision=args.precision,
                  atmos=bool(args.atmos), caller_device=args.caller_device, device=gpu, atmos_map=args.atmos_map,
                  stream=torch.cuda.current_stream(dev), engine_options=engine_options)
    n, la = wl.n, wl.la
    torch.cuda.synchronize()
    layout = wl.engines[0].device_layout()
    # algorithmic bytes of one fcx_run: every distinct field array read once / written once,
    # plus (fused accumulation) 4+8 B/cell of atmosphere index and weight and the outputs
    alg_bytes = wl.alg_bytes

    # config 5 (--bias): hourly steps whose timed half crosses 1961-01-31 -> 02-01, so the
    # bias month slice changes inside the timed region (init_date 19610101)
    t_base = 31 * 86400 - 3600 * (args.steps // 2) if args.bias else 0
    # fcx_run_group merges the fused T = 1 passes (the accumulation in the flux kernel, no grid
    # cap); elsewhere the engines would run one by one inside it, so the one-launch roofline
    # does not apply and the step runs them as fcx_run
    args.group = int(bool(args.group) and la is not None and len(variants) >= 2 and (args.types == 1 or not f32)
                     and (args.max_blocks is None or args.max_blocks <= 0))
    m = measure(wl, args, world, dist, coll, args.steps, args.warmup, t_base, cold=True)
    t_max = m["t_max"]
    ms_per_step = t_max / args.steps * 1e3
    cells_per_step = n_global * len(variants)
    value = cells_per_step * args.steps / t_max / 1e6

    mean_ms = m["kern_mean"]
    dom = m["dom"]
    grouped = m["group_ms"] is not None
    if grouped:  # the one launch of the step: every variant's algorithmic bytes
        dom_bytes, dom_ms = int(sum(alg_bytes)), m["group_ms"]
        dom_name = f"cells_atmos_group_kernel[{'+'.join(variants)}]"
    else:
        dom_bytes, dom_ms = int(alg_bytes[dom]), float(mean_ms[dom])
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    per_variant = {
        v: {"kernel_ms": round(float(mean_ms[i]), 4),
            "alg_bytes": int(alg_bytes[i]),
            "bytes_per_cell": round(alg_bytes[i] / n, 3),
            "GBps": round(alg_bytes[i] / (mean_ms[i] * 1e-3) / 1e9, 1)}
        for i, v in enumerate(variants)}
    # the accumulation runs inside the flux kernel (T = 1, or T >= 2 with the register averages
    # in fp64) unless a grid-stride cap is set; otherwise it is its own kernel after it
    fused = la is not None and (args.max_blocks is None or args.max_blocks <= 0) and (args.types == 1 or not f32)
    traffic, traffic_source = None, None
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tfile):
        try:
            t = json.load(open(tfile))
            # the timed launch carries the accumulation only when it is fused (fp64)
            tkey = traffic_key("GROUP" if grouped else variants[dom], n, args.types, args.bias, fused,
                               args.precision)
            traffic = t.get(tkey)
            if traffic is not None:
                traffic_source = t.get("_sources", {}).get(tkey)
        except Exception:
            traffic = None

    mg = multi_gpu_check(wl, world, rank, dist) if la is not None else None
    ar = allreduce_cost(comm, wl, world, dist)

    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "Mcells/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "warmup_run": {"steps": m["warm"], "seconds": round(m["warmup_s"], 3),
                       "rule": f"at least --warmup steps and at least {MIN_WARMUP_S} s of device work, then an "
                               "event-timed block (every engine) and one more block without events"},
        "timed_ms": round(t_max * 1e3, 3),
        "cold_step_ms": round(m["cold_ms"], 4),
        "higher_is_better": True,
        "scaling": "strong" if args.global_cells else "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (SURVEY.md 8d distributions, seeded PCG64)",
        "config": {
            "workload": ("config3/4: synthetic exchange grid, CCLM+MOM5+RCO fused flux kernels "
                         + ("in one launch per coupling step (fcx_run_group)" if args.group else
                            "back-to-back per coupling step")
                         + (" + exchange->atmosphere accumulation" if la is not None else "")
                         + (" (its own kernel after the flux pass)" if la is not None and not fused else "")
                         + (", fp32 variant (config 5)" if f32 else "") + ", inputs HBM-resident"),
            "cells_per_gpu": n,
            "cells_global": n_global,
            "cells_per_step": cells_per_step,
            "variants": list(variants),
            "surface_types": args.types,
            "bias_corrections": bool(args.bias),
            "grids": "u/v grids = t grid",
            "field_layout": ("caller's contiguous device arrays" if args.caller_device else
                             "engine-owned mirrors, " + (f"tile-blocked ({layout[0]}-cell tiles, tile stride "
                                                         f"{layout[1]} elements)" if layout[1] > layout[0]
                                                         else "contiguous")),
            "parallelism": f"dp{world} (APPLE contiguous cell ranges)"
                           + (f", REHEARSAL: all ranks on GPU 0 over {args.backend}" if args.same_device else ""),
            "atmos_accumulation": (f"6 fluxes -> {la.n_atmos} atmosphere cells per GPU (1 per ~4 "
                                   f"exchange cells, {args.atmos_map} runs), one all-reduce of the shared "
                                   "boundary cells per step"
                                   + ((" (libfcx RCCL communicator" + (", FCX_RCCL_LIBRARY stand-in)"
                                                                         if os.environ.get("FCX_RCCL_LIBRARY") else ")"))
                                      if comm is not None else
                                      " (torch.distributed, rehearsal)" if world > 1 else " (none needed at N=1)")
                                   if la is not None else "off"),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": (dom_name if grouped else
                       f"cells_atmos_kernel[{variants[dom]}]" if fused else f"cells_kernel[{variants[dom]}]"),
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_source,
            "alg_bytes_per_launch": dom_bytes,
            "alg_bytes_rule": ("every distinct field array read once and written once, the atmosphere outputs, "
                               "a weight per exchange cell and the exchange->atmosphere map as the launch reads it "
                               "(halo launches and fp32: start bits, prefix counts and one cell per segment; "
                               "otherwise a 4-B index per cell; DESIGN.md section 3)"),
            "mean_kernel_ms": round(dom_ms, 4),
            "events": ("one HIP event pair around the timed steps on the launches' stream, mean per step: the "
                       "step's one launch (fcx_run_group: the variants' fused flux passes in one grid) and its "
                       "kernel boundary; no events between the timed launches" if grouped else
                       "one HIP event pair per timed step, around the dominant engine's launch on its stream "
                       "(picked in an event-timed warm-up block of every engine)" if args.kernel_events == "dominant"
                       else "HIP event pairs around every engine's launch in every timed step"),
        },
        "kernels": per_variant,
        "kernels_rule": ("kernel_ms of each variant's own launch, from the event-timed warm-up block (one launch per "
                         "engine); the timed steps run them as one group launch" if grouped else
                         "kernel_ms from the timed steps' events for " + ", ".join(variants[i] for i in m["timed_events"])
                         + ("; from the event-timed warm-up block for the others" if len(m["timed_events"]) < len(variants)
                            else "")),
    }
    if mg is not None:
        out["multi_gpu_check"] = mg
    if ar is not None:
        out["allreduce"] = ar
    wl.close()
    del wl
    torch.cuda.synchronize()

    # the same workload on the other atmosphere map (periodic: no carried segment, no fix-up)
    if args.other_map and args.atmos:
        other = "periodic" if args.atmos_map == "random" else "random"
        wo = Workload(n_global, rank, world, variants, types=args.types, bias=args.bias, precision=args.precision,
                      atmos=True, caller_device=args.caller_device, device=gpu, atmos_map=other,
                      stream=torch.cuda.current_stream(dev), engine_options=engine_options)
        wl = wo
        mo = measure(wo, args, world, dist, coll if comm is None else comm, args.steps, args.warmup)
        ko = mo["kern_mean"]
        do = mo["dom"]
        out["other_map"] = {
            "atmos_map": other,
            "value": round(n_global * len(variants) * args.steps / mo["t_max"] / 1e6, 1),
            "unit": "Mcells/s",
            "ms_per_step": round(mo["t_max"] / args.steps * 1e3, 4),
            "dominant_kernel_ms": round(float(ko[do]), 4),
            "frac": round(wo.alg_bytes[do] / (ko[do] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        }
        if mo["group_ms"] is not None:
            out["other_map"]["group_kernel_ms"] = round(mo["group_ms"], 4)
            out["other_map"]["group_frac"] = round(sum(wo.alg_bytes) / (mo["group_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        wo.close()
        del wo, wl
        torch.cuda.synchronize()

    # config 5's fp32 kernels on the same workload (N = 1): Mcells/s and the roofline fraction
    # of the step's one launch, next to the fp64 line
    if args.config5 and world == 1 and not f32 and args.atmos:
        w5 = Workload(n_global, rank, world, variants, types=args.types, bias=args.bias, precision="f32",
                      atmos=True, caller_device=args.caller_device, device=gpu, atmos_map=args.atmos_map,
                      stream=torch.cuda.current_stream(dev), engine_options=engine_options)
        wl = w5
        m5 = measure(w5, args, world, dist, None, args.steps, args.warmup)
        k5, d5 = m5["kern_mean"], m5["dom"]
        g5 = m5["group_ms"]
        out["config5_fp32"] = {
            "workload": "the same synthetic grid and variants in the fp32 engine (BASELINE configs[4]'s fp32 kernel "
                        "variant): fp32 fields and arithmetic, the accumulation's weights, products and sums in fp64",
            "value": round(n_global * len(variants) * args.steps / m5["t_max"] / 1e6, 1),
            "unit": "Mcells/s",
            "ms_per_step": round(m5["t_max"] / args.steps * 1e3, 4),
            "alg_bytes_per_step": int(sum(w5.alg_bytes)),
            "frac": round(sum(w5.alg_bytes) / ((g5 if g5 is not None else float(k5[d5])) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "kernel_ms": round(g5 if g5 is not None else float(k5[d5]), 4),
            "dtype": "f32",
            "tolerance": "tests/test_gpu_fp32.py: the kernel's arithmetic within 64 fp32 ulps of the fp64 oracle on "
                         "the same rounded inputs, or 4x the oracle's movement under 16-ulp perturbations "
                         "(profiles/r06/.../fp32_error_*.json)",
        }
        w5.close()
        del w5, wl
        torch.cuda.synchronize()

    # config 4 at this N: the fixed 40M-cell grid over the same ranks (strong scaling)
    if args.config4 and not args.global_cells:
        w4 = Workload(args.config4, rank, world, variants, types=1, precision=args.precision,
                      atmos=bool(args.atmos), device=gpu, stream=torch.cuda.current_stream(dev),
                      engine_options=engine_options, atmos_map=args.atmos_map)
        wl = w4
        m4 = measure(w4, args, world, dist, coll if comm is None else comm, args.steps, args.warmup)
        k4 = m4["kern_mean"]
        d4 = m4["dom"]
        mg4 = multi_gpu_check(w4, world, rank, dist) if w4.la is not None else None
        ar4 = allreduce_cost(comm, w4, world, dist)
        out["config4"] = {
            "baseline_config": "BASELINE.json configs[3]: the 40M-cell grid sharded 8 ways by decomp_def ranges -- "
                               "THE 1/2/4/8-GPU strong-scaling curve (this object at N = 1, 2, 4, 8); the line's own "
                               "`value` is weak scaling (10M cells per GPU)",
            "workload": "config 4: fixed synthetic grid sharded by APPLE ranges over the ranks (strong scaling), "
                        "CCLM+MOM5+RCO fused kernels + accumulation, one all-reduce of the boundary slots per step, "
                        f"{args.atmos_map} atmosphere map",
            "cells_global": args.config4,
            "cells_per_gpu": w4.n,
            "value": round(args.config4 * len(variants) * args.steps / m4["t_max"] / 1e6, 1),
            "unit": "Mcells/s",
            "ms_per_step": round(m4["t_max"] / args.steps * 1e3, 4),
            "scaling": "strong",
            "steps": args.steps,
            "warmup_steps_run": m4["warm"],
            "dominant_kernel_ms": round(float(k4[d4]), 4),
            "frac": round(w4.alg_bytes[d4] / (k4[d4] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        }
        if m4["group_ms"] is not None:
            out["config4"]["group_kernel_ms"] = round(m4["group_ms"], 4)
            out["config4"]["group_frac"] = round(sum(w4.alg_bytes) / (m4["group_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        out["config4"]["ranks_seen"] = mg4["ranks_seen"] if mg4 is not None else world
        if mg4 is not None:
            out["config4"]["multi_gpu_check"] = mg4
        if ar4 is not None:
            out["config4"]["allreduce_us_per_step"] = ar4["us_per_allreduce"]
        w4.close()
        del w4, wl
        torch.cuda.synchronize()

    if rank == 0 and world == 1 and args.e2e:
        out["e2e"] = e2e_host(args, variants)
    if rank == 0 and world == 1 and not args.no_cpu:
        # the reference path on this box's host cores at BASELINE's config sizes: config 1/2's
        # Baltic-size grid (32,768 cells) and this workload's size, on one core (one MPI rank
        # of the reference) and on the box's CPU share as APPLE-range ranks (cpu_legs.py)
        import cpu_legs

        legs = cpu_legs.legs(variants, sizes=(32_768, n), seconds=args.cpu_seconds)
        mine = legs["sizes"][str(n)]
        one = mine["one_core"]
        out["cpu_baseline"] = {
            "value": one["value"], "unit": "Mcells/s", "cores": 1, "kind": one["kind"],
            "sample": one["sample"] + " (this workload's size and inputs; the reference's call order)",
            "sizes": legs["sizes"], "threads_all_cores": legs["threads"],
            "affinity_cpus": legs["affinity_cpus"], "machine_cpus": legs["machine_cpus"],
            "rule": "one_core: the reference flux_lib on 1 thread = one reference MPI rank; all_cores: the same "
                    "on threads_all_cores processes over APPLE ranges (this box's CPU share), step = common "
                    "barrier to the last rank; same inputs as the GPU workload of that size"}
        out["cpu_baseline_all_cores"] = mine["all_cores"]
        out["host_cpu"] = host_cpu()
        if "e2e" in out and "32768" in out["e2e"]["sizes"]:
            e = out["e2e"]["sizes"]["32768"]
            c1, cp = legs["sizes"]["32768"]["one_core"], legs["sizes"]["32768"]["all_cores"]
            gpu_us = sum(v["us_per_step_median"] for v in e["variants"].values())
            out["baltic_size"] = {
                "cells": 32_768, "variants": list(variants),
                "gpu_dropin_host_arrays_us_per_step": round(gpu_us, 1),
                "gpu_dropin_Mcells_per_s": e["value"],
                "cpu_one_core_us_per_step": c1["us_per_step"],
                "cpu_all_cores_us_per_step": cp["us_per_step"], "cpu_all_cores_cores": cp["cores"],
                "gpu_vs_all_cores": round(cp["us_per_step"] / gpu_us, 2),
                "rule": "one coupling step of every variant from the caller's host arrays (e2e, fcx_step with the "
                        "default transport) against the reference on this box's host cores, same grid size"}
            conc = e2e_concurrent(args, variants)
            out["baltic_size"]["gpu_dropin_concurrent"] = conc
            out["baltic_size"]["gpu_concurrent_vs_all_cores"] = round(cp["us_per_step"] / conc["us_per_step_median"], 2)
            asy = e2e_async(args, variants)
            out["baltic_size"]["gpu_dropin_async"] = asy
            out["baltic_size"]["gpu_async_vs_all_cores"] = round(cp["us_per_step"] / asy["us_per_step_median"], 2)
            lib = e2e_library_memory(args, variants)
            out["baltic_size"]["gpu_dropin_library_memory"] = lib
            # one ratio per transport and mode (no best-of-two after the fact)
            out["baltic_size"]["gpu_library_memory_vs_all_cores"] = {
                f"{tr}_{mode}": round(cp["us_per_step"] / lib[tr][f"{mode}_us_per_step_median"], 2)
                for tr in ("spans", "zero_copy") for mode in ("sequential", "async")}
            # the host link's bound: the step's fields must cross it once
            # each way; measured both directions at once on this box
            from link_probe import link_rates
            try:
                lk = link_rates(*link_bytes(variants, 32_768, args))
            except Exception as ex:  # a measurement beside the line: never the line's end
                out["baltic_size"]["host_link"] = {"error": f"{type(ex).__name__}: {ex}"}
                lk = None
            if lk is not None:
                both = lk["256MiB"]["both_GBps"]
                b_step = lk["step"]["h2d_bytes"] + lk["step"]["d2h_bytes"]
                both = max(both, lk["step"]["both_GBps"])
                st = lk["step"]
                duplex = max(st["h2d_bytes"] / st["h2d_GBps"], st["d2h_bytes"] / st["d2h_GBps"]) / 1e3
                out["baltic_size"]["host_link"] = dict(lk, bound_us=round(b_step / both / 1e3, 1),
                                                       bound_vs_all_cores=round(cp["us_per_step"] / (b_step / both / 1e3), 2),
                                                       bound_duplex_us=round(duplex, 1),
                                                       rule="bound_us: the step's input bytes up plus output bytes down at "
                                                            "the best rate this probe measured for both directions at once "
                                                            "(the step's sizes or 256 MiB copies); bound_duplex_us: the "
                                                            "slower direction alone, the floor if the two directions fully "
                                                            "overlap (the engines' own copies do overlap them in part, "
                                                            "DESIGN.md section 7); the host copies between the caller's "
                                                            "arrays and page-locked memory come on top of either")
                # the library-memory step against the link's duplex floor
                out["baltic_size"]["gpu_library_memory_vs_duplex_floor"] = {
                    f"{tr}_{mode}": round(lib[tr][f"{mode}_us_per_step_median"] / max(duplex, 1e-9), 3)
                    for tr in ("zero_copy", "spans") for mode in ("sequential", "async")}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
