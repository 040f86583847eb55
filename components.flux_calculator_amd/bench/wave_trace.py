#!/usr/bin/env python3
"""Wave timeline of the fused kernels (measurement tool; needs an FCX_WAVE_TRACE A/B build).

  tools/build_variant.sh ab/trace -DFCX_WAVE_TRACE=1
  FCX_LIBRARY=ab/trace/libfcx.so python wave_trace.py [--precision f32] [--types 2]

Every wave of cells_atmos_kernel stores {start, end, HW_ID | XCC_ID << 32, loop entry} (the
device's constant wall clock; `end` after the wave's own stores completed; loop entry = the
first tile's first instruction, after the scalar set-up).  The tool runs the bench workload
(3 variants, 10M cells, random-run atmosphere map, caller device arrays) back to back and
reads the last step's three launches.  Per launch it reports the span, the wave lifetimes,
the occupancy over time (ramp-up until 90 % of the peak count of resident waves, drain after
the last time at 90 %) and the wave-time lost against a launch that held its peak count
from the first to the last timestamp; the gaps between consecutive launches; and how much
waves that share a SIMD start together (lock-step) early and late in the launch; the gap
between one wave's end and the next wave's start in the same wave slot; and when each XCD
finished its share of the workgroups.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))

VARIANTS = ("CCLM", "MOM5", "RCO")
FIELDS = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))


def analyse(tr, khz, bin_us):
    ok = tr[:, 0] != 0
    tr = tr[ok]
    us = 1e3 / khz  # wall-clock ticks -> microseconds
    t0 = tr[:, 0].min()
    start = (tr[:, 0] - t0) * us
    end = (tr[:, 1] - t0) * us
    span = float(end.max())
    life = end - start
    # resident waves over time: +1 at start, -1 at end
    ev = np.concatenate([np.stack([start, np.ones_like(start)], 1), np.stack([end, -np.ones_like(end)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    t, d = ev[:, 0], ev[:, 1]
    active = np.cumsum(d)
    peak = float(active.max())
    dt = np.diff(t, append=t[-1])
    wave_us = float((active * dt).sum())
    hi = np.nonzero(active >= 0.9 * peak)[0]
    ramp = float(t[hi[0]]) if len(hi) else span
    drain = float(span - t[hi[-1]]) if len(hi) else span
    bins = np.arange(0.0, span + bin_us, bin_us)
    occ = [float(((np.minimum(end, b + bin_us) - np.maximum(start, b)).clip(0)).sum() / bin_us)
           for b in bins[:-1]]
    # SIMD of every wave: HW_ID simd [5:4], cu [11:8], sh [12], se [15:13]; XCC_ID [3:0]
    hw, xcc = tr[:, 2].astype(np.int64) & 0xFFFFFFFF, (tr[:, 2].astype(np.int64) >> 32) & 0xF
    setup = (tr[:, 3].astype(np.float64) - tr[:, 0]) * us
    simd = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 7) | (((hw >> 8) & 0xF) << 3) | ((hw >> 4) & 3)
    # lock-step: per wave, other waves of the same SIMD that started within 0.2 us of it
    close = np.zeros(len(start))
    order = np.lexsort((start, simd))
    s_sorted, k_sorted = start[order], simd[order]
    for j in range(1, 4):
        same = (k_sorted[j:] == k_sorted[:-j]) & (s_sorted[j:] - s_sorted[:-j] < 0.2)
        close[order[j:]] += same
        close[order[:-j]] += same
    # refill gaps: consecutive waves of one wave slot (SIMD + HW_ID wave_id [3:0]); mid-span
    slot = (simd << 4) | (hw & 0xF)
    o2 = np.lexsort((start, slot))
    same_slot = slot[o2][1:] == slot[o2][:-1]
    gap = (start[o2][1:] - end[o2][:-1])[same_slot]
    gmid = gap[(start[o2][1:][same_slot] > 0.2 * span) & (start[o2][1:][same_slot] < 0.8 * span)]
    # XCD balance: every XCD gets 1/8 of the workgroups (round-robin dispatch)
    xcds = {}
    for x in np.unique(xcc):
        m = xcc == x
        xcds[int(x)] = {"waves": int(m.sum()), "last_end_us": round(float(end[m].max()), 2),
                        "mean_lifetime_us": round(float(life[m].mean()), 2)}
    xe = np.array([v["last_end_us"] for v in xcds.values()])
    early = start < 0.1 * span
    late = (start > 0.3 * span) & (start < 0.7 * span)
    return {
        "waves": int(len(tr)),
        "span_us": round(span, 2),
        "peak_resident_waves": int(peak),
        "simds_seen": int(len(np.unique(simd))),
        "lifetime_us": {"mean": round(float(life.mean()), 2), "p10": round(float(np.percentile(life, 10)), 2),
                        "p90": round(float(np.percentile(life, 90)), 2),
                        "first_10pct_of_span": round(float(life[early].mean()), 2),
                        "mid_span": round(float(life[late].mean()), 2)},
        "setup_us_start_to_loop": {"median": round(float(np.median(setup)), 3),
                                   "p90": round(float(np.percentile(setup, 90)), 3)},
        "ramp_us_to_90pct": round(ramp, 2),
        "drain_us_from_90pct": round(drain, 2),
        "lost_us_vs_peak_occupancy": round(span - wave_us / peak, 2),
        "same_simd_starts_within_0p2us": {"first_10pct_of_span": round(float(close[early].mean()), 2),
                                          "mid_span": round(float(close[late].mean()), 2)},
        "slot_refill_gap_us_mid_span": {"median": round(float(np.median(gmid)), 3) if len(gmid) else None,
                                        "p10": round(float(np.percentile(gmid, 10)), 3) if len(gmid) else None,
                                        "p90": round(float(np.percentile(gmid, 90)), 3) if len(gmid) else None},
        "xcd_last_end_spread_us": round(float(xe.max() - xe.min()), 2),
        "xcds": xcds,
        "occupancy_per_bin": [round(x, 1) for x in occ],
        "_t0": int(t0), "_end": int(tr[:, 1].max()),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--types", type=int, default=1)
    ap.add_argument("--precision", choices=("f64", "f32"), default="f64")
    ap.add_argument("--steps", type=int, default=200, help="back-to-back steps before the traced one")
    ap.add_argument("--bin-us", type=float, default=2.0)
    a = ap.parse_args()

    import torch
    from fcx import _lib
    from fcx.basic import PHASE_ALL, PHASE_NORMAL
    from fcx.engine import Engine
    from fcx.parallel import BlockedRandomAtmosMap
    from fcx.synthetic import as_dtype, build_case, inputs_for_bench

    lib = _lib.load()
    if not hasattr(lib, "fcx_debug_wave_trace"):
        sys.exit("wave_trace.py needs an FCX_WAVE_TRACE build (FCX_LIBRARY=ab/trace/libfcx.so)")
    lib.fcx_debug_wave_trace.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_int64)]
    n = a.cells
    dev = torch.device("cuda", 0)
    data = {k: torch.as_tensor(v).to(dev) for k, v in inputs_for_bench(n).items()}
    stream = torch.cuda.current_stream(dev)
    la = BlockedRandomAtmosMap().local(0, n, 0, 1, n)
    f32 = a.precision == "f32"
    s0 = 0 if a.types >= 2 else 1
    engines = []
    for v in VARIANTS:
        c = build_case(v, n=n, T=a.types, device=dev, data=data if a.types == 1 else None)
        c = as_dtype(c, "float32") if f32 else c
        outs = {name: torch.empty(la.n_atmos, dtype=torch.float32 if f32 else torch.float64, device=dev)
                for name, _ in FIELDS}
        engines.append((Engine(c.lf, c.num_surface_types, c.methods, corrections=c.corrections,
                               averages=c.averages, device=0, stream=stream.cuda_stream,
                               atmos={"local": la, "fields": [(PHASE_NORMAL, s0, g, name, outs[name])
                                                              for name, g in FIELDS]},
                               options={"atmos_in_run": 0, "timing": 0, "host_staging": 0}), c, outs))
    stride = (n // 64 + 8192) * 4  # words per launch: {start, end, hw, xcc} per wave
    buf = torch.zeros(len(VARIANTS) * stride, dtype=torch.int64, device=dev)
    khz = ctypes.c_int64(0)
    _lib.check(lib.fcx_debug_wave_trace(ctypes.c_void_p(buf.data_ptr()), stride, len(VARIANTS), ctypes.byref(khz)))
    for k in range(a.steps + 1):  # launch j of a step lands in slot j
        for e, _, _ in engines:
            e.run(PHASE_ALL, k * 3600)
        if k % 10 == 9:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    lib.fcx_debug_wave_trace(None, 0, 1, ctypes.byref(khz))
    raw = buf.cpu().numpy().view(np.uint64).reshape(len(VARIANTS), -1, 4)
    out = {"cells": n, "types": a.types, "precision": a.precision, "wall_clock_khz": khz.value,
           "bin_us": a.bin_us, "launches": {}}
    prev_end = None
    for v, r in zip(VARIANTS, raw):
        s = analyse(r, khz.value, a.bin_us)
        if prev_end is not None:
            s["gap_after_previous_launch_us"] = round((s["_t0"] - prev_end) * 1e3 / khz.value, 2)
        prev_end = s["_end"]
        out["launches"][v] = {k: x for k, x in s.items() if not k.startswith("_")}
    for e, _, _ in engines:
        e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
