#!/usr/bin/env python3
"""Row f3 measurement: the exchange -> model remap (fcx_add_remap, atmos_kernel on the model
grid's CSR) on config-3 sizes.  10M exchange cells (CCLM, T=1, fields HBM-resident), a
2.5M-cell model grid (synthetic_model_map: runs of 1..8 exchange cells per model cell,
scattered; 1 or 2 links per exchange cell), the 6 fluxes OASIS would send to the bottom
model.  The remap time is the step with the remap minus the step without it (HIP events,
medians of interleaved rounds); the kernel alone is in the rocprof summary of the same run.

Algorithmic bytes of one remap launch: per link 4 (column) + 8 (weight) + 8 per field (the
gathered value); per model cell 4 (row pointer) + 8 per field (the written sum).

  python components.flux_calculator_amd/bench/remap_bench.py [--cells N] [--model M]
  python components.flux_calculator_amd/bench/remap_bench.py --map geometric [--side 1300]

--map geometric: the exchange grid of an atmosphere grid (side^2 cells) intersected with a
finer ocean grid (fcx.parallel.geometric_maps; 9.2M exchange cells, 3.0M ocean cells at
side 1300), the conservative exchange -> ocean remap (one link per exchange cell), so a
model cell's links come from a few atmosphere rows as on the real grids.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))
FIELDS = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--model", type=int, default=2_500_000)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--map", choices=("synthetic", "geometric"), default="synthetic")
    ap.add_argument("--side", type=int, default=1300, help="geometric: atmosphere cells per side")
    ap.add_argument("--pack", default="0,2",
                    help="FCX_OPT_REMAP_PACK values to compare (0: gather from the field arrays, "
                         "2: packed records)")
    ap.add_argument("--links", default="1,2", help="links per exchange cell (synthetic map)")
    ap.add_argument("--atmos", action="store_true",
                    help="every engine also accumulates the six fluxes to the atmosphere (fused), as "
                         "in a coupled step")
    a = ap.parse_args()
    import torch

    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.parallel import geometric_maps, synthetic_model_map
    from fcx.synthetic import build_case, inputs_for_bench

    geo = geometric_maps(a.side)[1] if a.map == "geometric" else None
    if geo is not None:
        a.cells, a.model = geo.src.size, geo.n_model
    n, m = a.cells, a.model
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    data = {k: torch.as_tensor(v).to(dev) for k, v in inputs_for_bench(n).items()}
    case = build_case("CCLM", n=n, T=1, device=dev, data=data)
    if a.atmos:
        from fcx.parallel import local_atmos, synthetic_atmos_map
        amap = synthetic_atmos_map(n)
        la = local_atmos(amap, 0, 1)

        def atmos_spec():
            outs = {k: torch.empty(la.n_atmos, dtype=torch.float64, device=dev) for k, _ in FIELDS}
            return {"local": la, "fields": [(2, 1, g, k, outs[k]) for k, g in FIELDS]}
    engines = {"none": Engine(case.lf, 1, case.methods, device=0, stream=stream.cuda_stream,
                              **({"atmos": atmos_spec()} if a.atmos else {}))}
    alg = {}
    packs = [int(x) for x in a.pack.split(",")]
    for links in ((1,) if geo is not None else tuple(int(x) for x in a.links.split(","))):
        mm = geo if geo is not None else synthetic_model_map(n, m, links_per_cell=links)
        nl, nf = mm.src.size, len(FIELDS)
        for pack in packs:
            outs = {k: torch.empty(m, dtype=torch.float64, device=dev) for k, _ in FIELDS}
            rm = {"n_dst": m, "src": mm.src, "dst": mm.dst, "w": mm.weight,
                  "fields": [(2, 1, g, k, outs[k]) for k, g in FIELDS]}
            key = f"{links} link(s)/cell pack={pack}"
            engines[key] = Engine(case.lf, 1, case.methods, device=0, stream=stream.cuda_stream, remaps=[rm],
                                  options={"remap_pack": pack}, **({"atmos": atmos_spec()} if a.atmos else {}))
            engines[key].run(PHASE_ALL, 0)
            sc, packed = engines[key].remap_info(0)
            alg[key] = {"links": int(nl), "bytes": int(nl * (4 + 8 + 8 * nf) + m * (4 + 8 * nf)),
                        "scatter": round(sc, 3), "packed": packed}
    times = {k: [] for k in engines}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        order = list(engines)
        np.random.default_rng(r).shuffle(order)
        for k in order:
            eng = engines[k]
            eng.run(PHASE_ALL, 0)
            e0.record(stream)
            for _ in range(a.reps):
                eng.run(PHASE_ALL, 0)
            e1.record(stream)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.reps)
    base = float(np.median(times["none"]))
    out = {"map": a.map, "cells": n, "model_cells": m, "fields": len(FIELDS), "atmos": a.atmos,
           "step_ms_without_remap": round(base, 4)}
    for k, v in alg.items():
        ms = float(np.median(times[k])) - base
        out[k] = {**v, "remap_ms": round(ms, 4), "GBps_algorithmic": round(v["bytes"] / (ms * 1e-3) / 1e9, 1)}
    for e in engines.values():
        e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
