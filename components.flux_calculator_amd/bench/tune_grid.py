#!/usr/bin/env python3
"""Grid-size sweep (FCX_OPT_MAX_BLOCKS) of the three cell-kernel families on the config-3
workload: the fp64 flux kernel, the fp64 kernel with the fused atmosphere accumulation, and
the fp32 kernel.  Candidate grids include the ones that give every wave the same number of
units (no half-empty last round).  Interleaved rounds, median of HIP-event times, reported
as GB/s of algorithmic bytes (cdna_hip_programming.md 5.4).

  python tune_grid.py [--cells N] [--rounds R] [--families fused,f64,f32]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))

ATM = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))


def grids(units_per_block_round, waves_units):
    """Caps giving k units per thread/wave exactly, for k = 1..4, plus the round numbers."""
    out = {1024, 2048, 4096, 8192, 16384, 0}
    for k in (1, 2, 3, 4, 6):
        out.add(int(np.ceil(waves_units / (units_per_block_round * k))))
    return sorted(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--families", default="fused,f64,f32")
    ap.add_argument("--out", default=None)
    ap.add_argument("--types", type=int, default=1,
                    help="surface types (>= 2: the type-0 averages are accumulated, as in bench.py)")
    a = ap.parse_args()
    import torch

    from fcx.basic import PHASE_ALL, PHASE_NORMAL
    from fcx.engine import Engine
    from fcx.parallel import PeriodicAtmosMap
    from fcx.synthetic import as_dtype, build_case, inputs_for_bench

    n = a.cells
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    data = {k: torch.as_tensor(v).to(dev) for k, v in inputs_for_bench(n).items()}
    la = PeriodicAtmosMap().local(0, n, 0, 1, n)
    engines = {}
    for fam in a.families.split(","):
        for v in ("CCLM", "MOM5", "RCO"):
            c = build_case(v, n=n, T=a.types, device=dev, data=data if a.types == 1 else None)
            atmos = None
            if fam == "fused":
                outs = [torch.empty(la.n_atmos, dtype=torch.float64, device=dev) for _ in ATM]
                s0 = 0 if a.types >= 2 else 1
                atmos = {"local": la, "fields": [(PHASE_NORMAL, s0, g, name, o) for (name, g), o in zip(ATM, outs)]}
            if fam == "f32":
                c = as_dtype(c, "float32")
            e = Engine(c.lf, c.num_surface_types, c.methods, averages=c.averages, device=0,
                       stream=stream.cuda_stream, atmos=atmos)
            if fam == "fused":
                units, per_block = (n + 127) // 128, 4  # wave tiles, 4 waves per block
            else:
                units, per_block = (n + (4 if fam == "f32" else 2) - 1) // (4 if fam == "f32" else 2), 256
            engines[(fam, v)] = (c, e, grids(per_block, units))
    times = {}
    for key, (_, _, gl) in engines.items():
        for mb in gl:
            times[(key, mb)] = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        order = list(times)
        np.random.default_rng(r).shuffle(order)
        for (key, mb) in order:
            _, e, _ = engines[key]
            e.set_option("max_blocks", mb)
            e.run(PHASE_ALL, 0)
            ev0.record(stream)
            for _ in range(a.reps):
                e.run(PHASE_ALL, 0)
            ev1.record(stream)
            ev1.synchronize()
            times[(key, mb)].append(ev0.elapsed_time(ev1) / a.reps)
    rows = []
    for ((fam, v), mb), ts in times.items():
        _, e, _ = engines[(fam, v)]
        ms = float(np.median(ts))
        rows.append(dict(family=fam, variant=v, max_blocks=mb, ms=round(ms, 4),
                         GBps=round(e.algorithmic_bytes(PHASE_ALL) / (ms * 1e-3) / 1e9, 1)))
    rows.sort(key=lambda r: (r["family"], r["variant"], -r["GBps"]))
    for r in rows:
        print(json.dumps(r))
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
