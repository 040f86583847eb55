#!/usr/bin/env python3
"""Sweep the cells-kernel launch options (fcx_set_option) on the config-3 workload.

One process, interleaved rounds (cdna_hip_programming.md 5.4 rule 24): every option set is
timed once per round with HIP events on the engine stream; the median over rounds is
reported as GB/s of algorithmic bytes.  Usage: python tune_launch.py [--cells N] [--rounds R]
"""
import argparse
import itertools
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.synthetic import build_case, inputs_for_bench

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream(dev)
    data = {k: torch.as_tensor(v).to(dev) for k, v in inputs_for_bench(args.cells).items()}
    engines = {}
    for v in ("CCLM", "MOM5", "RCO"):
        c = build_case(v, n=args.cells, T=1, device=dev, data=data)
        engines[v] = (c, Engine(c.lf, 1, c.methods, device=0, stream=stream.cuda_stream))
    grid = list(itertools.product((1, 2), (0, 1), (1024, 2048, 4096, 8192, 0), (0, 1)))
    times = {(v, cfg): [] for v in engines for cfg in grid}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(args.rounds):
        order = list(times)
        np.random.default_rng(r).shuffle(order)
        for (v, cfg) in order:
            c, e = engines[v]
            cpt, nt, mb, spec = cfg
            e.set_option("cells_per_thread", cpt)
            e.set_option("nontemporal", nt)
            e.set_option("max_blocks", mb)
            e.set_option("specialize", spec)
            e.run(PHASE_ALL, 0)  # warm
            ev0.record(stream)
            for _ in range(args.reps):
                e.run(PHASE_ALL, 0)
            ev1.record(stream)
            ev1.synchronize()
            times[(v, cfg)].append(ev0.elapsed_time(ev1) / args.reps)
    rows = []
    for (v, cfg), ts in times.items():
        c, e = engines[v]
        ms = float(np.median(ts))
        gbs = e.algorithmic_bytes(PHASE_ALL) / (ms * 1e-3) / 1e9
        rows.append(dict(variant=v, cells_per_thread=cfg[0], nontemporal=cfg[1], max_blocks=cfg[2],
                         specialize=cfg[3], ms=round(ms, 4), GBps=round(gbs, 1),
                         min_ms=round(float(np.min(ts)), 4)))
    rows.sort(key=lambda r: (r["variant"], -r["GBps"]))
    for r in rows:
        print(json.dumps(r))
    if args.out:
        json.dump(rows, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
