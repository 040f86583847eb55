#!/usr/bin/env python3
"""The Baltic-size step (32,768 cells, CCLM + MOM5 + RCO) from fcx_host_malloc arrays with the
zero-copy transport only, one build per process (FCX_LIBRARY) -- for A/Bs of the library
memory's allocation flags, run alternately by a driver script (measurement tool).

  FCX_LIBRARY=ab/x/libfcx.so python libmem_ab.py [--steps 500]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--cells", type=int, default=32_768)
    a = ap.parse_args()
    import torch
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.host_alloc import Arena
    from fcx.synthetic import build_case, inputs_for_bench

    data = inputs_for_bench(a.cells)
    streams = [torch.cuda.Stream() for _ in range(3)]
    cases = [build_case(v, n=a.cells, T=1, bias=False, data=data) for v in ("CCLM", "MOM5", "RCO")]
    out = {"library": os.environ.get("FCX_LIBRARY", "default"), "cells": a.cells, "steps": a.steps}
    with Arena() as arena:
        for c in cases:
            arena.adopt(c.lf)
        engines = [Engine(c.lf, c.num_surface_types, c.methods, corrections=c.corrections, averages=c.averages,
                          stream=st.cuda_stream) for c, st in zip(cases, streams)]
        assert all(e.zero_copy_active() for e in engines)
        for mode in ("sequential", "async"):
            ts = []
            for k in range(50 + a.steps):
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
            out[f"{mode}_us_median"] = round(float(np.median(ts)) * 1e6, 1)
            out[f"{mode}_us_p90"] = round(float(np.percentile(ts, 90)) * 1e6, 1)
        for e in engines:
            e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
