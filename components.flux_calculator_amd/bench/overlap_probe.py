#!/usr/bin/env python3
"""The step with its boundary exchange, sequential against overlapped, on ONE GPU
(measurement tool): rank 0's half of a 2-rank decomposition (10M cells per rank, a right
boundary slot per variant) with a one-rank RCCL communicator, so the all-reduce is real RCCL
but completes locally.  Blocks of steps alternate between

  seq      fcx_run_group, then fcx_atmos_allreduce (the collective after the launch)
  overlap  fcx_run_group_exchange (boundary tiles + the all-reduce on the communicator's
           stream beside the main launch)

and each block is timed on the host around synchronisations (wall time per step).  A
one-rank all-reduce is cheaper than an 8-rank one over xGMI, so this shows what the split
costs and a lower bound of what it hides.

  python overlap_probe.py [--cells 10000000] [--rounds 8] [--steps 50]
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
    ap.add_argument("--cells", type=int, default=10_000_000)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()

    import torch
    from fcx.comm import Comm, unique_id
    from fcx.workload import Workload

    torch.cuda.set_device(0)
    comm = Comm(0, 1, 0, unique_id())
    wl = Workload(2 * a.cells, 0, 2, atmos_map="random", stream=torch.cuda.current_stream())
    assert wl.la.right >= 0, "rank 0 of 2 must share its last atmosphere cell"

    def seq(t):
        wl.run_group(t)
        comm.atmos_allreduce(wl.engines)

    def ovl(t):
        comm.run_group_exchange(wl.engines, t)

    modes = {"seq": seq, "overlap": ovl}
    for f in modes.values():  # plans, communicator, clocks
        for k in range(100):
            f(k * 3600)
    torch.cuda.synchronize()
    res = {m: [] for m in modes}
    for r in range(a.rounds):
        for m, f in modes.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.steps):
                f(k * 3600)
            torch.cuda.synchronize()
            res[m].append((time.perf_counter() - t0) / a.steps * 1e3)
    out = {"cells_per_rank": a.cells, "rounds": a.rounds, "steps_per_block": a.steps,
           "overlapped_exchanges": comm.overlapped(),
           "ms_per_step": {m: round(float(np.mean(v)), 4) for m, v in res.items()},
           "ms_per_step_blocks": {m: [round(x, 4) for x in v] for m, v in res.items()}}
    out["overlap_saves_us"] = round((out["ms_per_step"]["seq"] - out["ms_per_step"]["overlap"]) * 1e3, 1)
    print(json.dumps(out), flush=True)
    wl.close()
    comm.close()


if __name__ == "__main__":
    main()
