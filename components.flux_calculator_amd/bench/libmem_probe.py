#!/usr/bin/env python3
"""The Baltic-size step (32,768 cells, CCLM + MOM5 + RCO) from fcx_host_malloc arrays, both
transports (the span transport and zero-copy), next to the host link's floors -- bench.py's
own baltic_size legs without the rest of the bench (measurement tool).

  python libmem_probe.py [--steps 500]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "bench"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--types", type=int, default=1)
    a = ap.parse_args()
    import bench
    from link_probe import link_rates

    args = argparse.Namespace(types=a.types, bias=False)
    variants = bench.VARIANTS
    out = {"library_memory": bench.e2e_library_memory(args, variants, steps=a.steps)}
    out["async_heap_arrays"] = bench.e2e_async(args, variants, steps=a.steps)
    lk = link_rates(*bench.link_bytes(variants, 32_768, args))
    st = lk["step"]
    out["host_link"] = dict(lk, bound_duplex_us=round(max(st["h2d_bytes"] / st["h2d_GBps"],
                                                          st["d2h_bytes"] / st["d2h_GBps"]) / 1e3, 1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
