#!/usr/bin/env python3
"""Host-link probe at the Baltic size (BASELINE config 2: 32,768 exchange cells): what the
link between the host and one MI355X allows for one coupling step of the three variants
from host arrays.

Bytes of one step from the caller's heap arrays (T = 1, u/v = t grid, fp64):
  H2D  CCLM 10 arrays + MOM5 11 + RCO 5  = 208 B/cell
  D2H  CCLM 7 + MOM5 7 + RCO 6           = 160 B/cell

  dma      page-locked host <-> device copies of those bytes: H2D alone, D2H alone, both at
           once on two streams (full duplex), as one copy per direction and as one copy per
           array; the median over many repetitions
  host     the host copies of the staging arena (heap array -> page-locked image and back)
           with 1 and N threads
  engine   fcx_upload / fcx_run / fcx_download / fcx_step of each variant's engine, and the
           three variants' steps back to back, median wall time

  python components.flux_calculator_amd/bench/link_probe.py [--cells 32768] [--reps 400]
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))

VARIANTS = ("CCLM", "MOM5", "RCO")
ARRAYS_IN = {"CCLM": 10, "MOM5": 11, "RCO": 5}
ARRAYS_OUT = {"CCLM": 7, "MOM5": 7, "RCO": 6}


def med_us(f, reps, warm=20):
    for _ in range(warm):
        f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e6, 1)


def link_rates(b_in, b_out, reps=200):
    """Page-locked host <-> device DMA of b_in bytes up and b_out bytes down, one copy per
    direction: each alone, and both at once on two streams; plus 256 MiB copies (the link's
    asymptotic rate).  Median microseconds and GB/s.  The copies are libfcx's: hipMemcpyAsync
    with hipMemcpyDefault between hipHostMalloc memory and device memory (an explicit
    device-to-host kind takes a slow path in this ROCm, profiles/r05/dma2/)."""
    import ctypes

    import torch

    # the process's one HIP runtime: torch's own copy (the file torch loaded), else the system's
    own = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    hip = ctypes.CDLL(own if os.path.exists(own) else "libamdhip64.so")
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip_default = 4  # hipMemcpyDefault

    def host_alloc(n):
        p = ctypes.c_void_p()
        if hip.hipHostMalloc(ctypes.byref(p), n, 0) != 0:
            raise RuntimeError("hipHostMalloc failed")
        return p

    def dev_alloc(n):  # plain hipMalloc, as libfcx's pools (not torch's caching allocator)
        p = ctypes.c_void_p()
        if hip.hipMalloc(ctypes.byref(p), n) != 0:
            raise RuntimeError("hipMalloc failed")
        return p

    dev = torch.device("cuda", 0)
    # two non-blocking streams of the runtime's own, as libfcx's engines create them (torch's
    # pooled streams may share a hardware queue, which serialises the two directions)
    s1, s2 = ctypes.c_void_p(), ctypes.c_void_p()
    for st in (s1, s2):
        if hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) != 0:
            raise RuntimeError("hipStreamCreateWithFlags failed")
    out = {}
    for name, bi, bo, r in (("step", b_in, b_out, reps), ("256MiB", 256 << 20, 256 << 20, 10)):
        hi, ho = host_alloc(bi), host_alloc(bo)
        di, do = dev_alloc(bi), dev_alloc(bo)

        def up():
            if hip.hipMemcpyAsync(di, hi, bi, hip_default, s1) != 0:
                raise RuntimeError("hipMemcpyAsync H2D failed")

        def down():
            if hip.hipMemcpyAsync(ho, do, bo, hip_default, s2) != 0:
                raise RuntimeError("hipMemcpyAsync D2H failed")

        def run(fs):
            def f():
                for g in fs:
                    g()
                hip.hipStreamSynchronize(s1)
                hip.hipStreamSynchronize(s2)
            return f
        torch.cuda.synchronize()
        t_in = med_us(run([up]), r, warm=3)
        t_out = med_us(run([down]), r, warm=3)
        t_both = med_us(run([up, down]), r, warm=3)
        out[name] = {"h2d_bytes": bi, "d2h_bytes": bo, "h2d_us": t_in, "d2h_us": t_out, "both_us": t_both,
                     "h2d_GBps": round(bi / t_in / 1e3, 1), "d2h_GBps": round(bo / t_out / 1e3, 1),
                     "both_GBps": round((bi + bo) / t_both / 1e3, 1)}
        torch.cuda.synchronize()
        hip.hipHostFree(hi)
        hip.hipHostFree(ho)
        hip.hipFree(di)
        hip.hipFree(do)
    hip.hipStreamDestroy(s1)
    hip.hipStreamDestroy(s2)
    out["copies"] = "hipMemcpyAsync(hipMemcpyDefault), hipHostMalloc memory <-> hipMalloc memory, two non-blocking streams"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=32_768)
    ap.add_argument("--reps", type=int, default=400)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    a = ap.parse_args()

    import torch

    n = a.cells
    n_in, n_out = sum(ARRAYS_IN.values()), sum(ARRAYS_OUT.values())
    b_in, b_out = n_in * 8 * n, n_out * 8 * n
    out = {"cells": n, "h2d_bytes": b_in, "d2h_bytes": b_out, "reps": a.reps}
    dev = torch.device("cuda", 0)
    h_in = torch.empty(b_in, dtype=torch.uint8).pin_memory()
    h_out = torch.empty(b_out, dtype=torch.uint8).pin_memory()
    d_in = torch.empty(b_in, dtype=torch.uint8, device=dev)
    d_out = torch.empty(b_out, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    per = 8 * n

    def h2d(split=False, s=s1):
        with torch.cuda.stream(s):
            if split:
                for k in range(n_in):
                    d_in[k * per:(k + 1) * per].copy_(h_in[k * per:(k + 1) * per], non_blocking=True)
            else:
                d_in.copy_(h_in, non_blocking=True)

    def d2h(split=False, s=s2):
        with torch.cuda.stream(s):
            if split:
                for k in range(n_out):
                    h_out[k * per:(k + 1) * per].copy_(d_out[k * per:(k + 1) * per], non_blocking=True)
            else:
                h_out.copy_(d_out, non_blocking=True)

    def run(fs):
        def f():
            for g in fs:
                g()
            s1.synchronize()
            s2.synchronize()
        return f

    dma = {}
    for split in (False, True):
        key = "per_array" if split else "one_copy"
        t_in = med_us(run([lambda: h2d(split)]), a.reps)
        t_out = med_us(run([lambda: d2h(split)]), a.reps)
        t_both = med_us(run([lambda: h2d(split), lambda: d2h(split)]), a.reps)
        t_seq = med_us(run([lambda: h2d(split, s1), lambda: d2h(split, s1)]), a.reps)
        dma[key] = {"h2d_us": t_in, "d2h_us": t_out, "both_two_streams_us": t_both, "both_one_stream_us": t_seq,
                    "h2d_GBps": round(b_in / t_in / 1e3, 1), "d2h_GBps": round(b_out / t_out / 1e3, 1),
                    "duplex_GBps": round((b_in + b_out) / t_both / 1e3, 1)}
    # large copies: the link's asymptotic rate
    big = 256 << 20
    hb = torch.empty(big, dtype=torch.uint8).pin_memory()
    db = torch.empty(big, dtype=torch.uint8, device=dev)
    hb2 = torch.empty(big, dtype=torch.uint8).pin_memory()
    db2 = torch.empty(big, dtype=torch.uint8, device=dev)

    def big_h2d():
        with torch.cuda.stream(s1):
            db.copy_(hb, non_blocking=True)

    def big_d2h():
        with torch.cuda.stream(s2):
            hb2.copy_(db2, non_blocking=True)
    t_bi = med_us(run([big_h2d]), 20, warm=3)
    t_bo = med_us(run([big_d2h]), 20, warm=3)
    t_bb = med_us(run([big_h2d, big_d2h]), 20, warm=3)
    dma["256MiB"] = {"h2d_GBps": round(big / t_bi / 1e3, 1), "d2h_GBps": round(big / t_bo / 1e3, 1),
                     "duplex_GBps": round(2 * big / t_bb / 1e3, 1)}
    del hb, db, hb2, db2
    out["dma"] = dma

    # host copies of the staging arena: heap (numpy) -> page-locked image and back
    heap_in = [np.random.default_rng(k).random(n) for k in range(n_in)]
    heap_out = [np.empty(n) for _ in range(n_out)]
    img_in = h_in.numpy().view(np.float64)
    img_out = h_out.numpy().view(np.float64)

    def gather(ks):
        for k in ks:
            np.copyto(img_in[k * n:(k + 1) * n], heap_in[k])

    def scatter(ks):
        for k in ks:
            np.copyto(heap_out[k], img_out[k * n:(k + 1) * n])
    host = {"gather_1thread_us": med_us(lambda: gather(range(n_in)), a.reps),
            "scatter_1thread_us": med_us(lambda: scatter(range(n_out)), a.reps)}
    with ThreadPoolExecutor(a.threads) as ex:
        def par(fn, m):
            list(ex.map(fn, [range(k, m, a.threads) for k in range(a.threads)]))
        host[f"gather_{a.threads}threads_us"] = med_us(lambda: par(gather, n_in), a.reps)
        host[f"scatter_{a.threads}threads_us"] = med_us(lambda: par(scatter, n_out), a.reps)
    out["host_copies"] = host

    # the engine: each call of one variant's step on its own, and fcx_step
    from fcx.basic import PHASE_ALL
    from fcx.engine import Engine
    from fcx.synthetic import build_case, inputs_for_bench

    data = inputs_for_bench(n)
    eng = {}
    for v in VARIANTS:
        c = build_case(v, n=n, T=1, bias=True, data=data)
        e = Engine(c.lf, 1, c.methods, corrections=c.corrections)
        for k in range(50):
            e.step(PHASE_ALL, k * 3600)

        def up():
            e.upload(PHASE_ALL)
            e.synchronize()

        def rn():
            e.run(PHASE_ALL, 3600)
            e.synchronize()

        def dn():
            e.download(PHASE_ALL)
            e.synchronize()
        eng[v] = {"upload_us": med_us(up, a.reps), "run_us": med_us(rn, a.reps), "download_us": med_us(dn, a.reps),
                  "step_us": med_us(lambda: e.step(PHASE_ALL, 3600), a.reps)}
        e.close()
    out["engine"] = eng
    out["engine_steps_sum_us"] = round(sum(x["step_us"] for x in eng.values()), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
