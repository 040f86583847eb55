"""CPU legs of bench.py: the reference flux path timed on the GPU box's own host cores, at
BASELINE.json's config sizes, on the same inputs as the GPU workload (SURVEY.md 8d "CPU
timing beside it").

  one core   the reference flux_lib (oracle/_ref, kind "reference"; the C port oracle/fco.c,
             kind "port", where the reference was not built) in the reference call order
             (flux_calculator.F90:902-1008): one MPI rank of the reference
  all cores  P processes -- P = this box's CPU share (OMP_NUM_THREADS, 16 per GPU on the
             pool), else the process affinity set -- each running the same code on its APPLE
             range (decomp_def.F90:23-31): the reference's own MPI range decomposition.
             A step starts at a common barrier and ends when the last rank is done, as an
             MPI step ends at the next MPI_BARRIER (flux_calculator.F90:867)

Inputs: fcx.synthetic.inputs_for_bench(n), the arrays the GPU workload of the same size
uses (bench.py, fcx.workload), shared with the ranks through a memory-mapped scratch copy.
TEST INFRASTRUCTURE: the oracle is the measured CPU baseline here, never the product path.
"""
import multiprocessing as mp
import os
import shutil
import tempfile
import time

import numpy as np


def oracle_kind():
    import oracle_lib

    return "reference" if oracle_lib.load("ref") is not None else "port"


def _cases(n, variants, data):
    from fcx.synthetic import build_case

    return [build_case(v, n=n, T=1, data=data) for v in variants]


def _states(cases):
    import oracle_lib

    return [oracle_lib.OracleState(c, 0) for c in cases]


def _step(states, kind):
    import oracle_lib

    lib_kind = "ref" if kind == "reference" else "c"
    for st in states:
        oracle_lib.run_state(st, lib_kind)


def one_core(n, variants, kind, seconds, data=None):
    """Single process, single thread: steps until `seconds` have passed (at least 2)."""
    from fcx.synthetic import inputs_for_bench

    data = inputs_for_bench(n) if data is None else data
    states = _states(_cases(n, variants, data))
    _step(states, kind)  # first touch
    reps, t0 = 0, time.perf_counter()
    while True:
        _step(states, kind)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds and reps >= 2:
            break
    return {"value": round(n * len(variants) * reps / el / 1e6, 2), "unit": "Mcells/s", "cores": 1, "kind": kind,
            "us_per_step": round(el / reps * 1e6, 1),
            "sample": f"{reps} coupling steps x {len(variants)} variants over {n} cells, 1 thread, {el:.2f} s"}


def _rank(rank, nranks, n, variants, kind, folder, keys, reps, barrier, q):
    try:
        from fcx.parallel import apple_range

        off, size = apple_range(n, rank, nranks)
        data = {k: np.ascontiguousarray(np.load(os.path.join(folder, k + ".npy"), mmap_mode="r")[off: off + size])
                for k in keys}
        states = _states(_cases(size, variants, data))
        _step(states, kind)  # first touch
        dts = []
        for _ in range(reps):
            barrier.wait()
            t0 = time.perf_counter()
            _step(states, kind)
            dts.append(time.perf_counter() - t0)
        barrier.wait()
        q.put((rank, dts, None))
    except Exception as ex:  # noqa: BLE001 -- reported to the parent
        q.put((rank, None, repr(ex)))
        barrier.abort()


def all_cores(n, variants, kind, nranks, reps, data=None):
    """nranks processes over APPLE ranges, `reps` barrier-synchronised steps."""
    from fcx.synthetic import inputs_for_bench

    data = inputs_for_bench(n) if data is None else data
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    folder = tempfile.mkdtemp(prefix="fcx_cpu_legs_", dir=base)
    try:
        for k, a in data.items():
            np.save(os.path.join(folder, k + ".npy"), np.ascontiguousarray(a))
        ctx = mp.get_context("spawn")
        barrier, q = ctx.Barrier(nranks), ctx.SimpleQueue()
        procs = [ctx.Process(target=_rank, args=(r, nranks, n, variants, kind, folder, list(data), reps, barrier, q))
                 for r in range(nranks)]
        for p in procs:
            p.start()
        res = [q.get() for _ in range(nranks)]
        for p in procs:
            p.join(timeout=120)
    finally:
        shutil.rmtree(folder, ignore_errors=True)
    errs = [e for _, _, e in res if e]
    if errs:
        raise RuntimeError(f"CPU all-cores leg: {errs[0]}")
    per = np.array([dts for _, dts, _ in sorted(res, key=lambda x: x[0])])  # [rank][rep]
    step = per.max(axis=0)  # a step ends when the last rank is done
    el = float(step.sum())
    return {"value": round(n * len(variants) * reps / el / 1e6, 2), "unit": "Mcells/s", "cores": nranks, "kind": kind,
            "us_per_step": round(el / reps * 1e6, 1),
            "rank_imbalance": round(float(per.mean(axis=1).max() / per.mean()), 3),
            "sample": f"{reps} coupling steps x {len(variants)} variants over {n} cells, {nranks} processes on "
                      f"APPLE ranges (the reference's MPI decomposition), step = barrier to last rank, {el:.2f} s"}


def box_threads():
    """The CPU share of this GPU's box: OMP_NUM_THREADS where set (16 per GPU on the pool),
    else every CPU of the process affinity set."""
    affinity = len(os.sched_getaffinity(0))
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or affinity, affinity


def legs(variants, sizes=(32_768, 10_000_000), seconds=3.0):
    """{size: {"one_core": ..., "all_cores": ...}} on the same inputs per size."""
    from fcx.synthetic import inputs_for_bench

    kind = oracle_kind()
    threads, affinity = box_threads()
    out = {}
    for n in sizes:
        data = inputs_for_bench(n)
        one = one_core(n, variants, kind, seconds, data=data)
        # the all-cores leg runs about `seconds` too, from the 1-core rate (ideal scaling)
        est = one["us_per_step"] * 1e-6 / threads
        reps = int(min(2000, max(3, seconds / max(est, 1e-6))))
        out[str(n)] = {"one_core": one, "all_cores": all_cores(n, variants, kind, threads, reps, data=data)}
        del data
    return {"kind": kind, "threads": threads, "affinity_cpus": affinity, "machine_cpus": os.cpu_count(),
            "sizes": out}
