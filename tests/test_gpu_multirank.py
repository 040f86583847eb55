"""Row (e) on the GPU: sharded coupling steps with the exchange -> atmosphere accumulation
kernel, the shared boundary slots and fcx_atmos_finish.

* in one process: P engines on disjoint APPLE shards of one grid, their boundary buffers
  summed on the device (what the all-reduce does), then finish;
* in two processes on the one GPU of the box: the same through torch.distributed (gloo,
  since RCCL refuses two ranks on one device; the 8-GPU RCCL run is bench.py's).
Checked against the CPU oracle's single-process accumulation (tests/parity.py tolerance).
"""
import os
import socket

import numpy as np
import pytest

import oracle_lib
from parity import assert_parity

pytestmark = pytest.mark.gpu

from fcx.basic import PHASE_ALL  # noqa: E402
from fcx.parallel import local_atmos, synthetic_atmos_map  # noqa: E402
from fcx.synthetic import build_case  # noqa: E402

FIELDS = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))


def reference(n, variant, seed=911):
    case = build_case(variant, n=n, T=1, bias=True, seed=seed)
    out = oracle_lib.run_case(case, "c", current_step_time=7200)
    amap = synthetic_atmos_map(n)
    ref = {name: oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, out[(1, g, name)], amap.n_atmos)
           for name, g in FIELDS}
    return case, amap, ref


def shard_case(full, lo, hi, variant, seed=911):
    case = build_case(variant, n=hi - lo, T=1, bias=True, seed=seed)
    remap = {}
    for key, a in full.lf.field.items():
        if id(a) not in remap:
            remap[id(a)] = np.ascontiguousarray(np.asarray(a)[lo:hi])
        case.lf.field[key] = remap[id(a)]
    init_date, corr = full.corrections
    case.corrections = (init_date, np.ascontiguousarray(corr[lo:hi]))
    return case


def make_engine(case, la, shared, stride, device="cuda:0", fused=True, options=None, fields=None):
    """fields: [(phase, name, grid)] in registration order (default: FIELDS, normal phase)"""
    import torch
    from fcx.engine import Engine

    fields = fields or [(2, name, g) for name, g in FIELDS]
    outs = {name: torch.full((max(la.n_atmos, 1),), float("nan"), dtype=torch.float64, device=device)
            for _, name, _ in fields}
    atmos = {"local": la, "fields": [(ph, 1, g, name, outs[name]) for ph, name, g in fields],
             "shared": (shared, stride) if shared is not None else None}
    # specialize=0 turns the T=1 kernels (and with them the fused accumulation) off
    opts = dict(options or {})
    if not fused:
        opts["specialize"] = 0
    eng = Engine(case.lf, 1, case.methods, corrections=case.corrections, atmos=atmos, options=opts or None)
    return eng, outs


def random_run_map(n, lengths, seed):
    """An atmosphere map with the given run-length range (exchange cells per atmosphere
    cell), ordered by atmosphere cell, normalised weights."""
    from fcx.parallel import AtmosMap

    rng = np.random.default_rng(seed)
    runs = rng.integers(lengths[0], lengths[1] + 1, n)
    while runs.sum() < n:  # (ranges with empty runs can fall short of n cells)
        runs = np.concatenate([runs, rng.integers(lengths[0], lengths[1] + 1, n)])
    ends = np.cumsum(runs)
    n_atmos = int(np.searchsorted(ends, n, side="left")) + 1
    idx = np.repeat(np.arange(n_atmos, dtype=np.int32), runs[:n_atmos])[:n]
    area = rng.uniform(0.5, 1.5, n)
    w = area / np.bincount(idx, weights=area, minlength=n_atmos)[idx]
    return AtmosMap(np.ascontiguousarray(idx, dtype=np.int32), np.ascontiguousarray(w), n_atmos)


# run lengths: 1..5, 1..7, 1..9 (halo tiles: 1, 3 and 4 halo lanes), 1..10 (one cell too long
# for the halo: crossing records + fix-up), 20..64 (the fix-up; heads longer than the records'
# kRecHead kept products are recomputed); 130..140 and 1..400 (longer than half a tile: the
# engine runs atmos_kernel instead); 0..5 and 0..10: atmosphere cells without exchange cells
# (land on an intersection grid) among them, whose sums are 0
@pytest.mark.parametrize("lengths", [(1, 5), (1, 7), (1, 9), (1, 10), (20, 64), (130, 140), (1, 400), (0, 5),
                                     (0, 10)])
@pytest.mark.parametrize("mode", ["default", "nohalo", "capped", "pipelined", "pipelined_runtime"])
def test_fused_accumulation_long_segments(lengths, mode):
    """The accumulation with segments crossing 128-cell wave tiles: completed inside the launch
    by halo tiles (default, short segments, and under a grid-stride cap), by crossing records
    and the fix-up kernel (FCX_OPT_ATMOS_HALO 0, or segments too long for the halo), and across
    the chunk launches of the pipelined host step (through the staging arena, and with one
    runtime copy per array); long segments through atmos_kernel.  Bit-identical to the
    sequential sum of the GPU's own fluxes."""
    import torch
    from fcx.engine import Engine
    from fcx.parallel import local_atmos

    n = 300_001 if mode.endswith("pipelined") else 70_001
    case = build_case("CCLM", n=n, T=1, bias=True, seed=17)
    amap = random_run_map(n, lengths, seed=lengths[1])
    la = local_atmos(amap, 0, 1)
    outs = {name: torch.full((la.n_atmos,), float("nan"), dtype=torch.float64, device="cuda:0")
            for name, _ in FIELDS}
    atmos = {"local": la, "fields": [(2, 1, g, name, outs[name]) for name, g in FIELDS]}
    pipe = {"pipeline_chunks": 4, "pipeline_min_chunk": 65536, "zero_copy": 0}
    opts = {"default": {}, "nohalo": {"atmos_halo": 0}, "capped": {"max_blocks": 64}, "pipelined": pipe,
            "pipelined_runtime": {**pipe, "host_staging": 0}}[mode]
    eng = Engine(case.lf, 1, case.methods, corrections=case.corrections, atmos=atmos, options=opts)
    for step in range(3):  # later runs reuse the crossing records
        for o in outs.values():
            o.fill_(float("nan"))
        eng.step(PHASE_ALL, 3600 * step)
        torch.cuda.synchronize()
        for name, g in FIELDS:
            gpu_flux = np.asarray(case.lf.field[(1, g, name)])
            want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, gpu_flux, amap.n_atmos)
            np.testing.assert_array_equal(outs[name].cpu().numpy(), want, err_msg=f"{name} step {step}")
    eng.close()


@pytest.mark.parametrize("lengths", [(1, 5), (1, 9), (1, 10), (20, 64), (0, 5)])
@pytest.mark.parametrize("mode", ["default", "nohalo", "pipelined"])
def test_fused_accumulation_of_averages_long_segments(lengths, mode):
    """Two surface types: the type-0 averages accumulated by the multi-type fused kernel on
    maps whose segments cross its 128-cell wave tiles (1..5 and 1..9 cells: halo tiles where
    the kernel takes them, 1..10 and 20..64: crossing records + fix-up), with the crossing
    records forced (FCX_OPT_ATMOS_HALO 0), and across the pipelined step's chunk launches.
    Bit-identical to the sequential sum of the GPU's own averages."""
    import torch
    from fcx.engine import Engine
    from fcx.parallel import local_atmos

    n = 300_001 if mode == "pipelined" else 70_001
    case = build_case("CCLM", n=n, T=2, bias=True, seed=23)
    amap = random_run_map(n, lengths, seed=lengths[1] + 11)
    la = local_atmos(amap, 0, 1)
    outs = {name: torch.full((la.n_atmos,), float("nan"), dtype=torch.float64, device="cuda:0")
            for name, _ in FIELDS}
    atmos = {"local": la, "fields": [(2, 0, g, name, outs[name]) for name, g in FIELDS]}
    opts = {"default": {}, "nohalo": {"atmos_halo": 0},
            "pipelined": {"pipeline_chunks": 4, "pipeline_min_chunk": 65536, "zero_copy": 0}}[mode]
    eng = Engine(case.lf, 2, case.methods, corrections=case.corrections, averages=case.averages, atmos=atmos,
                 options=opts)
    for step in range(2):
        for o in outs.values():
            o.fill_(float("nan"))
        eng.step(PHASE_ALL, 3600 * step)
        torch.cuda.synchronize()
        for name, g in FIELDS:
            avg = np.asarray(case.lf.field[(0, g, name)])
            want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, avg, amap.n_atmos)
            np.testing.assert_array_equal(outs[name].cpu().numpy(), want, err_msg=f"{name} step {step}")
    eng.close()


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
def test_atmos_accumulation_bit_exact_single_rank(variant, fused):
    """One rank owns every cell: fused (tile sums + carried prefixes) and separate (LDS
    kernel) accumulation both reproduce the sequential SCRIP sum bit for bit."""
    n = 70_001  # > 100 tiles of 512 cells, segments straddling tile boundaries
    full, amap, ref = reference(n, variant)
    la = local_atmos(amap, 0, 1)
    eng, outs = make_engine(full, la, None, len(FIELDS), fused=fused)
    eng.step(PHASE_ALL, 7200)  # upload, run, download: full.lf now holds the GPU fluxes
    for name, g in FIELDS:
        # the accumulation is checked on the GPU's own fluxes (they differ from the
        # oracle's by ulps of exp/pow), against the sequential sum
        gpu_flux = np.asarray(full.lf.field[(1, g, name)])
        want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, gpu_flux, amap.n_atmos)
        np.testing.assert_array_equal(outs[name].cpu().numpy(), want, err_msg=name)
    assert_parity({k: outs[k].cpu().numpy() for k, _ in FIELDS}, ref, label=variant)
    eng.close()


def test_atmos_unsorted_map_uses_csr():
    """A map whose exchange cells are not ordered by atmosphere cell (CSR with columns)."""
    n = 9_001
    full, amap, _ = reference(n, "CCLM")
    perm = np.random.default_rng(5).permutation(amap.n_atmos).astype(np.int32)
    idx = perm[amap.atmos_index]
    from fcx.parallel import LocalAtmos

    la = LocalAtmos(0, n, 0, amap.n_atmos, idx, amap.weight, -1, -1, 0)
    eng, outs = make_engine(full, la, None, len(FIELDS))
    eng.step(PHASE_ALL, 7200)
    for name, g in FIELDS:
        ref = oracle_lib.atmos_accumulate(idx, amap.weight, np.asarray(full.lf.field[(1, g, name)]), amap.n_atmos)
        np.testing.assert_array_equal(outs[name].cpu().numpy(), ref, err_msg=name)
    eng.close()


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("variant,world", [("CCLM", 2), ("MOM5", 4), ("RCO", 8)])
def test_sharded_engines_one_process(variant, world, fused):
    import torch

    n = 20_011
    full, amap, ref = reference(n, variant)
    stride = len(FIELDS)
    engines = []
    for r in range(world):
        la = local_atmos(amap, r, world)
        shared = torch.zeros(max(world - 1, 1) * stride, dtype=torch.float64, device="cuda:0")
        case = shard_case(full, la.offset, la.offset + la.size, variant)
        eng, outs = make_engine(case, la, shared, stride, fused=fused)
        engines.append((la, shared, eng, outs))
    for la, shared, eng, outs in engines:
        eng.upload(PHASE_ALL)  # the shard's fields are host arrays
        eng.run(PHASE_ALL, 7200)
        eng.synchronize()
    total = sum(sh for _, sh, _, _ in engines)  # the all-reduce (sum) of the boundary slots
    for la, shared, eng, outs in engines:
        shared.copy_(total)
        eng.atmos_finish()
        eng.synchronize()
        assert float(shared.abs().sum()) == 0.0  # re-zeroed for the next step
    got = {name: np.full(amap.n_atmos, np.nan) for name, _ in FIELDS}
    for la, shared, eng, outs in engines:
        for name, _ in FIELDS:
            got[name][la.atmos_offset: la.atmos_offset + la.n_atmos] = outs[name].cpu().numpy()[: la.n_atmos]
        eng.close()
    assert_parity(got, ref, label=f"{variant} x{world}")


@pytest.mark.parametrize("fused", [True, False])
def test_sharded_engines_with_empty_atmosphere_cells(fused):
    """A map with atmosphere cells that no exchange cell maps to (runs of 0..5 cells), over 3
    shards: inside a shard they get the zero sum, the shared boundary cells still close
    through the slots; fused and unfused paths."""
    import torch

    n, world, variant = 30_011, 3, "MOM5"
    full = build_case(variant, n=n, T=1, bias=True, seed=911)
    out = oracle_lib.run_case(full, "c", current_step_time=7200)
    amap = random_run_map(n, (0, 5), seed=23)
    ref = {name: oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, out[(1, g, name)], amap.n_atmos)
           for name, g in FIELDS}
    stride = len(FIELDS)
    engines = []
    for r in range(world):
        la = local_atmos(amap, r, world)
        shared = torch.zeros(max(world - 1, 1) * stride, dtype=torch.float64, device="cuda:0")
        case = shard_case(full, la.offset, la.offset + la.size, variant)
        eng, outs = make_engine(case, la, shared, stride, fused=fused)
        engines.append((la, shared, eng, outs))
    for la, shared, eng, outs in engines:
        eng.upload(PHASE_ALL)
        eng.run(PHASE_ALL, 7200)
        eng.synchronize()
    total = sum(sh for _, sh, _, _ in engines)
    for la, shared, eng, outs in engines:
        shared.copy_(total)
        eng.atmos_finish()
        eng.synchronize()
    got = {name: np.full(amap.n_atmos, np.nan) for name, _ in FIELDS}
    covered = np.zeros(amap.n_atmos, bool)
    for la, shared, eng, outs in engines:
        covered[la.atmos_offset: la.atmos_offset + la.n_atmos] = True
        for name, _ in FIELDS:
            got[name][la.atmos_offset: la.atmos_offset + la.n_atmos] = outs[name].cpu().numpy()[: la.n_atmos]
        eng.close()
    # cells between two ranks' ranges have no exchange cell on any rank: no rank holds them
    # (the host assembles the field from the ranks' ranges; their sum over no links is 0)
    assert not np.bincount(amap.atmos_index, minlength=amap.n_atmos)[~covered].any()
    for name, _ in FIELDS:
        got[name][~covered] = 0.0
    assert_parity(got, ref, label=f"{variant} x{world} with empty atmosphere cells")


@pytest.mark.parametrize("fused", [True, False])
def test_sharded_engines_field_order_and_phases(fused):
    """Fields registered out of the fused kernel's slot order, RBBR accumulated at the end of
    the early phase and the rest at the end of the normal one: every path writes a field's
    boundary partial sums into the column of its registration index, so the all-reduce and
    fcx_atmos_finish complete the right cells."""
    import torch

    n, world, variant = 20_011, 3, "MOM5"
    full, amap, ref = reference(n, variant)
    fields = [(2, "VMOM", 3), (1, "RBBR", 1), (2, "HSEN", 1), (2, "MEVA", 1), (2, "UMOM", 2), (2, "HLAT", 1)]
    stride = len(fields)
    engines = []
    for r in range(world):
        la = local_atmos(amap, r, world)
        shared = torch.zeros((world - 1) * stride, dtype=torch.float64, device="cuda:0")
        case = shard_case(full, la.offset, la.offset + la.size, variant)
        eng, outs = make_engine(case, la, shared, stride, fused=fused, fields=fields)
        engines.append((la, shared, eng, outs))
    for la, shared, eng, outs in engines:
        eng.upload(PHASE_ALL)
        eng.run(1, 7200)  # early phase: RBBR and its accumulation
        eng.run(2, 7200)  # normal phase: the rest
        eng.synchronize()
    total = sum(sh for _, sh, _, _ in engines)
    for la, shared, eng, outs in engines:
        shared.copy_(total)
        eng.atmos_finish()
        eng.synchronize()
    got = {name: np.full(amap.n_atmos, np.nan) for name, _ in FIELDS}
    for la, shared, eng, outs in engines:
        for name, _ in FIELDS:
            got[name][la.atmos_offset: la.atmos_offset + la.n_atmos] = outs[name].cpu().numpy()[: la.n_atmos]
        eng.close()
    assert_parity(got, ref, label=f"field order, phases, fused={fused}")


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        n = 12_007
        full, amap, _ = reference(n, "CCLM")
        la = local_atmos(amap, rank, world)
        stride = len(FIELDS)
        shared = torch.zeros((world - 1) * stride, dtype=torch.float64, device="cuda:0")
        case = shard_case(full, la.offset, la.offset + la.size, "CCLM")
        eng, outs = make_engine(case, la, shared, stride)
        eng.upload(PHASE_ALL)
        eng.run(PHASE_ALL, 7200)
        eng.synchronize()
        dist.all_reduce(shared)  # ONE collective per step
        eng.atmos_finish()
        eng.synchronize()
        q.put((rank, la.atmos_offset, {k: v.cpu().numpy()[: la.n_atmos].tolist() for k, v in outs.items()}))
        eng.close()
    finally:
        dist.destroy_process_group()


def test_two_processes_share_one_gpu_gloo():
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get() for _ in range(2)]
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    _, amap, ref = reference(12_007, "CCLM")
    got = {name: np.full(amap.n_atmos, np.nan) for name, _ in FIELDS}
    for rank, a0, outs in sorted(res):
        for name, vals in outs.items():
            got[name][a0: a0 + len(vals)] = vals
    assert_parity(got, ref, label="2 processes")


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("variant,T", [("CCLM", 2), ("MOM5", 3), ("RCO", 2)])
def test_atmos_accumulation_of_type0_averages(variant, T, fused):
    """Several surface types: OASIS sends the type-0 averages (S A xxxx 00).  The averages
    are accumulated in LDS as the types are produced (register slots) and, fused, handed to
    the accumulation without being re-read; both paths give the sequential SCRIP sum of the
    GPU's own averages bit for bit, and the averages match the oracle."""
    import torch
    from fcx.engine import Engine

    n = 40_003
    case = build_case(variant, n=n, T=T, bias=True, seed=913)
    ref = oracle_lib.run_case(case, "c", current_step_time=7200)
    amap = synthetic_atmos_map(n)
    la = local_atmos(amap, 0, 1)
    outs = {name: torch.full((la.n_atmos,), float("nan"), dtype=torch.float64, device="cuda:0")
            for name, _ in FIELDS}
    atmos = {"local": la, "fields": [(2, 0, g, name, outs[name]) for name, g in FIELDS]}
    eng = Engine(case.lf, T, case.methods, corrections=case.corrections, averages=case.averages, atmos=atmos,
                 options=None if fused else {"specialize": 0})
    eng.step(PHASE_ALL, 7200)
    for name, g in FIELDS:
        avg = np.asarray(case.lf.field[(0, g, name)])
        want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, avg, amap.n_atmos)
        np.testing.assert_array_equal(outs[name].cpu().numpy(), want, err_msg=name)
    assert_parity({k: np.asarray(case.lf.field[k]) for k in case.outputs},
                  {k: ref[k] for k in case.outputs}, label=f"{variant} T{T}")
    eng.close()


@pytest.mark.parametrize("fused", [True, False])
def test_sharded_engines_empty_middle_rank(fused):
    """Three shards from a task vector whose middle rank owns no cells (io:101-104), the cut
    between ranks 0 and 2 inside an atmosphere cell: the empty rank's engine steps and takes
    part in the slot sum, and the shared cell is completed through one slot
    (fcx.parallel.task_ranges)."""
    import torch
    from fcx.parallel import task_ranges

    n, world = 20_011, 3
    full, amap, ref = reference(n, "MOM5")
    k = next(i for i in range(n // 2, n) if amap.atmos_index[i - 1] == amap.atmos_index[i])
    task = np.full(n, 2, np.int32)
    task[:k] = 0
    stride = len(FIELDS)
    engines = []
    for r, (off, size, right_slot) in enumerate(task_ranges(task, world)):
        la = local_atmos(amap, r, world, off, size, right_slot=right_slot)
        shared = torch.zeros((world - 1) * stride, dtype=torch.float64, device="cuda:0")
        case = shard_case(full, off, off + size, "MOM5")
        eng, outs = make_engine(case, la, shared, stride, fused=fused)
        engines.append((la, shared, eng, outs))
    assert engines[0][0].right == engines[2][0].left == 1 and engines[1][0].size == 0
    for la, shared, eng, outs in engines:
        eng.upload(PHASE_ALL)
        eng.run(PHASE_ALL, 7200)
        eng.synchronize()
    total = sum(sh for _, sh, _, _ in engines)
    for la, shared, eng, outs in engines:
        shared.copy_(total)
        eng.atmos_finish()
        eng.synchronize()
    got = {name: np.full(amap.n_atmos, np.nan) for name, _ in FIELDS}
    for la, shared, eng, outs in engines:
        for name, _ in FIELDS:
            got[name][la.atmos_offset: la.atmos_offset + la.n_atmos] = outs[name].cpu().numpy()[: la.n_atmos]
        eng.close()
    assert_parity(got, ref, label="empty middle rank")
