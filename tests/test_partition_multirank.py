"""Row (e) on the CPU: APPLE / task-vector partitions, the synthetic exchange -> atmosphere
map, and the sharded coupling step with ONE all-reduce of the shared boundary slots, run as
world_size-2 (and 3) process groups on gloo.  The per-rank compute is the CPU oracle; the
GPU path uses the same partition/boundary logic (tests/test_gpu_multirank.py)."""
import os
import socket

import numpy as np
import pytest

import oracle_lib
from fcx.parallel import (apple_range, boundary_slots, local_atmos, pack_boundaries, synthetic_atmos_map,
                          task_ranges, task_range, unpack_boundaries)
from fcx.synthetic import build_case
from parity import assert_parity, mixed_error

ATMOS_FIELDS = ("MEVA", "HLAT", "HSEN", "RBBR", "UMOM", "VMOM")


@pytest.mark.parametrize("n,p", [(10, 1), (10, 3), (40_000_000, 8), (7, 8), (1001, 4)])
def test_apple_ranges_cover_grid_once(n, p):
    cover = []
    for r in range(p):
        off, size = apple_range(n, r, p)
        assert size >= 0
        cover.append((off, off + size))
    assert cover[0][0] == 0 and cover[-1][1] == n
    assert all(cover[i][1] == cover[i + 1][0] for i in range(p - 1))
    assert all(apple_range(n, r, p)[1] == n // p for r in range(p - 1))  # decomp_def.F90:25-26


def test_task_vector_rule():
    task = np.array([0, 0, 1, 1, 1, 2])
    assert task_range(task, 0) == (0, 2)
    assert task_range(task, 1) == (2, 3)
    assert task_range(task, 2) == (5, 1)
    assert task_range(task, 3) == (0, 0)  # empty task (io:101-104)


def test_task_ranges_slot_rule():
    """Right slot = (next rank with cells) - 1; empty ranks anywhere (io:101-104)."""
    t = np.array([0, 0, 2, 2, 2, 4], np.int32)  # ranks 1 and 3 empty, 5 absent
    assert task_ranges(t, 6) == [(0, 2, 1), (0, 0, 1), (2, 3, 3), (0, 0, 3), (5, 1, 4), (0, 0, 5)]
    assert task_ranges(np.zeros(4, np.int32), 3) == [(0, 4, 0), (0, 0, 1), (0, 0, 2)]
    # with every rank owning cells the rule is the APPLE one: right slot = rank
    assert [r for _, _, r in task_ranges(np.repeat(np.arange(4), 3), 4)] == [0, 1, 2, 3]


@pytest.mark.parametrize("mapcls", ["PeriodicAtmosMap", "BlockedRandomAtmosMap"])
def test_structured_maps_take_the_task_slot_rule(mapcls):
    """The O(size) structured maps of the bench build the same local views as local_atmos on
    their global map, with the task_ranges slot rule when a middle rank is empty."""
    import fcx.parallel as par

    mk = getattr(par, mapcls)()
    n = 30_001
    g = mk.global_map(n)
    t = np.repeat(np.array([0, 2, 3], np.int32), [12_007, 9_001, n - 21_008])  # rank 1 empty
    for rank, (off, size, right_slot) in enumerate(task_ranges(t, 4)):
        a = mk.local(off, size, rank, 4, n, right_slot=right_slot)
        b = local_atmos(g, rank, 4, off, size, right_slot=right_slot)
        assert (a.left, a.right, a.n_atmos) == (b.left, b.right, b.n_atmos), rank
        np.testing.assert_array_equal(a.atmos_index, b.atmos_index)
        np.testing.assert_allclose(a.weight, b.weight, rtol=1e-14)
    # rank 0's right boundary and rank 2's left one are the same slot
    r0 = mk.local(0, 12_007, 0, 4, n, right_slot=1)
    r2 = mk.local(12_007, 9_001, 2, 4, n, right_slot=2)
    if r0.right >= 0:
        assert r0.right == r2.left == 1


def test_boundary_slots_rules():
    """boundary_slots: slot m - 1 before rank m's cells; an empty rank has none; every rank
    holding part of one atmosphere cell uses the slot of the first boundary inside it."""
    idx = np.array([0, 0, 1, 1, 1, 1, 1, 1, 2, 2, 3, 3])  # cell 1 spans 6 exchange cells
    at = lambda x: idx[x]  # noqa: E731
    # APPLE-like: cuts at 3, 5, 7 all inside cell 1: ranks 1 and 2 lie inside it
    assert boundary_slots([(0, 3), (3, 2), (5, 2), (7, 5)], at) == [(-1, 0), (0, 0), (0, 0), (0, -1)]
    # a cut between two cells shares nothing
    assert boundary_slots([(0, 2), (2, 10)], at) == [(-1, -1), (-1, -1)]
    # an empty rank between two ranks that share cell 1: the slot of the next rank with cells
    assert boundary_slots([(0, 4), (0, 0), (4, 8)], at) == [(-1, 1), (-1, -1), (1, -1)]
    # a rank inside cell 1 after an empty rank
    assert boundary_slots([(0, 3), (0, 0), (3, 2), (5, 7)], at) == [(-1, 1), (-1, -1), (1, 1), (1, -1)]
    # the task_ranges rule for every rank with cells is the same
    t = np.array([0, 0, 2, 2, 2, 4], np.int32)
    tr = task_ranges(t, 6)
    got = boundary_slots([(o, s) for o, s, _ in tr], lambda x: np.array([0, 1, 1, 2, 3, 3])[x])
    assert got[0] == (-1, 1) and got[2] == (1, 3) and got[4] == (3, -1)


@pytest.mark.parametrize("cuts", [(1, 2, 3), (1, 3), (1, 2, 3, 4), (2, 4, 7)])
def test_one_atmosphere_cell_over_several_ranks(cuts):
    """A cell spread over three or more ranks: each rank writes its partial sum into the one
    slot (left == right for the ranks inside it), the slot sum over all ranks completes the
    cell for every one of them (what fcx_atmos_allreduce does on the device)."""
    amap = synthetic_atmos_map(64)
    first = int(np.flatnonzero(np.bincount(amap.atmos_index) >= 5)[0])
    c0 = int(np.searchsorted(amap.atmos_index, first))
    bounds = [0] + [c0 + c for c in cuts if c0 + c < 64] + [64]
    ranges = [(a, b - a) for a, b in zip(bounds[:-1], bounds[1:])]
    p = len(ranges)
    x = np.random.default_rng(3).normal(size=64)
    want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, x, amap.n_atmos)
    views = [local_atmos(amap, r, p, ranges=ranges) for r in range(p)]
    total = np.zeros((p - 1, 1))
    parts = []
    for la in views:
        part = oracle_lib.atmos_accumulate(la.atmos_index, la.weight, x[la.offset: la.offset + la.size], la.n_atmos)
        parts.append(part)
        total += pack_boundaries(la, [part], 1)
    for la, part in zip(views, parts):
        unpack_boundaries(la, total, [part])
        np.testing.assert_allclose(part, want[la.atmos_offset: la.atmos_offset + la.n_atmos], rtol=1e-13)
    inside = [la for la in views if la.n_atmos == 1 and la.left >= 0 and la.right >= 0]
    assert inside and all(la.left == la.right for la in inside)


def test_synthetic_map_is_conservative_and_sorted():
    m = synthetic_atmos_map(100_003)
    assert np.all(np.diff(m.atmos_index) >= 0)
    sums = np.bincount(m.atmos_index, weights=m.weight, minlength=m.n_atmos)
    np.testing.assert_allclose(sums, 1.0, rtol=1e-12)
    lengths = np.bincount(m.atmos_index)
    assert 3.5 < lengths.mean() < 4.5 and lengths.min() >= 1


@pytest.mark.parametrize("p", [2, 3, 8])
def test_local_views_agree_on_shared_boundaries(p):
    m = synthetic_atmos_map(50_001)
    views = [local_atmos(m, r, p) for r in range(p)]
    for r in range(p - 1):
        assert (views[r].right == r) == (views[r + 1].left == r)
        if views[r].right >= 0:
            assert views[r].atmos_offset + views[r].n_atmos - 1 == views[r + 1].atmos_offset
        else:
            assert views[r].atmos_offset + views[r].n_atmos == views[r + 1].atmos_offset
    assert sum(v.size for v in views) == 50_001


@pytest.mark.parametrize("cls", ["periodic", "blocked_random"])
@pytest.mark.parametrize("p", [1, 2, 3, 8])
def test_local_structured_maps_match_their_global_map(cls, p):
    """The bench's locally built maps (PeriodicAtmosMap, BlockedRandomAtmosMap): every rank's
    view built from its own range equals the slice of the global map (indices, weights,
    boundary slots as local_atmos gives them); weights conservative; runs of 3..5 cells."""
    from fcx.parallel import BlockedRandomAtmosMap, PeriodicAtmosMap

    n = 50_003  # not a multiple of the 4096-cell blocks: a truncated last block
    mk = PeriodicAtmosMap() if cls == "periodic" else BlockedRandomAtmosMap(seed=5)
    g = mk.global_map(n)
    assert np.all(np.diff(g.atmos_index) >= 0) and g.atmos_index[0] == 0
    np.testing.assert_allclose(np.bincount(g.atmos_index, weights=g.weight), 1.0, rtol=1e-12)
    lengths = np.bincount(g.atmos_index)
    assert lengths[:-1].min() >= 3 and lengths.max() <= 5
    for r in range(p):
        off, size = apple_range(n, r, p)
        v, w = mk.local(off, size, r, p, n), local_atmos(g, r, p)
        assert (v.atmos_offset, v.n_atmos, v.left, v.right) == (w.atmos_offset, w.n_atmos, w.left, w.right)
        np.testing.assert_array_equal(v.atmos_index, w.atmos_index)
        np.testing.assert_array_equal(v.weight, w.weight)
    if cls == "blocked_random":  # segments cross the kernel's 128-cell wave tiles
        b = np.arange(128, n, 128)
        cross = np.mean(g.atmos_index[b - 1] == g.atmos_index[b])
        assert 0.6 < cross < 0.85, cross


def _global_reference(n, amap):
    case = build_case("CCLM", n=n, T=1, bias=True, seed=777)
    out = oracle_lib.run_case(case, "c", current_step_time=3600)
    fields = {}
    for name in ATMOS_FIELDS:
        g = 2 if name == "UMOM" else 3 if name == "VMOM" else 1
        fields[name] = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, out[(1, g, name)], amap.n_atmos)
    return case, out, fields


def _rank_main(rank, world, port, n, q, task=None):
    import torch.distributed as dist
    import torch

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        amap = synthetic_atmos_map(n)
        full, _, _ = _global_reference(n, amap)
        if task is None:
            la = local_atmos(amap, rank, world)
        else:  # the exchange grid's task vector; a rank may own no cells
            off, size, right_slot = task_ranges(task, world)[rank]
            la = local_atmos(amap, rank, world, off, size, right_slot=right_slot)
        lo, hi = la.offset, la.offset + la.size
        # this rank's shard: the same inputs, cut to its APPLE range
        case = build_case("CCLM", n=la.size, T=1, bias=True, seed=777)
        remap = {}
        for key, a in full.lf.field.items():
            if id(a) not in remap:
                remap[id(a)] = np.ascontiguousarray(np.asarray(a)[lo:hi])
            case.lf.field[key] = remap[id(a)]
        init_date, corr = full.corrections
        case.corrections = (init_date, np.ascontiguousarray(corr[lo:hi]))
        out = oracle_lib.run_case(case, "c", current_step_time=3600)
        partial = []
        for name in ATMOS_FIELDS:
            g = 2 if name == "UMOM" else 3 if name == "VMOM" else 1
            partial.append(oracle_lib.atmos_accumulate(la.atmos_index, la.weight, out[(1, g, name)], la.n_atmos))
        buf = torch.from_numpy(pack_boundaries(la, partial, len(ATMOS_FIELDS)))
        dist.all_reduce(buf)  # the ONE collective of the step
        unpack_boundaries(la, buf.numpy(), partial)
        q.put((rank, la.atmos_offset, la.left, [p.tolist() for p in partial],
               {name: out[(1, 2 if name == "UMOM" else 3 if name == "VMOM" else 1, name)][:5].tolist()
                for name in ATMOS_FIELDS}))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _empty_middle_task(n, amap):
    """Task vector of 3 ranks: rank 1 owns no cells (io:101-104), and the cut between ranks 0
    and 2 falls inside an atmosphere cell, so ranks 0 and 2 share it across the empty rank."""
    k = next(i for i in range(n // 2, n) if amap.atmos_index[i - 1] == amap.atmos_index[i])
    task = np.full(n, 2, np.int32)
    task[:k] = 0
    return task


@pytest.mark.parametrize("world,empty_middle", [(2, False), (3, False), (3, True)])
def test_sharded_step_with_one_allreduce_matches_single_process(world, empty_middle):
    import torch.multiprocessing as mp

    n = 30_011
    task = _empty_middle_task(n, synthetic_atmos_map(n)) if empty_middle else None
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, n, q, task)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get() for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    amap = synthetic_atmos_map(n)
    _, _, ref = _global_reference(n, amap)
    got = {name: np.full(amap.n_atmos, np.nan) for name in ATMOS_FIELDS}
    for rank, a0, left, partial, _ in sorted(results):
        for f, name in enumerate(ATMOS_FIELDS):
            vals = np.array(partial[f])
            if left >= 0:  # the shared first cell was completed by the previous rank too
                assert got[name][a0] == vals[0] or np.isnan(got[name][a0])
            got[name][a0: a0 + vals.size] = vals
    for name in ATMOS_FIELDS:
        assert not np.isnan(got[name]).any(), name
        # cells owned by one rank are bit-identical; shared cells differ by association only
        assert mixed_error(got[name], ref[name]) <= 1e-12, name
    assert_parity({k: got[k] for k in ATMOS_FIELDS}, ref, label=f"world={world}")


def _remap_rank(rank, world, port, n, q):
    import torch
    import torch.distributed as dist

    from fcx.parallel import local_links, synthetic_model_map

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        mmap = synthetic_model_map(n, 300, links_per_cell=2)
        x = np.random.default_rng(3).normal(size=n)
        off, size = apple_range(n, rank, world)
        src, dst, w = local_links(mmap, off, size)
        part = torch.from_numpy(oracle_lib.remap_apply(src, dst, w, x[off: off + size], mmap.n_model))
        dist.all_reduce(part)  # the one collective: partial sums of the whole model grid
        q.put((rank, part.numpy().tolist()))
    finally:
        dist.destroy_process_group()


def test_sharded_model_remap_one_allreduce():
    """Exchange -> model remap on APPLE shards: each rank applies its own links to the whole
    model grid, one all-reduce completes it; equal to the single-process remap up to the
    association of the shared model cells."""
    import torch.multiprocessing as mp

    from fcx.parallel import synthetic_model_map

    n, world = 20_003, 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_remap_rank, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get() for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    mmap = synthetic_model_map(n, 300, links_per_cell=2)
    x = np.random.default_rng(3).normal(size=n)
    ref = oracle_lib.remap_apply(mmap.src, mmap.dst, mmap.weight, x, mmap.n_model)
    for _, vals in res:
        assert mixed_error(np.array(vals), ref) <= 1e-12
    np.testing.assert_array_equal(np.array(res[0][1]), np.array(res[1][1]))  # every rank gets it


def test_geometric_maps_are_conservative_and_ordered():
    """fcx.parallel.geometric_maps: every exchange cell in exactly one atmosphere and one
    ocean cell, exchange cells ordered by atmosphere cell (contiguous runs), weights summing
    to 1 per atmosphere and per (covered) ocean cell, areas tiling the domain."""
    from fcx.parallel import geometric_maps

    am, mm = geometric_maps(40)
    n = am.atmos_index.size
    assert mm.src.size == n and np.array_equal(mm.src, np.arange(n))
    assert np.all(np.diff(am.atmos_index) >= 0) and am.n_atmos == 1600
    runs = np.bincount(am.atmos_index, minlength=am.n_atmos)
    assert runs.min() >= 1 and runs.max() <= 9
    np.testing.assert_allclose(np.bincount(am.atmos_index, weights=am.weight), 1.0, rtol=1e-13)
    s = np.bincount(mm.dst, weights=mm.weight, minlength=mm.n_model)
    np.testing.assert_allclose(s[s > 0], 1.0, rtol=1e-13)
    # within an atmosphere cell the ocean cells come row by row
    assert n == pytest.approx(am.n_atmos * (1 + 1 / 0.75) ** 2, rel=0.05)


@pytest.mark.parametrize("mapcls", ["PeriodicAtmosMap", "BlockedRandomAtmosMap"])
def test_structured_maps_take_the_boundary_slot_rule(mapcls):
    """With every rank's ranges, the O(size) structured maps of the bench give the slots of
    boundary_slots on their global map -- including ranks inside one atmosphere cell
    (left == right) and APPLE ranges of many ranks."""
    import fcx.parallel as par

    mk = getattr(par, mapcls)()
    n = 20_000
    g = mk.global_map(n)
    c0 = int(np.flatnonzero(np.bincount(g.atmos_index) >= 4)[5])
    c0 = int(np.searchsorted(g.atmos_index, c0))
    cases = [[apple_range(n, r, 7) for r in range(7)],
             [(0, c0 + 1), (c0 + 1, 1), (c0 + 2, 1), (c0 + 3, n - c0 - 3)]]
    for ranges in cases:
        p = len(ranges)
        for rank, (off, size) in enumerate(ranges):
            a = mk.local(off, size, rank, p, n, ranges=ranges)
            b = local_atmos(g, rank, p, ranges=ranges)
            assert (a.left, a.right, a.n_atmos, a.atmos_offset) == (b.left, b.right, b.n_atmos, b.atmos_offset)


def _random_run_map(n, lengths, rng):
    """A sorted exchange -> atmosphere map with runs of `lengths` cells (0: atmosphere cells
    no exchange cell maps to), normalised weights."""
    from fcx.parallel import AtmosMap

    runs = rng.integers(lengths[0], lengths[1] + 1, n + 1)
    while runs.sum() < n:  # (ranges with empty runs can fall short of n cells)
        runs = np.concatenate([runs, rng.integers(lengths[0], lengths[1] + 1, n + 1)])
    ends = np.cumsum(runs)
    n_atmos = int(np.searchsorted(ends, n, side="left")) + 1
    idx = np.repeat(np.arange(n_atmos, dtype=np.int32), runs[:n_atmos])[:n]
    area = rng.uniform(0.5, 1.5, n)
    w = area / np.maximum(np.bincount(idx, weights=area, minlength=n_atmos)[idx], 1e-300)
    return AtmosMap(np.ascontiguousarray(idx), np.ascontiguousarray(w), n_atmos)


@pytest.mark.parametrize("seed", range(40))
def test_random_partitions_complete_every_cell(seed):
    """Random maps (runs of 0..5 up to 1..300 cells), 1-16 ranks, APPLE ranges or random task
    ranges with empty ranks anywhere: every rank's partial sums plus ONE sum over the ranks of
    the packed boundary slots (what the all-reduce does) complete every atmosphere cell of
    every rank, equal to the global sequential sum (exactly for the cells one rank owns)."""
    rng = np.random.default_rng([seed, 41])
    n = int(rng.integers(1, 5_000))
    lengths = [(0, 5), (1, 5), (1, 10), (20, 64), (1, 300)][int(rng.integers(0, 5))]
    amap = _random_run_map(n, lengths, rng)
    p = int(rng.integers(1, 17))
    if rng.random() < 0.5:
        ranges = None  # APPLE (decomp_def.F90:23-31)
    else:  # a task vector's ranges: sorted cuts, empty ranks allowed (io:101-104)
        cuts = np.sort(rng.integers(0, n + 1, p - 1))
        b = np.concatenate([[0], cuts, [n]])
        ranges = [(int(b[r]), int(b[r + 1] - b[r])) for r in range(p)]
    x = rng.normal(size=n)
    want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, x, amap.n_atmos)
    views = [local_atmos(amap, r, p, ranges=ranges) for r in range(p)]
    total = np.zeros((max(p - 1, 1), 1))
    parts = []
    for la in views:
        part = oracle_lib.atmos_accumulate(la.atmos_index, la.weight, x[la.offset: la.offset + la.size], la.n_atmos)
        parts.append(part)
        if p > 1:
            total += pack_boundaries(la, [part], 1)
    owners = np.zeros(amap.n_atmos, np.int32)
    for la, part in zip(views, parts):
        if p > 1:
            unpack_boundaries(la, total, [part])
        sl = slice(la.atmos_offset, la.atmos_offset + la.n_atmos)
        owners[sl] += 1
        np.testing.assert_allclose(part, want[sl], rtol=1e-12, atol=1e-12, err_msg=f"seed {seed} rank view {la}")
    # every atmosphere cell some rank maps to is covered; a cell of one rank is exact
    covered = np.zeros(amap.n_atmos, bool)
    covered[np.unique(amap.atmos_index)] = True
    assert np.all(owners[covered] >= 1), f"seed {seed}: atmosphere cells no rank completes"
    for la, part in zip(views, parts):
        sl = np.arange(la.atmos_offset, la.atmos_offset + la.n_atmos)
        one = owners[sl] == 1
        np.testing.assert_array_equal(part[one], want[sl][one], err_msg=f"seed {seed}")


def test_synthetic_maps_cover_every_exchange_cell():
    """The synthetic exchange -> atmosphere and exchange -> model maps give every exchange
    cell a link (a remap draw of 48 exchange cells, 3 model cells and 2 links per cell once
    drew runs covering fewer cells than the grid: seed base 450000 of the random remap test),
    and 2 links per cell need 2 model cells."""
    from fcx.parallel import synthetic_atmos_map, synthetic_model_map

    for n in list(range(1, 130)) + [4095, 4097]:
        for seed in range(3):
            m = 2 + seed
            one = synthetic_model_map(n, m, links_per_cell=1, seed=seed)
            two = synthetic_model_map(n, m, links_per_cell=2, seed=seed)
            for mm, links in ((one, 1), (two, 2)):
                assert mm.src.size == links * n and np.array_equal(np.unique(mm.src), np.arange(n))
            # conservative: the weights of a model cell's exchange cells sum to 1; the second
            # link splits each cell's weight, so the total stays the number of owner cells
            np.testing.assert_allclose(one.weight.sum(), np.unique(one.dst).size, rtol=1e-12)
            np.testing.assert_allclose(two.weight.sum(), one.weight.sum(), rtol=1e-12)
            for cpa in (1, 4):
                am = synthetic_atmos_map(n, cells_per_atmos=cpa, seed=seed)
                assert am.atmos_index.size == n and np.all(np.diff(am.atmos_index) >= 0)
    mm = synthetic_model_map(48, 3, links_per_cell=2, seed=4508101)
    assert mm.src.size == 96
    with pytest.raises(ValueError):
        synthetic_model_map(10, 1, links_per_cell=2)

