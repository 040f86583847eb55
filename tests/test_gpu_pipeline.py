"""The host-bound fcx_step: caller heap arrays through the engine's page-locked staging arena
(FCX_OPT_HOST_STAGING, default) or one runtime copy per array, arrays in library memory
(fcx_host_malloc, direct DMA or zero-copy), and the step pipelined over cell chunks
(FCX_OPT_PIPELINE_CHUNKS: H2D of chunk k+1, kernel of chunk k, D2H of chunk k-1 on three
streams, the staging copies of chunk k+1 and k-2 on the host in between).  Every transport
and chunking must give the bits of the sequential upload/run/download step, and those are
within tests/parity.py of the oracle."""
import numpy as np
import pytest

import oracle_lib
from parity import assert_parity

pytestmark = pytest.mark.gpu

from fcx.basic import PHASE_ALL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.parallel import local_atmos, synthetic_atmos_map  # noqa: E402
from fcx.synthetic import build_case  # noqa: E402

STEP_T = 3600 * 24 * 40


def library(case):
    """The case's arrays moved into library-allocated page-locked memory (fcx_host_malloc),
    which the kernels use in place (zero-copy); close the returned arena after the engines."""
    from fcx.host_alloc import Arena

    arena = Arena()
    arena.adopt(case.lf)
    return arena


def run(case, options, atmos_n=None):
    """One fcx_step on fresh copies of the case's outputs; returns the outputs (and the
    atmosphere fields when atmos_n is given)."""
    for k in case.outputs:
        case.lf.field[k][:] = np.nan
    atmos, outs = None, None
    if atmos_n is not None:
        amap = synthetic_atmos_map(atmos_n)
        outs = {name: np.full(amap.n_atmos, np.nan) for name in ("MEVA", "HSEN", "UMOM")}
        atmos = {"local": local_atmos(amap, 0, 1),
                 "fields": [(2, 1, 1, "MEVA", outs["MEVA"]), (2, 1, 1, "HSEN", outs["HSEN"]),
                            (2, 1, 2, "UMOM", outs["UMOM"])]}
    # small test grids: let the pipeline cut chunks down to 1024 cells
    options = {"pipeline_min_chunk": 1024, **options}
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, atmos=atmos, options=options)
    eng.step(PHASE_ALL, STEP_T)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    if outs is not None:
        got.update({("atm", name): v.copy() for name, v in outs.items()})
    return got


def same_bits(a, b):
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=str(k))


@pytest.mark.parametrize("variant", ["CCLM", "RCO"])
def test_pipeline_chunkings_bit_identical(variant):
    case = build_case(variant, n=100_003, T=1, bias=True)
    seq = run(case, {"pipeline_chunks": 1})
    for chunks in (2, 3, 8, 97):
        same_bits(run(case, {"pipeline_chunks": chunks}), seq)
        same_bits(run(case, {"pipeline_chunks": chunks, "host_staging": 0}), seq)
    # the heap arrays' arena used in place by every chunk launch (zero-copy forced)
    same_bits(run(case, {"pipeline_chunks": 8, "zero_copy": 1}), seq)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(seq, ref, label=variant)


def test_pipeline_with_fused_atmosphere_accumulation():
    """Chunk boundaries cut atmosphere segments: carries + the fix-up after the last chunk."""
    n = 50_001
    case = build_case("MOM5", n=n, T=1, bias=True)
    seq = run(case, {"pipeline_chunks": 1}, atmos_n=n)
    for chunks in (4, 7):
        same_bits(run(case, {"pipeline_chunks": chunks}, atmos_n=n), seq)


def test_pipeline_generic_kernel_separate_grids_and_averages():
    case = build_case("CCLM", n=20_011, T=3, sep_grids=(19_997, 20_101), bias=True)
    seq = run(case, {"pipeline_chunks": 1})
    same_bits(run(case, {"pipeline_chunks": 5}), seq)
    same_bits(run(case, {"pipeline_chunks": 5, "host_staging": 0}), seq)
    same_bits(run(case, {"pipeline_chunks": 5, "tiled_layout": 0}), seq)  # plain mirror pool
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(seq, ref, label="T3 sep")


@pytest.mark.parametrize("n", [3_000, 32_768])
@pytest.mark.parametrize("atmos", [False, True])
@pytest.mark.parametrize("zero_copy", [0, 1])
def test_staging_matches_runtime_copies(n, atmos, zero_copy):
    """The Baltic-size step (32,768 cells) and small arrays several to a heap page (3,000
    cells, T = 2): the staging arena -- moved by DMA (zero_copy 0) or used by the kernels in
    place (zero_copy 1, the small-grid default) -- gives the bits of one runtime copy per
    array, with the atmosphere outputs staged too; only the staged engine holds an arena."""
    case = build_case("CCLM", n=n, T=2 if n < 10_000 else 1, bias=True)
    a = run(case, {"pipeline_chunks": 2, "zero_copy": zero_copy}, atmos_n=n if atmos else None)
    b = run(case, {"pipeline_chunks": 1, "host_staging": 0}, atmos_n=n if atmos else None)
    same_bits(a, b)
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages)
    assert eng.staging_bytes() > 0
    eng.close()
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, options={"host_staging": 0})
    assert eng.staging_bytes() == 0
    eng.close()


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_staging_host_threads(threads):
    """The arena's host copies on 1, 3 or 8 threads: the same bits."""
    case = build_case("MOM5", n=40_001, T=1, bias=True)
    same_bits(run(case, {"host_threads": threads}), run(case, {"host_staging": 0}))


def test_engines_sharing_heap_arrays_and_pages():
    """Two live engines over the same heap arrays and a third whose small arrays sit on the
    same heap pages, each with its own arena, closed in every order: every remaining engine
    stays correct (nothing of the caller's memory is locked or mapped, so nothing is shared
    between them but the arrays)."""
    a = build_case("CCLM", n=2_001, T=2, bias=True)
    b = build_case("CCLM", n=2_001, T=2, bias=True)  # allocated right after: shares pages
    ref_a = run(a, {"host_staging": 0})
    ref_b = run(b, {"host_staging": 0})

    def engine(case):
        return Engine(case.lf, 2, case.methods, corrections=case.corrections, averages=case.averages)

    def step(eng, case):
        for k in case.outputs:
            case.lf.field[k][:] = np.nan
        eng.step(PHASE_ALL, STEP_T)
        return {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}

    for close_first in (0, 1, 2):
        e = [engine(a), engine(a), engine(b)]
        e[close_first].close()
        for i, (eng, case, ref) in enumerate(((e[0], a, ref_a), (e[1], a, ref_a), (e[2], b, ref_b))):
            if i != close_first:
                same_bits(step(eng, case), ref)
        for i in range(3):
            if i != close_first:
                e[i].close()


def test_upload_run_download_synchronize():
    """The split step: outputs reach the caller's arrays at fcx_synchronize; an upload issued
    while a download still owes its host copies completes that download first."""
    case = build_case("RCO", n=20_011, T=1, bias=True)
    want = run(case, {"host_staging": 0})
    for k in case.outputs:
        case.lf.field[k][:] = np.nan
    eng = Engine(case.lf, 1, case.methods, corrections=case.corrections, averages=case.averages)
    for rep in range(2):
        eng.upload(PHASE_ALL)
        eng.run(PHASE_ALL, STEP_T)
        eng.download(PHASE_ALL)
        if rep == 1:
            eng.synchronize()
        else:
            eng.upload(PHASE_ALL)  # no synchronize in between: the download is completed here
        same_bits({k: np.array(case.lf.field[k], copy=True) for k in case.outputs}, want)
    eng.close()


def test_default_min_chunk_keeps_small_grids_sequential():
    """Below 2 x 256K cells the default step is the sequential mirrored one (same bits as an
    explicitly sequential engine)."""
    case = build_case("RCO", n=70_000, T=1)
    for k in case.outputs:
        case.lf.field[k][:] = np.nan
    eng = Engine(case.lf, 1, case.methods)
    eng.step(PHASE_ALL, STEP_T)
    a = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    same_bits(a, run(case, {"pipeline_chunks": 1}))


def steps_with_changing_inputs(case, options, steps=3):
    """Several fcx_steps, the host rewriting every input between them (as oasis_get does):
    zero-copy kernels must see each step's fresh host data and leave their writes visible."""
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, options=options)
    inputs = [k for k in case.lf.field if k not in case.outputs]
    seen, res = set(), []
    orig = {}
    for k in inputs:
        a = case.lf.field[k]
        if id(a) not in seen:
            seen.add(id(a))
            orig[id(a)] = a.copy()
    for step in range(steps):
        for k in inputs:
            a = case.lf.field[k]
            if k[2] in ("TSUR", "TATM", "UATM", "VATM", "QATM"):
                a[:] = orig[id(a)] * (1.0 + 1e-3 * step)  # inputs of this step
        for k in case.outputs:
            case.lf.field[k][:] = np.nan
        eng.step(PHASE_ALL, STEP_T + 3600 * step)
        res.append({k: np.array(case.lf.field[k], copy=True) for k in case.outputs})
    eng.close()
    for k in inputs:  # restore
        a = case.lf.field[k]
        a[:] = orig[id(a)]
    return res


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
def test_staged_steps_see_fresh_inputs(variant):
    """Heap arrays through the staging arena over several steps, the host rewriting the inputs
    between them: each step gathers the current host values."""
    case = build_case(variant, n=40_001, T=1, bias=True)
    staged = steps_with_changing_inputs(case, {})
    direct = steps_with_changing_inputs(case, {"host_staging": 0})
    for a, b in zip(staged, direct):
        same_bits(a, b)
    assert not any(np.isnan(v).any() for v in staged[-1].values())


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
def test_zero_copy_matches_mirrors_over_steps(variant):
    case = build_case(variant, n=40_001, T=1, bias=True)
    arena = library(case)
    zc = steps_with_changing_inputs(case, {"zero_copy": 1})
    mir = steps_with_changing_inputs(case, {"zero_copy": 0, "pipeline_chunks": 1})
    arena.close()
    for a, b in zip(zc, mir):
        same_bits(a, b)
    assert not any(np.isnan(v).any() for v in zc[-1].values())


def test_zero_copy_generic_separate_grids_averages_and_atmosphere():
    case = build_case("CCLM", n=9_001, T=3, sep_grids=(8_999, 9_011), bias=True)
    arena = library(case)
    same_bits(run(case, {"zero_copy": 1}), run(case, {"zero_copy": 0}))
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(run(case, {"zero_copy": 1}), ref, label="zero-copy T3 sep")
    arena.close()
    c1 = build_case("MOM5", n=30_001, T=1, bias=True)
    arena = library(c1)
    same_bits(run(c1, {"zero_copy": 1}, atmos_n=30_001), run(c1, {"zero_copy": 0}, atmos_n=30_001))
    arena.close()


def test_zero_copy_per_call_dropin():
    """The per-call reference subroutines on a zero-copy engine over library arrays (no
    copies at all; each kernel reads the previous call's outputs in host memory)."""
    from fcx.basic import IDX

    case = build_case("CCLM", n=5_003, T=2, bias=True)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    arena = library(case)
    for k in case.outputs:
        case.lf.field[k][:] = np.nan
    eng = Engine(case.lf, 2, case.methods, corrections=case.corrections, averages=case.averages,
                 options={"zero_copy": 1})
    assert eng.zero_copy_bytes() > 0 and eng.staging_bytes() == 0
    lib, h = eng.lib, eng.h
    assert lib.fcx_calc_flux_radiation_blackbody(h) == 0
    for g in (1, 2, 3):
        assert lib.fcx_calc_spec_vapor_surface(h, g) == 0
    assert lib.fcx_calc_flux_mass_evap(h, STEP_T) == 0
    assert lib.fcx_calc_flux_heat_latent(h) == 0
    assert lib.fcx_calc_flux_heat_sensible(h) == 0
    assert lib.fcx_calc_flux_momentum_east(h, 2) == 0
    assert lib.fcx_calc_flux_momentum_north(h, 3) == 0
    for ph, g, name in case.averages:
        assert lib.fcx_average_across_surface_types(h, g, IDX[name]) == 0
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    arena.close()
    assert_parity(got, ref, label="zero-copy per call")


def test_pipeline_multi_type_register_averages_and_fused_accumulation():
    """T=3: type-0 averages in the LDS slots, their accumulation fused, chunked host step."""
    n = 60_001
    case = build_case("CCLM", n=n, T=3, bias=True)
    amap = synthetic_atmos_map(n)
    outs = {name: np.full(amap.n_atmos, np.nan) for name in ("MEVA", "HSEN", "UMOM")}
    atmos = {"local": local_atmos(amap, 0, 1),
             "fields": [(2, 0, 1, "MEVA", outs["MEVA"]), (2, 0, 1, "HSEN", outs["HSEN"]),
                        (2, 0, 2, "UMOM", outs["UMOM"])]}
    res = []
    for chunks in (1, 6):
        for k in case.outputs:
            case.lf.field[k][:] = np.nan
        for v in outs.values():
            v[:] = np.nan
        eng = Engine(case.lf, 3, case.methods, corrections=case.corrections, averages=case.averages,
                     atmos=atmos, options={"pipeline_min_chunk": 1024, "pipeline_chunks": chunks})
        eng.step(PHASE_ALL, STEP_T)
        eng.close()
        res.append({**{k: np.array(case.lf.field[k], copy=True) for k in case.outputs},
                    **{("atm", k): v.copy() for k, v in outs.items()}})
    same_bits(res[0], res[1])
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity({k: res[0][k] for k in case.outputs}, ref, label="T3 chunked")
    for name in outs:
        g = 2 if name == "UMOM" else 1
        want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, res[0][(0, g, name)], amap.n_atmos)
        np.testing.assert_array_equal(res[0][("atm", name)], want, err_msg=name)


@pytest.mark.parametrize("n", [32_768, 600_001])
def test_download_fills_heap_arrays_without_synchronize(n):
    """fcx_download through the staging arena fills the caller's heap arrays before it
    returns: a host that waits with a device-wide sync of its own (torch.cuda.synchronize),
    never calling fcx_synchronize, reads the outputs.  With FCX_OPT_DEFERRED_SCATTER they
    arrive at fcx_synchronize instead."""
    import torch

    case = build_case("MOM5", n=n, T=1, bias=True)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    for deferred in (0, 1):
        for k in case.outputs:
            case.lf.field[k][:] = np.nan
        eng = Engine(case.lf, 1, case.methods, corrections=case.corrections,
                     options={"deferred_scatter": deferred})
        assert eng.staging_bytes() > 0 or eng.zero_copy_active()
        eng.upload(PHASE_ALL)
        eng.run(PHASE_ALL, STEP_T)
        eng.download(PHASE_ALL)
        torch.cuda.synchronize()
        got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
        if deferred:
            assert all(np.isnan(v).all() for v in got.values())  # still in the arena
            eng.synchronize()
            got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
        eng.close()
        assert_parity(got, {k: ref[k] for k in case.outputs}, label=f"n={n} deferred={deferred}")


def test_staging_arena_failure_falls_back_to_direct_copies(monkeypatch):
    """A node that cannot page-lock the staging arena (FCX_TEST_PIN_FAIL=1 makes every image
    fail at fcx_commit): the pools fall back to one runtime copy per array, the step runs,
    no pinned bytes are reported, and the outputs are the bits of the staged step."""
    case = build_case("CCLM", n=600_001, T=2, bias=True)
    opts = {"pipeline_chunks": 4, "pipeline_min_chunk": 65_536, "zero_copy": 0}
    want = run(case, opts, atmos_n=600_001)
    monkeypatch.setenv("FCX_TEST_PIN_FAIL", "1")
    got = run(case, opts, atmos_n=600_001)
    same_bits(got, want)
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, options=opts)
    assert eng.staging_bytes() == 0
    eng.close()


@pytest.mark.parametrize("n", [32_768, 600_001])
def test_step_async_engines_started_from_one_thread(n):
    """fcx_step_async (the asynchronous phase, Fortran fcx_start_phase / fcx_finish_phase):
    three engines on their own streams started one after the other from ONE host thread,
    the host overwriting every input array before it synchronizes (as the next oasis_get
    would) -- the outputs are those of fcx_step on the inputs at the start, bit for bit.  At
    32,768 cells the downloads complete at fcx_synchronize; at 600,001 the chunk pipeline
    completes inside the call."""
    import torch

    variants = ("CCLM", "MOM5", "RCO")
    cases = [build_case(v, n=n, T=1, bias=True, seed=3 + i) for i, v in enumerate(variants)]
    want = []
    for c in cases:  # reference: the synchronous step of fresh engines
        for k in c.outputs:
            c.lf.field[k][:] = np.nan
        e = Engine(c.lf, 1, c.methods, corrections=c.corrections)
        e.step(PHASE_ALL, STEP_T)
        want.append({k: np.array(c.lf.field[k], copy=True) for k in c.outputs})
        e.close()
    streams = [torch.cuda.Stream() for _ in cases]
    engines = [Engine(c.lf, 1, c.methods, corrections=c.corrections, stream=s.cuda_stream)
               for c, s in zip(cases, streams)]
    inputs = []
    for c in cases:
        seen = {id(c.lf.field[k]) for k in c.outputs}  # (outputs are aliased under other slots too)
        for k, a in c.lf.field.items():
            if id(a) not in seen:
                seen.add(id(a))
                inputs.append((a, a.copy()))
        for k in c.outputs:
            c.lf.field[k][:] = np.nan
    for e in engines:
        e.step_async(PHASE_ALL, STEP_T)
    for a, _ in inputs:  # the host reuses its input arrays before the steps are waited for
        a *= 2.0
    for e in engines:
        e.synchronize()
    got = [{k: np.array(c.lf.field[k], copy=True) for k in c.outputs} for c in cases]
    for e in engines:
        e.close()
    for a, orig in inputs:
        a[:] = orig
    for g, w in zip(got, want):
        same_bits(g, w)


def test_step_async_engines_on_library_memory():
    """The Baltic-size step bench.py reports as baltic_size.gpu_dropin_library_memory: the
    three variants' fields in fcx_host_malloc memory (read and written in place, zero-copy),
    started with fcx_step_async from one thread on their own streams, then a second step on
    changed inputs, asynchronous and again with fcx_step one engine after the other -- the
    bits of the synchronous step on caller heap arrays every time.  (fcx_host_malloc inputs
    are read in place until fcx_synchronize, so the host leaves them alone until then.)"""
    import torch
    from fcx.host_alloc import Arena

    n = 32_768
    variants = ("CCLM", "MOM5", "RCO")

    def make():
        return [build_case(v, n=n, T=1, bias=True, seed=30 + i) for i, v in enumerate(variants)]

    def scale_inputs(c):  # every distinct input array once (aliases share it)
        outs = {id(c.lf.field[k]) for k in c.outputs}
        for a in {id(a): a for a in c.lf.field.values() if id(a) not in outs}.values():
            a *= 1.001

    def outputs(c):
        return {k: np.array(c.lf.field[k], copy=True) for k in c.outputs}

    want = [[], []]
    for c in make():  # the reference: caller heap arrays, synchronous steps
        e = Engine(c.lf, 1, c.methods, corrections=c.corrections)
        e.step(PHASE_ALL, STEP_T)
        want[0].append(outputs(c))
        scale_inputs(c)
        e.step(PHASE_ALL, STEP_T + 3600)
        want[1].append(outputs(c))
        e.close()
    cases = make()
    with Arena() as arena:
        for c in cases:
            arena.adopt(c.lf)
            for k in c.outputs:
                c.lf.field[k][:] = np.nan
        streams = [torch.cuda.Stream() for _ in cases]
        engines = [Engine(c.lf, 1, c.methods, corrections=c.corrections, stream=s.cuda_stream)
                   for c, s in zip(cases, streams)]
        assert all(e.staging_bytes() == 0 for e in engines)  # used in place: no staging arena
        for step, t in enumerate((STEP_T, STEP_T + 3600)):
            if step:
                for c in cases:
                    scale_inputs(c)
            for e in engines:
                e.step_async(PHASE_ALL, t)
            for e in engines:
                e.synchronize()
            for c, w in zip(cases, want[step]):
                same_bits(outputs(c), w)
        for c in cases:
            for k in c.outputs:
                c.lf.field[k][:] = np.nan
        for e in engines:
            e.step(PHASE_ALL, STEP_T + 3600)
        for c, w in zip(cases, want[1]):
            same_bits(outputs(c), w)
        for e in engines:
            e.close()


@pytest.mark.parametrize("n", [32_768, 600_001])
@pytest.mark.parametrize("variant", ["CCLM", "MOM5"])
def test_fields_handed_over_one_by_one(variant, n):
    """fcx_upload_field (the OASIS staging glue: each input field handed over after its
    oasis_get, staged by the engine's upload thread): all of them, or every other one with
    fcx_step moving the rest, over two steps with changed inputs -- the bits of fcx_step."""
    case = build_case(variant, n=n, T=1, bias=True, seed=9)
    outs = {id(case.lf.field[k]) for k in case.outputs}
    slots, seen = [], set()
    for (s, g, name), a in case.lf.field.items():
        if id(a) not in outs and id(a) not in seen:
            seen.add(id(a))
            slots.append(((s, g, name), a))
    orig = [a.copy() for _, a in slots]

    def steps(hand_over):
        res = []
        eng = Engine(case.lf, 1, case.methods, corrections=case.corrections)
        for step in range(2):
            for (_, a), o in zip(slots, orig):
                a[:] = o * (1.0 + 1e-3 * step)  # this step's inputs, as oasis_get writes them
            for k in case.outputs:
                case.lf.field[k][:] = np.nan
            for i, (key, _) in enumerate(slots):
                if hand_over == "all" or (hand_over == "half" and i % 2 == 0):
                    eng.upload_field(*key)
            eng.step(PHASE_ALL, STEP_T + 3600 * step)
            res.append({k: np.array(case.lf.field[k], copy=True) for k in case.outputs})
        eng.close()
        return res

    want = steps(None)
    for mode in ("all", "half"):
        for a, b in zip(steps(mode), want):
            same_bits(a, b)
    for (_, a), o in zip(slots, orig):
        a[:] = o


def test_staging_pins_only_what_a_step_transfers():
    """the staging arena page-locks, at fcx_commit, the pools a whole step moves;
    the pool of bound arrays no step reads or writes (here CMOI, CHEA, CMOM, FARE, ALBE,
    ALBA, RSDD of a CCLM case: 7 of its 24 arrays) is page-locked only if a call ever
    transfers it.  The step's results are unchanged.  (The grid is below the zero-copy size,
    so that transport is switched off: its mapped arena holds every heap array by design.)"""
    n = 200_000
    case = build_case("CCLM", n=n, T=1, bias=False, seed=4)
    distinct = {id(a) for a in case.lf.field.values()}
    eng = Engine(case.lf, 1, case.methods, options={"zero_copy": 0})
    pinned = eng.staging_bytes()
    assert 0 < pinned < 0.85 * len(distinct) * n * 8, (pinned, len(distinct))
    for k in case.outputs:
        case.lf.field[k][:] = np.nan
    eng.step(PHASE_ALL, STEP_T)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    assert eng.staging_bytes() == pinned  # a whole step transfers nothing outside those pools
    eng.close()
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(got, ref, label="lazy staging pools")


def test_lazy_pool_pin_failure_takes_the_direct_path(monkeypatch):
    """a lazy staging pool (page-locked at its first transfer) whose image cannot
    be page-locked is disabled and its arrays take the direct path (one runtime copy each),
    as at commit -- no FCX_E_NOMEM reaches the caller.  FCX_TEST_PIN_FAIL=2 fails only the
    lazy pools; CMOI of a CCLM case lives in one (no whole step reads it) and is handed over
    with fcx_upload_field, then a step and the per-call subroutines run."""
    from fcx import flux_calculator_calculate as fcc  # noqa: F401  (the module loads the ABI)

    n = 200_000
    case = build_case("CCLM", n=n, T=1, bias=False, seed=4)
    eng = Engine(case.lf, 1, case.methods, options={"zero_copy": 0})
    pinned = eng.staging_bytes()
    monkeypatch.setenv("FCX_TEST_PIN_FAIL", "2")
    eng.upload_field(1, 1, "CMOI")  # the lazy pool: its pin fails, the direct copy runs
    for k in case.outputs:
        case.lf.field[k][:] = np.nan
    eng.step(PHASE_ALL, STEP_T)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    assert eng.staging_bytes() == pinned  # the failed pool holds no image
    lib = eng.lib
    for k in case.outputs:
        case.lf.field[k][:] = np.nan
    for g in (1, 2, 3):
        assert lib.fcx_calc_spec_vapor_surface(eng.h, g) == 0, lib.fcx_last_error()
    assert lib.fcx_calc_flux_mass_evap(eng.h, STEP_T) == 0, lib.fcx_last_error()
    assert lib.fcx_calc_flux_heat_latent(eng.h) == 0
    assert lib.fcx_calc_flux_heat_sensible(eng.h) == 0
    assert lib.fcx_calc_flux_momentum_east(eng.h, 2) == 0
    assert lib.fcx_calc_flux_momentum_north(eng.h, 3) == 0
    assert lib.fcx_calc_flux_radiation_blackbody(eng.h) == 0
    per_call = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(got, ref, label="lazy pool pin failure, step")
    assert_parity(per_call, ref, label="lazy pool pin failure, per call")


def test_handed_over_arrays_may_change_after_the_next_call():
    """fcx_upload_field's contract (include/fcx.h): the array must not change
    until the next engine call returns; after that the host may overwrite it and the run uses
    the value handed over.  Every input handed over, fcx_synchronize returns, the inputs are
    overwritten with garbage, then the step: bit-identical to a step on the original inputs."""
    case = build_case("MOM5", n=32_768, T=1, bias=True, seed=12)
    outs = {id(case.lf.field[k]) for k in case.outputs}
    slots, seen = [], set()
    for (s, g, name), a in case.lf.field.items():
        if id(a) not in outs and id(a) not in seen:
            seen.add(id(a))
            slots.append(((s, g, name), a))
    orig = [a.copy() for _, a in slots]
    eng = Engine(case.lf, 1, case.methods, corrections=case.corrections)
    eng.step(PHASE_ALL, STEP_T)
    want = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    for key, _ in slots:
        eng.upload_field(*key)
    eng.synchronize()  # the next engine call: the handed-over arrays are the engine's now
    for _, a in slots:
        a[:] = -1.0e30
    for k in case.outputs:
        case.lf.field[k][:] = np.nan
    eng.step(PHASE_ALL, STEP_T)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    for (_, a), o in zip(slots, orig):
        a[:] = o
    same_bits(got, want)
