"""Exchange -> model remaps on the GPU (fcx_add_remap): the SCRIP weight
application OASIS performs on the fields sent to a bottom model, CSR by destination in link
order, checked bit for bit against the sequential application (oracle/fco.c:fco_remap_apply)
on the GPU's own fluxes; the fluxes themselves against the oracle (tests/parity.py)."""
import numpy as np
import pytest

import oracle_lib
from parity import assert_parity, mixed_error

pytestmark = pytest.mark.gpu

from fcx.basic import PHASE_ALL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.parallel import apple_range, local_links, synthetic_model_map  # noqa: E402
from fcx.synthetic import as_dtype, build_case  # noqa: E402

STEP_T = 3600 * 24 * 40
FIELDS = (("MEVA", 1), ("HSEN", 1), ("UMOM", 2), ("VMOM", 3))


def remap_spec(mmap, outs, s=1, src=None, dst=None, w=None):
    return {"n_dst": mmap.n_model, "src": mmap.src if src is None else src, "dst": mmap.dst if dst is None else dst,
            "w": mmap.weight if w is None else w,
            "fields": [(2, s, g, name, outs[name]) for name, g in FIELDS]}


@pytest.mark.parametrize("links", [1, 2])
@pytest.mark.parametrize("device_out", [False, True])
@pytest.mark.parametrize("pack", [0, 1, 2])
def test_remap_bit_exact(links, device_out, pack):
    """pack: FCX_OPT_REMAP_PACK -- the gather from the field arrays (0), or from the packed
    records (1, 2 = auto with these four fields); the same bits every way."""
    torch = pytest.importorskip("torch")
    n = 30_011
    case = build_case("CCLM", n=n, T=1, bias=True)
    mmap = synthetic_model_map(n, 2_000, links_per_cell=links)
    if device_out:
        outs = {k: torch.full((mmap.n_model,), float("nan"), dtype=torch.float64, device="cuda:0") for k, _ in FIELDS}
    else:
        outs = {k: np.full(mmap.n_model, np.nan) for k, _ in FIELDS}
    eng = Engine(case.lf, 1, case.methods, corrections=case.corrections, remaps=[remap_spec(mmap, outs)],
                 options={"remap_pack": pack})
    eng.step(PHASE_ALL, STEP_T)
    eng.close()
    for name, g in FIELDS:
        want = oracle_lib.remap_apply(mmap.src, mmap.dst, mmap.weight, np.asarray(case.lf.field[(1, g, name)]),
                                      mmap.n_model)
        got = outs[name].cpu().numpy() if device_out else outs[name]
        np.testing.assert_array_equal(got, want, err_msg=name)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity({k: np.asarray(case.lf.field[k]) for k in case.outputs}, ref, label="remap fluxes")


def test_remap_of_type0_averages_in_a_pipelined_step():
    """T=3: the model receives the type-0 averages; chunked host step; two remap targets."""
    n = 40_003
    case = build_case("MOM5", n=n, T=3, bias=True)
    m1 = synthetic_model_map(n, 1_500, links_per_cell=2, seed=1)
    m2 = synthetic_model_map(n, 900, links_per_cell=1, seed=2)
    o1 = {k: np.full(m1.n_model, np.nan) for k, _ in FIELDS}
    o2 = {k: np.full(m2.n_model, np.nan) for k, _ in FIELDS}
    eng = Engine(case.lf, 3, case.methods, corrections=case.corrections, averages=case.averages,
                 remaps=[remap_spec(m1, o1, s=0), remap_spec(m2, o2, s=0)],
                 options={"pipeline_min_chunk": 1024, "pipeline_chunks": 5})
    eng.step(PHASE_ALL, STEP_T)
    eng.close()
    for mm, oo in ((m1, o1), (m2, o2)):
        for name, g in FIELDS:
            want = oracle_lib.remap_apply(mm.src, mm.dst, mm.weight, np.asarray(case.lf.field[(0, g, name)]),
                                          mm.n_model)
            np.testing.assert_array_equal(oo[name], want, err_msg=name)


def test_sharded_remap_partial_sums_complete_by_summation():
    """Three engines on APPLE shards write partial sums of the whole model grid; their sum
    (the all-reduce) equals the single-engine remap up to association."""
    n, world = 24_007, 3
    full = build_case("RCO", n=n, T=1, bias=False, seed=17)
    mmap = synthetic_model_map(n, 1_000, links_per_cell=2)
    total = {k: np.zeros(mmap.n_model) for k, _ in FIELDS}
    for r in range(world):
        off, size = apple_range(n, r, world)
        case = build_case("RCO", n=size, T=1, bias=False, seed=17)
        remap_arrays = {}
        for key, a in full.lf.field.items():
            if id(a) not in remap_arrays:
                remap_arrays[id(a)] = np.ascontiguousarray(np.asarray(a)[off: off + size])
            case.lf.field[key] = remap_arrays[id(a)]
        src, dst, w = local_links(mmap, off, size)
        outs = {k: np.full(mmap.n_model, np.nan) for k, _ in FIELDS}
        eng = Engine(case.lf, 1, case.methods, remaps=[remap_spec(mmap, outs, src=src, dst=dst, w=w)])
        eng.step(PHASE_ALL, 0)
        eng.close()
        for k in total:
            total[k] += outs[k]
        for key in case.outputs:  # the shard's fluxes back into the global arrays
            np.asarray(full.lf.field[key])[off: off + size] = case.lf.field[key]
    for name, g in FIELDS:
        want = oracle_lib.remap_apply(mmap.src, mmap.dst, mmap.weight, np.asarray(full.lf.field[(1, g, name)]),
                                      mmap.n_model)
        assert mixed_error(total[name], want) <= 1e-12, name


@pytest.mark.parametrize("variant", ["CCLM", "RCO"])
def test_geometric_grid_accumulation_and_remap(variant):
    """The exchange grid of an atmosphere grid intersected with a finer ocean grid
    (fcx.parallel.geometric_maps): the fused exchange -> atmosphere accumulation (runs of 4, 6
    or 9 cells) and the conservative exchange -> ocean remap in one step, both bit-identical
    to the sequential applications on the GPU's own fluxes."""
    from fcx.parallel import geometric_maps, local_atmos

    am, mm = geometric_maps(70)
    n = am.atmos_index.size
    case = build_case(variant, n=n, T=1, bias=True)
    la = local_atmos(am, 0, 1)
    atm = {k: np.full(am.n_atmos, np.nan) for k, _ in FIELDS}
    rmo = {k: np.full(mm.n_model, np.nan) for k, _ in FIELDS}
    eng = Engine(case.lf, 1, case.methods, corrections=case.corrections,
                 atmos={"local": la, "fields": [(2, 1, g, k, atm[k]) for k, g in FIELDS]},
                 remaps=[remap_spec(mm, rmo)])
    eng.step(PHASE_ALL, STEP_T)
    eng.close()
    for name, g in FIELDS:
        flux = np.asarray(case.lf.field[(1, g, name)])
        np.testing.assert_array_equal(atm[name], oracle_lib.atmos_accumulate(am.atmos_index, am.weight, flux,
                                                                              am.n_atmos), err_msg=name)
        np.testing.assert_array_equal(rmo[name], oracle_lib.remap_apply(mm.src, mm.dst, mm.weight, flux,
                                                                         mm.n_model), err_msg=name)


@pytest.mark.parametrize("nf", [1, 3, 5, 16, 17])
@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_remap_pack_record_widths(nf, precision):
    """Packed-record gather with record widths that are not a 16-B multiple (3, 5 fields: padded
    records), a full launch group (16) and one more (17: two launches, the second of one field),
    fp64 and fp32 engines, a grid whose size is not a multiple of the pack block; every output
    equals the gather from the arrays (FCX_OPT_REMAP_PACK 0) bit for bit, and the sequential
    application of the engine's own fluxes."""
    n = 9_973
    case = build_case("MOM5", n=n, T=1, bias=False, seed=5)
    mmap = synthetic_model_map(n, 700, links_per_cell=2, seed=9)
    dt = np.float32 if precision == "f32" else np.float64
    names = [("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3)]
    fields = [names[i % len(names)] for i in range(nf)]
    if precision == "f32":
        case = as_dtype(case, "float32")
    lf = case.lf
    res = {}
    for pack in (0, 1):
        outs = [np.full(mmap.n_model, np.nan, dtype=dt) for _ in fields]
        rm = {"n_dst": mmap.n_model, "src": mmap.src, "dst": mmap.dst, "w": mmap.weight,
              "fields": [(2, 1, g, k, outs[i]) for i, (k, g) in enumerate(fields)]}
        eng = Engine(lf, 1, case.methods, remaps=[rm], options={"remap_pack": pack})
        eng.step(PHASE_ALL, 0)
        eng.close()
        res[pack] = outs
        for i, (k, g) in enumerate(fields):
            flux = np.asarray(lf.field[(1, g, k)], dtype=np.float64)
            want = oracle_lib.remap_apply(mmap.src, mmap.dst, mmap.weight, flux, mmap.n_model)
            np.testing.assert_array_equal(outs[i], want.astype(dt), err_msg=f"{k} pack={pack}")
    for i in range(nf):
        np.testing.assert_array_equal(res[0][i], res[1][i])


def test_remap_pack_auto_follows_the_map_scatter():
    """FCX_OPT_REMAP_PACK auto: the shuffled 2-link map (about 0.66 distinct field segments per
    link) gathers packed records, the geometric intersection map (about 0.3: a model cell's
    links come from neighbouring cells) gathers from the arrays; a one-field remap never packs.
    Both give the sequential application's bits."""
    from fcx.parallel import geometric_maps

    _, geo = geometric_maps(200)
    n = geo.src.size
    case = build_case("CCLM", n=n, T=1, bias=False, seed=3)
    shuf = synthetic_model_map(n, n // 4, links_per_cell=2, seed=4)
    outs = [{k: np.full(mm.n_model, np.nan) for k, _ in FIELDS} for mm in (shuf, geo)]
    one = np.full(shuf.n_model, np.nan)
    remaps = [remap_spec(shuf, outs[0]), remap_spec(geo, outs[1]),
              {"n_dst": shuf.n_model, "src": shuf.src, "dst": shuf.dst, "w": shuf.weight,
               "fields": [(2, 1, 1, "HLAT", one)]}]
    eng = Engine(case.lf, 1, case.methods, remaps=remaps)
    info = [eng.remap_info(i) for i in range(3)]
    eng.step(PHASE_ALL, 0)
    eng.close()
    assert info[0][1] == 1 and info[0][0] > 0.5, info
    assert info[1][1] == 0 and info[1][0] < 0.5, info
    assert info[2][1] == 0, info
    for mm, oo in zip((shuf, geo), outs):
        for name, g in FIELDS:
            want = oracle_lib.remap_apply(mm.src, mm.dst, mm.weight, np.asarray(case.lf.field[(1, g, name)]),
                                          mm.n_model)
            np.testing.assert_array_equal(oo[name], want, err_msg=name)
    np.testing.assert_array_equal(one, oracle_lib.remap_apply(shuf.src, shuf.dst, shuf.weight,
                                                              np.asarray(case.lf.field[(1, 1, "HLAT")]), shuf.n_model))


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
@pytest.mark.parametrize("atmos", [False, True])
@pytest.mark.parametrize("host", ["device", "pipelined"])
def test_remap_records_from_the_flux_launch(variant, atmos, host):
    """T=1: the records of a remap of type-1 fluxes are written by the flux kernel itself
    (fcx_remap_info packed == 2, no packing pass), alone or beside the fused atmosphere
    accumulation, HBM-resident or in the pipelined host step; a second remap of the same fields
    (one record buffer per plan) and a remap with a field the kernel does not hold (TSUR) take
    the packing pass.  Every output equals the sequential application of the engine's own
    fluxes, bit for bit."""
    torch = pytest.importorskip("torch")
    from fcx.parallel import local_atmos, synthetic_atmos_map

    n = 70_001
    dev = torch.device("cuda", 0)
    case = build_case(variant, n=n, T=1, bias=True, seed=11, device=dev if host == "device" else None)
    shuf = synthetic_model_map(n, n // 4, links_per_cell=2, seed=12)
    names = [k for k in FIELDS if not (variant == "RCO" and k[0] == "QSUR")]
    outs = [{k: np.full(shuf.n_model, np.nan) for k, _ in names} for _ in range(2)]
    ts_out = {"HSEN": np.full(shuf.n_model, np.nan), "TSUR": np.full(shuf.n_model, np.nan)}
    remaps = [remap_spec(shuf, outs[0]), remap_spec(shuf, outs[1]),
              {"n_dst": shuf.n_model, "src": shuf.src, "dst": shuf.dst, "w": shuf.weight,
               "fields": [(2, 1, 1, "HSEN", ts_out["HSEN"]), (2, 1, 1, "TSUR", ts_out["TSUR"])]}]
    kw = {}
    if atmos:
        amap = synthetic_atmos_map(n)
        atm = {k: np.full(amap.n_atmos, np.nan) for k, _ in names}
        kw["atmos"] = {"local": local_atmos(amap, 0, 1), "fields": [(2, 1, g, k, atm[k]) for k, g in names]}
    opts = {"pipeline_min_chunk": 8192} if host == "pipelined" else {}
    eng = Engine(case.lf, 1, case.methods, corrections=case.corrections, remaps=remaps, options=opts, **kw)
    eng.step(PHASE_ALL, STEP_T)
    info = [eng.remap_info(i)[1] for i in range(3)]
    eng.close()
    assert info == [2, 1, 1], info

    def flux(k, g):
        a = case.lf.field[(1, g, k)]
        return a.cpu().numpy() if hasattr(a, "cpu") else np.asarray(a)

    for oo in outs:
        for name, g in names:
            want = oracle_lib.remap_apply(shuf.src, shuf.dst, shuf.weight, flux(name, g), shuf.n_model)
            np.testing.assert_array_equal(oo[name], want, err_msg=name)
    for name in ("HSEN", "TSUR"):
        want = oracle_lib.remap_apply(shuf.src, shuf.dst, shuf.weight, flux(name, 1), shuf.n_model)
        np.testing.assert_array_equal(ts_out[name], want, err_msg=name)
    if atmos:
        for name, g in names:
            want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, flux(name, g), amap.n_atmos)
            np.testing.assert_array_equal(atm[name], want, err_msg=f"atmos {name}")


@pytest.mark.parametrize("change", [("specialize", 0), ("cells_per_thread", 1)])
def test_launch_options_changed_after_runs(change):
    """A remap engine whose records the T=1 flux launch writes (specialize=1, two cells per
    lane): switching the launch options after runs drops the cached plans, so the next run
    takes the generic kernel and the packing pass with the same bits, and switching back
    returns to the records."""
    n = 30_011
    case = build_case("CCLM", n=n, T=1, bias=True)
    mmap = synthetic_model_map(n, 2_000, links_per_cell=2)
    outs = {k: np.full(mmap.n_model, np.nan) for k, _ in FIELDS}
    eng = Engine(case.lf, 1, case.methods, corrections=case.corrections, remaps=[remap_spec(mmap, outs)],
                 options={"remap_pack": 1})
    res = []
    for setting in (None, change[1], 1 if change[0] == "specialize" else 2):
        if setting is not None:
            eng.set_option(change[0], setting)
        for o in outs.values():
            o[:] = np.nan
        eng.step(PHASE_ALL, STEP_T)
        res.append(({k: o.copy() for k, o in outs.items()}, eng.remap_info(0)[1]))
    eng.close()
    assert [p for _, p in res] == [2, 1, 2]  # records from the flux launch / packing pass / flux launch
    for got, _ in res[1:]:
        for k in outs:
            np.testing.assert_array_equal(got[k], res[0][0][k], err_msg=k)
    for name, g in FIELDS:
        want = oracle_lib.remap_apply(mmap.src, mmap.dst, mmap.weight, np.asarray(case.lf.field[(1, g, name)]),
                                      mmap.n_model)
        np.testing.assert_array_equal(res[0][0][name], want, err_msg=name)
