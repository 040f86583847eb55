"""Tile-blocked device mirrors (FCX_OPT_TILED_LAYOUT, the default for engine-owned mirrors):
every path that touches a field buffer -- the fused flux kernels, the generic kernel with
separate u/v grids and type-0 averages, the pipelined chunk copies (2-D copies of whole
tiles, 1-D copies of partial ones), the fused and the separate atmosphere accumulation,
do_regridding and the exchange->model remaps, the fp32 engine -- must give exactly the bits
of the contiguous layout, and those are within tests/parity.py of the oracle.  Grid sizes
are not multiples of the 4096-cell tile, so partial tiles are always exercised."""
import ctypes

import numpy as np
import pytest

import oracle_lib
from parity import assert_parity

pytestmark = pytest.mark.gpu

from fcx import _lib  # noqa: E402
from fcx.basic import IDX, PHASE_ALL, PHASE_EARLY, PHASE_NORMAL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.parallel import local_atmos, synthetic_atmos_map, synthetic_model_map  # noqa: E402
from fcx.synthetic import as_dtype, build_case  # noqa: E402

STEP_T = 3600 * 24 * 40
TILE = 4096


ATM = (("MEVA", 1), ("HSEN", 1), ("UMOM", 2))


def run(case, options, atmos_n=None, remap=None, phases=(PHASE_ALL,), check_layout=None, atm=ATM):
    """Steps of a host-bound engine (no zero-copy, so the engine owns its mirrors); returns
    the outputs, the atmosphere and remap outputs."""
    for k in case.outputs:
        case.lf.field[k][:] = np.nan
    dt = np.float32 if getattr(case.lf, "dtype", "float64") == "float32" else np.float64
    atmos, outs, rspec, routs = None, {}, None, {}
    if atmos_n is not None:
        amap = synthetic_atmos_map(atmos_n)
        outs = {name: np.full(amap.n_atmos, np.nan, dtype=dt) for name, _ in atm}
        atmos = {"local": local_atmos(amap, 0, 1), "fields": [(2, 1, g, name, outs[name]) for name, g in atm]}
    if remap is not None:
        routs = {name: np.full(remap.n_model, np.nan, dtype=dt) for name in ("MEVA", "VMOM")}
        rspec = [{"n_dst": remap.n_model, "src": remap.src, "dst": remap.dst, "w": remap.weight,
                  "fields": [(2, 1, 1, "MEVA", routs["MEVA"]), (2, 1, 3, "VMOM", routs["VMOM"])]}]
    options = {"zero_copy": 0, "pipeline_min_chunk": 1024, **options}
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, regrid=case.regrid, atmos=atmos, remaps=rspec, options=options)
    tile, stride = eng.device_layout()
    assert tile == TILE
    if check_layout is not None:
        assert (stride > tile) == check_layout, (tile, stride)
    for ph in phases:
        eng.step(ph, STEP_T)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    got.update({("atm", k): v.copy() for k, v in outs.items()})
    got.update({("remap", k): v.copy() for k, v in routs.items()})
    return got


def same_bits(a, b):
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=str(k))


def fluxes(got, case):
    return {k: got[k] for k in case.outputs}


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
def test_fused_t1_with_accumulation(variant):
    n = 70_001
    case = build_case(variant, n=n, T=1, bias=True)
    plain = run(case, {"tiled_layout": 0, "pipeline_chunks": 1}, atmos_n=n, check_layout=False)
    seq = run(case, {"pipeline_chunks": 1}, atmos_n=n, check_layout=True)
    same_bits(seq, plain)
    for chunks in (3, 8):  # chunks of whole tiles (2-D copies) plus the partial last tile
        same_bits(run(case, {"pipeline_chunks": chunks}, atmos_n=n), plain)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(fluxes(seq, case), ref, label=f"{variant} tiled")


def test_generic_separate_grids_averages_and_separate_accumulation():
    case = build_case("CCLM", n=20_011, T=3, sep_grids=(19_997, 20_101), bias=True)
    atm = ATM[:2]  # the accumulation takes t-grid fields only
    plain = run(case, {"tiled_layout": 0, "pipeline_chunks": 1}, atmos_n=20_011, atm=atm)
    same_bits(run(case, {"pipeline_chunks": 1}, atmos_n=20_011, check_layout=True, atm=atm), plain)
    same_bits(run(case, {"pipeline_chunks": 5}, atmos_n=20_011, atm=atm), plain)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(fluxes(plain, case), ref, label="T3 sep tiled")


def test_regridding_staged_across_tiles():
    """do_regridding (basic:463-522) on tiled buffers: gathers and the zeroed destination
    span several tiles."""
    rng = np.random.default_rng(11)
    case = build_case("CCLM", n=9_001, T=2, bias=False, sep_grids=(8_503, 8_209))
    nt, nu, nv = case.grid_size
    mats = {}
    for which, (ns, nd) in {2: (nt, nu), 3: (nt, nv)}.items():
        nnz = 3 * nd
        mats[which] = (rng.integers(1, ns + 1, nnz), np.repeat(np.arange(1, nd + 1), 3)[rng.permutation(nnz)],
                       rng.uniform(0.0, 1.0, nnz))
    case.regrid = {"matrices": mats}
    for s in (1, 2):
        case.methods["which_spec_vapor_surface_u"][s - 1] = "none"
        case.lf.put_to[(s, 1, "QSUR")] = 2
        case.lf.put_to[(s, 1, "MEVA")] = 4
        case.lf.allocate_localvar("MEVA", s, 3, value=np.nan)
        case.outputs.append((s, 3, "MEVA"))
    phases = (PHASE_EARLY, PHASE_NORMAL)
    plain = run(case, {"tiled_layout": 0}, phases=phases)
    got = run(case, {}, phases=phases, check_layout=True)
    same_bits(got, plain)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T, regrid=True)
    assert_parity(got, ref, label="regrid tiled")


def test_remap_tiled_sources():
    n = 30_011
    case = build_case("MOM5", n=n, T=1, bias=True)
    mmap = synthetic_model_map(n, 2_000, links_per_cell=2)
    got = run(case, {}, remap=mmap, check_layout=True)
    same_bits(got, run(case, {"tiled_layout": 0}, remap=mmap))
    for name, g in (("MEVA", 1), ("VMOM", 3)):
        want = oracle_lib.remap_apply(mmap.src, mmap.dst, mmap.weight, got[(1, g, name)], mmap.n_model)
        np.testing.assert_array_equal(got[("remap", name)], want, err_msg=name)


@pytest.mark.parametrize("variant", ["CCLM", "RCO"])
def test_fp32_engine(variant):
    case = as_dtype(build_case(variant, n=50_003, T=1, bias=True), "float32")
    plain = run(case, {"tiled_layout": 0, "pipeline_chunks": 1}, atmos_n=50_003)
    same_bits(run(case, {"pipeline_chunks": 4}, atmos_n=50_003, check_layout=True), plain)


def test_device_layout_places_cells_by_tile():
    """Cell j of a mirror is element (j // tile) * stride + j % tile of its device buffer."""
    n = 3 * TILE + 123
    case = build_case("CCLM", n=n, T=1, bias=False)
    eng = Engine(case.lf, 1, case.methods, options={"zero_copy": 0})
    eng.upload(PHASE_ALL)
    eng.synchronize()
    tile, stride = eng.device_layout()
    assert stride > tile == TILE
    lib = _lib.load()
    for name in ("TSUR", "UATM"):
        host = np.asarray(case.lf.field[(1, 1, name)])
        base = eng.device_ptr(1, 1, name)
        for t in range(4):
            m = min(tile, n - t * tile)
            buf = np.empty(m)
            _lib.check(lib.fcx_memcpy(ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(base + t * stride * 8),
                                      m * 8, 2))
            np.testing.assert_array_equal(buf, host[t * tile: t * tile + m], err_msg=f"{name} tile {t}")
    eng.close()
    assert IDX["TSUR"] > 0
