"""GPU parity: libfcx (HIP, gfx950) against the CPU oracle on the same seeded inputs.

All calls go through the C ABI (include/fcx.h) via ctypes.  Tolerance: SURVEY.md 8d,
written in tests/parity.py (1e-10 mixed abs/rel per field, fp64).  The oracle is the C
restatement (oracle/fco.c), itself pinned bit-exactly to the reference flux_lib by
tests/test_oracle_golden.py.
"""
import numpy as np
import pytest

import oracle_lib
from parity import assert_parity, cell_report, conditioned_full, write_report

pytestmark = pytest.mark.gpu

fcx = pytest.importorskip("fcx")
from fcx.basic import PHASE_ALL, PHASE_EARLY, PHASE_NORMAL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.synthetic import build_case  # noqa: E402
from fcx import flux_calculator_calculate as fcc  # noqa: E402

STEP_T = 3600 * 24 * 31  # inside February of 1961: month 2 bias slice


def engine_for(case, **kw):
    return Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                  averages=case.averages, regrid=case.regrid, **kw)


def outputs(case):
    return {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}


def fused(case, t=STEP_T, phases=(PHASE_ALL,)):
    eng = engine_for(case)
    for ph in phases:
        eng.step(ph, t)
    got = outputs(case)
    eng.close()
    return got


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("n", [1, 2, 3, 4097])
def test_fused_t1(variant, bias, n):
    case = build_case(variant, n=n, T=1, bias=bias)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(fused(case), ref, label=case.name)


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
@pytest.mark.parametrize("zero_copy", [0, 1])
def test_fused_t1_host_modes(variant, zero_copy):
    """Host-bound fields through device mirrors (copies) and, for arrays allocated by
    fcx_host_malloc, through zero-copy mapping (FCX_OPT_ZERO_COPY=1): same oracle parity."""
    from fcx.host_alloc import Arena

    case = build_case(variant, n=10_007, T=1, bias=True)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    arena = Arena()
    if zero_copy:
        arena.adopt(case.lf)
    eng = engine_for(case, options={"zero_copy": zero_copy})
    assert eng.zero_copy_active() == bool(zero_copy)
    eng.step(PHASE_ALL, STEP_T)
    got = outputs(case)
    eng.close()
    arena.close()
    assert_parity(got, ref, label=f"{case.name} zero_copy={zero_copy}")


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
def test_fused_t3_averages(variant):
    case = build_case(variant, n=3001, T=3, bias=True)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(fused(case), ref, label=case.name)


def test_fused_ten_surface_types():
    case = build_case("MOM5", n=777, T=10, bias=True)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(fused(case), ref, label=case.name)


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
def test_separate_uv_grids(variant):
    case = build_case(variant, n=2049, T=2, bias=False, sep_grids=(2101, 1999))
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(fused(case), ref, label=case.name)


@pytest.mark.parametrize("T", [1, 3])
def test_zero_momentum_on_separate_grids(T):
    """'zero' momentum on separate u/v grids (prepare binds no wind for it): the u/v pass
    must not read the unbound wind arrays (found by tests/test_gpu_random_configs.py, seed 6:
    the kernel loaded through a null pointer and faulted)."""
    case = build_case("MOM5", n=4095, T=T, bias=False, sep_grids=(4097, 4097),
                      per_type={1: dict(which_flux_momentum="zero")})
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(fused(case), ref, label=case.name)


def test_early_then_normal_phase():
    case = build_case("CCLM", n=1500, T=3, bias=True)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(fused(case, phases=(PHASE_EARLY, PHASE_NORMAL)), ref, label=case.name)


@pytest.mark.parametrize("per_type", [
    {2: dict(which_flux_mass_evap="copy", which_flux_heat_latent="water")},
    {2: dict(which_flux_mass_evap="zero", which_flux_heat_sensible="zero",
             which_flux_momentum="zero", which_flux_radiation_blackbody="zero")},
    {3: dict(which_flux_mass_evap="copy", which_flux_heat_latent="copy",
             which_flux_heat_sensible="copy", which_flux_momentum="copy",
             which_flux_radiation_blackbody="copy", which_spec_vapor_surface_t="copy",
             which_spec_vapor_surface_u="copy", which_spec_vapor_surface_v="copy")},
    {1: dict(which_flux_mass_evap="RCO"), 2: dict(which_flux_heat_sensible="RCO")},
])
def test_method_edges(per_type):
    """zero / copy (bias added once more per aliased copy, calc:112-116) / mixed methods."""
    case = build_case("CCLM", n=1025, T=3, bias=True, per_type=per_type)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(fused(case), ref, label=str(per_type))


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
@pytest.mark.parametrize("T", [1, 3])
def test_shortwave_distribution(variant, T):
    """distribute_shortwave_radiation_flux (calc:347-364, flux_calculator.F90:991): with
    RSDD/ALBA bound every surface type's RSDR is the type-0 RSDD (the albedo factors are
    commented out in distribute_radiation_flux.F90:24), inside the fused step."""
    case = build_case(variant, n=4099, T=T, bias=True, rsdr=True)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    got = fused(case)
    assert_parity(got, ref, label=case.name)
    rsdd = np.asarray(case.lf.field[(0, 1, "RSDD")])
    for s in range(1, T + 1):
        np.testing.assert_array_equal(got[(s, 1, "RSDR")], rsdd, err_msg=f"RSDR({s})")


def test_per_call_dropin_sequence():
    """The reference subroutines one by one (calc:25-385) through the C ABI."""
    case = build_case("MOM5", n=2500, T=3, bias=True, rsdr=True)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    fcc.prepare(case.lf, 1, case.num_surface_types, case.methods, corrections=case.corrections)
    m = fcc.methods_2d(case.methods)
    T, gs, lf = case.num_surface_types, case.grid_size, case.lf
    fcc.calc_flux_radiation_blackbody(1, T, m["which_flux_radiation_blackbody"], gs, lf)
    for name, g in (("RBBR", 1), ("TSUR", 1)):
        fcc.average_across_surface_types(g, name, T, gs, lf)
    for g, tab in ((1, "which_spec_vapor_surface_t"), (2, "which_spec_vapor_surface_u"),
                   (3, "which_spec_vapor_surface_v")):
        fcc.calc_spec_vapor_surface(1, T, g, m[tab], gs, lf)
    fcc.calc_flux_mass_evap(1, T, m["which_flux_mass_evap"], gs, lf, current_step_time=STEP_T)
    fcc.calc_flux_heat_latent(1, T, m["which_flux_heat_latent"], gs, lf)
    fcc.calc_flux_heat_sensible(1, T, m["which_flux_heat_sensible"], gs, lf)
    fcc.calc_flux_momentum_east(1, T, 2, m["which_flux_momentum"], gs, lf)
    fcc.calc_flux_momentum_north(1, T, 3, m["which_flux_momentum"], gs, lf)
    fcc.distribute_shortwave_radiation_flux(1, T, gs, lf)
    for name, g in (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("UMOM", 2), ("VMOM", 3)):
        fcc.average_across_surface_types(g, name, T, gs, lf)
    got = outputs(case)
    fcc.release(lf)
    assert_parity(got, ref, label="per-call")


def test_bias_month_boundary():
    """Steps that cross a month boundary pick the right corrections slice."""
    for t in (0, 2678399, 2678400, 3600 * 24 * 59):
        case = build_case("CCLM", n=999, T=1, bias=True)
        ref = oracle_lib.run_case(case, "c", current_step_time=t)
        assert_parity(fused(case, t=t), ref, label=f"t={t}")


def test_regridding_staged():
    """do_regridding (basic:463-522) after each calc: QSUR t->u and MEVA t->v."""
    rng = np.random.default_rng(7)
    case = build_case("CCLM", n=600, T=2, bias=False, sep_grids=(550, 520))
    nt, nu, nv = case.grid_size
    mats = {}
    for which, (ns, nd) in {2: (nt, nu), 3: (nt, nv)}.items():
        nnz = 3 * nd
        mats[which] = (rng.integers(1, ns + 1, nnz), np.repeat(np.arange(1, nd + 1), 3)[rng.permutation(nnz)],
                       rng.uniform(0.0, 1.0, nnz))
    case.regrid = {"matrices": mats}
    for s in (1, 2):
        # QSUR on u is regridded from t instead of computed; MEVA lands on v too
        case.methods["which_spec_vapor_surface_u"][s - 1] = "none"
        case.lf.put_to[(s, 1, "QSUR")] = 2
        case.lf.put_to[(s, 1, "MEVA")] = 4
        case.lf.allocate_localvar("MEVA", s, 3, value=np.nan)
        case.outputs.append((s, 3, "MEVA"))
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T, regrid=True)
    got = fused(case, phases=(PHASE_EARLY, PHASE_NORMAL))
    assert_parity(got, ref, label="regrid")


def test_device_resident_zero_copy():
    """Fields bound as device memory (torch, FCX_MEM_DEVICE): no host staging."""
    torch = pytest.importorskip("torch")
    case_h = build_case("MOM5", n=4099, T=1, bias=True)
    ref = oracle_lib.run_case(case_h, "c", current_step_time=STEP_T)
    case = build_case("MOM5", n=4099, T=1, bias=True, device="cuda:0")
    eng = engine_for(case)
    eng.run(PHASE_ALL, STEP_T)
    eng.synchronize()
    got = {k: case.lf.to_numpy(*k) for k in case.outputs}
    eng.close()
    assert_parity(got, ref, label="device")
    del torch


def test_unaligned_device_pointers_use_scalar_path():
    torch = pytest.importorskip("torch")
    case_h = build_case("CCLM", n=1001, T=1, bias=False)
    ref = oracle_lib.run_case(case_h, "c", current_step_time=STEP_T)
    case = build_case("CCLM", n=1001, T=1, bias=False, device="cuda:0")
    # shift every array by one element (8-B aligned, not 16-B)
    shifted = {}
    for key, a in list(case.lf.field.items()):
        if id(a) not in shifted:
            b = torch.empty(a.shape[0] + 1, dtype=torch.float64, device="cuda:0")[1:]
            b.copy_(a)
            shifted[id(a)] = b
        case.lf.field[key] = shifted[id(a)]
    eng = engine_for(case)
    eng.run(PHASE_ALL, STEP_T)
    eng.synchronize()
    got = {k: case.lf.to_numpy(*k) for k in case.outputs}
    eng.close()
    assert_parity(got, ref, label="unaligned")


def test_large_grid_full():
    """10M cells (config 3 size), bias on: every cell of every output against the oracle
    over the whole grid (fco_step_threads on the host cores), all outputs finite."""
    n = 10_000_000
    case = build_case("CCLM", n=n, T=1, bias=True)
    got = fused(case)
    ref = oracle_lib.run_case_threads(case, current_step_time=STEP_T)
    rep = cell_report(got, ref)
    cond = conditioned_full(case, got, ref, STEP_T, "10M full grid")  # (the allowance: tests/parity.py)
    for k, v in cond.items():
        rep[k]["conditioned"] = v
    write_report("large_grid_cclm_bias", rep)
    for k, v in got.items():
        assert np.isfinite(v).all(), k


def _golden_cases():
    import test_oracle_golden as tg

    return tg.CASES


@pytest.mark.parametrize("stem", _golden_cases())
def test_golden_reference_outputs(stem):
    """libfcx against the REFERENCE flux_lib's own outputs (tests/golden, 1e-10 mixed)."""
    import test_oracle_golden as tg

    case, data, spec = tg.load_case(stem)
    ref = {(int(k.split(":")[0]), int(k.split(":")[1]), k.split(":")[2]): data[f"out:{k}"]
           for k in spec["outputs"]}
    got = fused(case, t=tg.MANIFEST["step_time"], phases=(PHASE_EARLY, PHASE_NORMAL))
    assert_parity(got, ref, label=stem)


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
def test_fp64_tolerance_report_config5(variant):
    """SURVEY.md 8d tolerance row: per field the mixed error (the gate), the plain elementwise
    max relative error, the count of cells above 1e-10 and error percentiles, on config 5
    (bias on, 32,768 cells, a step in February).  Written to gpurun_out/ for profiles/."""
    import json
    import os

    n = 32_768
    case = build_case(variant, n=n, T=1, bias=True)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    got = fused(case)
    worst = assert_parity(got, ref, label=case.name)
    rep = {}
    for key, r in ref.items():
        g = np.asarray(got[key])
        nz = np.abs(r) > 0
        rel = np.zeros_like(r)
        rel[nz] = np.abs(g[nz] - r[nz]) / np.abs(r[nz])
        rep["%d:%d:%s" % key] = {"mixed": worst[key], "max_rel": float(rel.max()),
                                 "cells_rel_gt_1e-10": int((rel > 1e-10).sum()),
                                 "p50_rel": float(np.percentile(rel, 50)), "p99_rel": float(np.percentile(rel, 99)),
                                 "bit_identical_cells": int((g == r).sum()), "cells": int(r.size)}
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"fp64_error_{variant}.json"), "w") as f:
        json.dump(rep, f, indent=1)


@pytest.mark.parametrize("quirk", [False, True])
def test_bias_window_of_rank_range(quirk):
    """Corrections of rank 1 of 2 cut from a global field by fcx.bias.window (intended, or the
    reference's one-cell-early read, P5), passed month-major [12][n]: same as the oracle fed
    with the same window."""
    from fcx.bias import window
    from fcx.parallel import apple_range

    n_global = 10_000
    off, n = apple_range(n_global, 1, 2)
    g = np.random.default_rng(5).normal(0.0, 1e-5, (12, n_global))
    w = window(g, off, n, reference_offset_quirk=quirk)
    np.testing.assert_array_equal(w, g[:, off - 1: off - 1 + n] if quirk else g[:, off: off + n])
    case = build_case("CCLM", n=n, T=1, bias=True)
    case.corrections = (case.corrections[0], np.ascontiguousarray(w.T))  # oracle: cell-major
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    eng = Engine(case.lf, 1, case.methods, corrections=(case.corrections[0], w))  # month-major
    eng.step(PHASE_ALL, STEP_T)
    got = outputs(case)
    eng.close()
    assert_parity(got, ref, label=f"bias window quirk={quirk}")


def test_regridding_matrices_read_from_files(tmp_path):
    """The staged regrid path with links read back by fcx.io.read_regridding_matrix from
    NetCDF-3 files (io:109-198), t->u and t->v, against the oracle on the same links."""
    from scipy.io import netcdf_file

    from fcx.io import read_regridding_matrix

    rng = np.random.default_rng(11)
    case = build_case("MOM5", n=700, T=2, bias=True, sep_grids=(640, 610))
    nt, nu, nv = case.grid_size
    mats = {}
    for which, (ns, nd, fname) in {2: (nt, nu, "t_to_u"), 3: (nt, nv, "t_to_v")}.items():
        nnz = 4 * nd
        src = rng.integers(1, ns + 1, nnz)
        dst = np.repeat(np.arange(1, nd + 1), 4)[rng.permutation(nnz)]
        w = rng.uniform(0.0, 1.0, nnz)
        path = str(tmp_path / f"regrid_{fname}.nc")
        with netcdf_file(path, "w") as f:
            f.createDimension("num_links", nnz)
            f.createDimension("num_wgts", 1)
            for name, vals, typ in (("src_address", src, "i"), ("dst_address", dst, "i")):
                v = f.createVariable(name, typ, ("num_links",))
                v[:] = vals.astype(np.int32)
            m = f.createVariable("remap_matrix", "d", ("num_links", "num_wgts"))
            m[:] = w[:, None]
        mats[which] = read_regridding_matrix(path, ns, 0, nd, 0)
    case.regrid = {"matrices": mats}
    for s in (1, 2):
        case.methods["which_spec_vapor_surface_u"][s - 1] = "none"
        case.lf.put_to[(s, 1, "QSUR")] = 2
        case.lf.put_to[(s, 1, "HSEN")] = 4
        case.lf.allocate_localvar("HSEN", s, 3, value=np.nan)
        case.outputs.append((s, 3, "HSEN"))
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T, regrid=True)
    assert_parity(fused(case, phases=(PHASE_EARLY, PHASE_NORMAL)), ref, label="regrid from files")
