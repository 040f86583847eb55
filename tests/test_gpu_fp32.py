"""fp32 variant of the cell pass ("fp32 and fp64 kernels ... report
max/percentile error vs oracle").  The fp32 engine (FCX_PRECISION_F32) stores and computes
in float; its outputs are compared with the fp64 oracle run on the SAME inputs (the float32
arrays widened exactly), so the reported error is the error of fp32 arithmetic alone.
Gate: tests/parity.py FP32_NORM_GATE on the norm-wise error (report, not a parity claim);
fp64 parity is tests/test_gpu_parity.py."""
import json
import os

import numpy as np
import pytest

import oracle_lib
from parity import FP32_NORM_GATE, error_report

pytestmark = pytest.mark.gpu

from fcx.basic import PHASE_ALL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.synthetic import as_dtype, build_case  # noqa: E402

STEP_T = 3600 * 24 * 31
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def run_fp32(case, options=None):
    c32 = as_dtype(case, "float32")
    c64 = as_dtype(c32, "float64")  # exactly the inputs the fp32 kernel saw
    ref = oracle_lib.run_case(c64, "c", current_step_time=STEP_T)
    eng = Engine(c32.lf, c32.num_surface_types, c32.methods, corrections=c32.corrections,
                 averages=c32.averages, options=options)
    eng.step(PHASE_ALL, STEP_T)
    got = {k: np.array(c32.lf.field[k], dtype=np.float64) for k in c32.outputs}
    eng.close()
    for k in c32.outputs:
        assert c32.lf.field[k].dtype == np.float32
    return got, ref


def check(got, ref, label):
    rep = error_report(got, ref)
    bad = {k: v for k, v in rep.items() if not v[0] <= FP32_NORM_GATE}
    assert not bad, f"{label}: fp32 norm-wise error over {FP32_NORM_GATE}: {bad}"
    return rep


EPS32 = float(np.finfo(np.float32).eps)
# the fp32 kernel's own arithmetic, gated cell by cell (config 5): within 64 fp32 ulps of the
# fp64 oracle fed the SAME fp32-rounded inputs (mixed scale, tests/parity.py), or -- where the
# flux cancels (HSEN's T_s - T_a EF, MEVA's q_s - q_a) -- within 4x the oracle's own movement
# when those inputs are perturbed by 16 fp32 ulps: 64 ulps scaled by the cell's conditioning
ULPS_GATE, PERTURB_ULPS = 64, 16


def perturbation_movement(c64, t, ulps=PERTURB_ULPS, trials=8):
    """max over seeded trials of |oracle(inputs * (1 +- ulps * eps32)) - oracle(inputs)| per cell"""
    base = oracle_lib.run_case(c64, "c", current_step_time=t)
    move = {k: np.zeros(np.shape(v)) for k, v in base.items()}
    for trial in range(trials):
        c = as_dtype(as_dtype(c64, "float32"), "float64")  # a fresh copy (the inputs are fp32 values)
        outs = {id(c.lf.field[k]) for k in c.outputs}  # (the copy's own output arrays stay unperturbed)
        rng = np.random.default_rng([trial, 32])
        seen = set()
        for a in c.lf.field.values():
            if id(a) in outs or id(a) in seen or not isinstance(a, np.ndarray) or a.dtype != np.float64:
                continue
            seen.add(id(a))
            a *= 1.0 + ulps * EPS32 * rng.choice([-1.0, 1.0], a.shape)
        rp = oracle_lib.run_case(c, "c", current_step_time=t)
        for k in move:
            move[k] = np.fmax(move[k], np.abs(np.asarray(rp[k]) - np.asarray(base[k])))
    return move


def column(got, ref):
    out = {}
    for key, (norm, mixed, rel) in error_report(got, ref).items():
        out["%d:%d:%s" % key] = {"norm": norm, "mixed": mixed, "max_rel": rel}
    return out


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
@pytest.mark.parametrize("n", [1, 3, 4099, 32_768])
def test_fp32_t1_bias(variant, n):
    """T=1 specialised fp32 kernels (4 cells per lane, 16-B loads), ragged tails.  At the
    config-5 size the report separates input rounding from the kernel's
    arithmetic -- per field, against the fp64 reference:
      fp32_kernel_vs_fp64_original_inputs : what a user of the fp32 engine sees;
      fp32_kernel_vs_fp64_rounded_inputs  : the kernel's own arithmetic (the oracle fed the
                                            fp32-rounded inputs), gated cell by cell below;
      input_rounding_only                 : fp64 oracle on the rounded inputs vs on the original."""
    case = build_case(variant, n=n, T=1, bias=True)
    got, ref = run_fp32(case)
    rep = check(got, ref, f"{variant} n={n}")
    if n != 32_768:
        return
    ref_orig = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    c64 = as_dtype(as_dtype(case, "float32"), "float64")
    move = perturbation_movement(c64, STEP_T)
    gate, bad = {}, []
    for key, r in ref.items():
        g, r = np.asarray(got[key], dtype=np.float64), np.asarray(r, dtype=np.float64)
        top = float(np.max(np.abs(r))) if r.size else 0.0
        scale = np.maximum(np.abs(r), 1e-6 * top)
        err = np.abs(g - r)
        allow = np.maximum(ULPS_GATE * EPS32 * scale, 4.0 * move[key])
        over_ulps = int(np.sum(err > ULPS_GATE * EPS32 * scale))
        with np.errstate(divide="ignore", invalid="ignore"):
            ratio = float(np.max(np.where(allow > 0, err / allow, 0.0)))
        gate["%d:%d:%s" % key] = {"cells_over_64_ulps": over_ulps, "max_err_over_allowance": ratio,
                                  "cells": int(r.size)}
        if np.any(err > allow):
            bad.append(f"{key}: {int(np.sum(err > allow))} cells, max err/allowance {ratio:.3g}")
    report = {"fp32_kernel_vs_fp64_original_inputs": column(got, ref_orig),
              "fp32_kernel_vs_fp64_rounded_inputs": column(got, ref),
              "input_rounding_only": column(ref, ref_orig),
              "kernel_gate": gate,
              "kernel_gate_rule": f"|x - ref| <= max({ULPS_GATE} eps32 max(|ref|, 1e-6 |ref|_inf), 4 x the oracle's "
                                  f"movement under {PERTURB_ULPS}-ulp fp32 input perturbations), ref = fp64 oracle "
                                  "on the fp32-rounded inputs"}
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"fp32_error_{variant}.json"), "w") as f:
        json.dump(report, f, indent=1)
    assert not bad, f"{variant}: fp32 kernel arithmetic over its gate: {bad}"
    assert rep is not None


@pytest.mark.parametrize("variant", ["CCLM", "RCO"])
def test_fp32_generic_t3_averages(variant):
    """Generic (VAR 0) fp32 kernel with surface types and type-0 averages."""
    got, ref = run_fp32(build_case(variant, n=3001, T=3, bias=True))
    check(got, ref, f"{variant} T=3")


def test_fp32_separate_grids():
    got, ref = run_fp32(build_case("MOM5", n=2003, T=2, sep_grids=(1999, 2011), bias=True))
    check(got, ref, "MOM5 separate u/v grids")


def test_fp32_one_cell_per_lane():
    got, ref = run_fp32(build_case("CCLM", n=1001, T=1, bias=True), options={"cells_per_thread": 1})
    check(got, ref, "CCLM cells_per_thread=1")


def test_fp32_device_resident_bytes_halved():
    """The fp32 engine moves half the bytes of the fp64 one for the same case."""
    torch = pytest.importorskip("torch")
    case = build_case("CCLM", n=10_000, T=1, bias=True, device="cuda:0")
    e64 = Engine(case.lf, 1, case.methods, corrections=case.corrections)
    b64 = e64.algorithmic_bytes(PHASE_ALL)
    e64.close()
    c32 = as_dtype(case, "float32")
    assert c32.lf.field[(1, 1, "TSUR")].dtype == torch.float32
    e32 = Engine(c32.lf, 1, c32.methods, corrections=c32.corrections)
    b32 = e32.algorithmic_bytes(PHASE_ALL)
    e32.run(PHASE_ALL, STEP_T)
    e32.synchronize()
    e32.close()
    assert b32 * 2 == b64
    assert torch.isfinite(c32.lf.field[(1, 1, "MEVA")]).all()


def regrid_f32(src1, dst1, w, x32, n_dst):
    """do_regridding (basic:480-487) in the single-precision build's REAL(4) arithmetic:
    dst = 0; dst(d_k) = dst(d_k) + src(s_k) * w_k in link order (1-based indices)."""
    out = np.zeros(n_dst, np.float32)
    w32 = np.asarray(w, np.float32)
    for k in range(len(w32)):
        d = int(dst1[k]) - 1
        out[d] = np.float32(out[d] + np.float32(x32[int(src1[k]) - 1] * w32[k]))
    return out


def test_fp32_regridding_staged():
    """Staged plan in fp32: QSUR t->u replaces the u-grid QSUR, MEVA t->v.  The regridded
    arrays are bit-identical to the REAL(4) sequential sum of the GPU's own t-grid values;
    every output is within the fp32 gate of the fp64 oracle."""
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
        case.methods["which_spec_vapor_surface_u"][s - 1] = "none"
        case.lf.put_to[(s, 1, "QSUR")] = 2
        case.lf.put_to[(s, 1, "MEVA")] = 4
        case.lf.allocate_localvar("MEVA", s, 3, value=np.nan)
        case.outputs.append((s, 3, "MEVA"))
    c32 = as_dtype(case, "float32")
    c64 = as_dtype(c32, "float64")
    ref = oracle_lib.run_case(c64, "c", current_step_time=STEP_T, regrid=True)
    eng = Engine(c32.lf, c32.num_surface_types, c32.methods, corrections=c32.corrections,
                 averages=c32.averages, regrid=c32.regrid)
    eng.step(1, STEP_T)
    eng.step(2, STEP_T)
    eng.close()
    got = {k: np.array(c32.lf.field[k], dtype=np.float64) for k in c32.outputs}
    check(got, ref, "fp32 regrid")
    for s in (1, 2):
        src, dst, w = mats[2]
        want = regrid_f32(src, dst, w, np.asarray(c32.lf.field[(s, 1, "QSUR")]), nu)
        np.testing.assert_array_equal(np.asarray(c32.lf.field[(s, 2, "QSUR")]), want, err_msg=f"QSUR u s={s}")
        src, dst, w = mats[3]
        want = regrid_f32(src, dst, w, np.asarray(c32.lf.field[(s, 1, "MEVA")]), nv)
        np.testing.assert_array_equal(np.asarray(c32.lf.field[(s, 3, "MEVA")]), want, err_msg=f"MEVA v s={s}")


ATM_FIELDS = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))


@pytest.mark.parametrize("device_out", [False, True])
def test_fp32_atmos_accumulation_and_remap(device_out):
    """fp32 engine with the exchange -> atmosphere accumulation and an exchange -> model
    remap: fp32 fields in, fp32 outputs, weights and sums in fp64 (OASIS maps in double).
    Bit-identical to the fp64 sequential sum of the GPU's own fp32 fluxes, rounded once."""
    torch = pytest.importorskip("torch")
    from fcx.parallel import local_atmos, synthetic_atmos_map, synthetic_model_map

    n = 20_011
    c32 = as_dtype(build_case("MOM5", n=n, T=1, bias=True), "float32")
    amap = synthetic_atmos_map(n)
    la = local_atmos(amap, 0, 1)
    mmap = synthetic_model_map(n, 1_700, links_per_cell=2)

    def out(m):
        if device_out:
            return torch.full((m,), float("nan"), dtype=torch.float32, device="cuda:0")
        return np.full(m, np.nan, np.float32)

    atm = {k: out(la.n_atmos) for k, _ in ATM_FIELDS}
    rmo = {k: out(mmap.n_model) for k, _ in ATM_FIELDS}
    eng = Engine(c32.lf, 1, c32.methods, corrections=c32.corrections,
                 atmos={"local": la, "fields": [(2, 1, g, k, atm[k]) for k, g in ATM_FIELDS]},
                 remaps=[{"n_dst": mmap.n_model, "src": mmap.src, "dst": mmap.dst, "w": mmap.weight,
                          "fields": [(2, 1, g, k, rmo[k]) for k, g in ATM_FIELDS]}])
    eng.step(PHASE_ALL, STEP_T)
    eng.close()

    def host(a):
        return a.cpu().numpy() if device_out else a

    for k, g in ATM_FIELDS:
        flux = np.asarray(c32.lf.field[(1, g, k)], dtype=np.float64)
        want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, flux, amap.n_atmos).astype(np.float32)
        np.testing.assert_array_equal(host(atm[k]), want, err_msg=f"atmos {k}")
        want = oracle_lib.remap_apply(mmap.src, mmap.dst, mmap.weight, flux, mmap.n_model).astype(np.float32)
        np.testing.assert_array_equal(host(rmo[k]), want, err_msg=f"remap {k}")


def test_fp32_engine_rejects_fp64_outputs():
    from fcx.parallel import local_atmos, synthetic_atmos_map

    n = 1_001
    c32 = as_dtype(build_case("CCLM", n=n, T=1), "float32")
    amap = synthetic_atmos_map(n)
    la = local_atmos(amap, 0, 1)
    with pytest.raises(TypeError):
        Engine(c32.lf, 1, c32.methods, atmos={"local": la, "fields": [(2, 1, 1, "MEVA", np.zeros(la.n_atmos))]})


# run lengths: 1..5, 1..9 (the fp32 fused kernel's halo tiles: 1 and 2 halo lanes of 4 cells),
# 1..10 and 40..64 (256-cell wave tiles crossed: records + fix-up), 1..400 (longer than half a
# 128-cell tile: atmos_kernel), 0..5 (atmosphere cells without exchange cells among them)
@pytest.mark.parametrize("lengths", [(1, 5), (1, 9), (1, 10), (40, 64), (1, 400), (0, 5)])
@pytest.mark.parametrize("mode", ["default", "nohalo", "capped", "pipelined", "pipelined_runtime"])
@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
def test_fp32_fused_accumulation(variant, mode, lengths):
    """The fp32 engine's flux kernel with the accumulation fused in (4 cells per lane,
    products and sums in fp64, outputs rounded once): segments across 256-cell tiles completed
    by halo tiles (default) or by the fix-up kernel (FCX_OPT_ATMOS_HALO 0, long segments, the
    chunk launches of the pipelined step through the staging arena and through runtime copies),
    and under a grid-stride cap.  Bit-identical to the sequential fp64 sum of the GPU's own
    fp32 fluxes, rounded once; the fluxes within the fp32 gate of the oracle."""
    from fcx.parallel import local_atmos
    from test_gpu_multirank import random_run_map

    n = 300_001 if mode.endswith("pipelined") else 70_001
    case = build_case(variant, n=n, T=1, bias=True, seed=23)
    c32 = as_dtype(case, "float32")
    amap = random_run_map(n, lengths, seed=lengths[1] + 5)
    la = local_atmos(amap, 0, 1)
    outs = {k: np.full(la.n_atmos, np.nan, np.float32) for k, _ in ATM_FIELDS}
    pipe = {"pipeline_chunks": 4, "pipeline_min_chunk": 65536, "zero_copy": 0}
    opts = {"default": {}, "nohalo": {"atmos_halo": 0}, "capped": {"max_blocks": 64}, "pipelined": pipe,
            "pipelined_runtime": {**pipe, "host_staging": 0}}[mode]
    eng = Engine(c32.lf, 1, c32.methods, corrections=c32.corrections,
                 atmos={"local": la, "fields": [(2, 1, g, k, outs[k]) for k, g in ATM_FIELDS]}, options=opts)
    for step in range(2):  # later runs reuse the crossing records
        for o in outs.values():
            o[:] = np.nan
        eng.step(PHASE_ALL, STEP_T + 3600 * step)
        for k, g in ATM_FIELDS:
            flux = np.asarray(c32.lf.field[(1, g, k)], dtype=np.float64)
            want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, flux, amap.n_atmos).astype(np.float32)
            np.testing.assert_array_equal(outs[k], want, err_msg=f"{variant} {mode} {k} step {step}")
    eng.close()
    c64 = as_dtype(c32, "float64")
    ref = oracle_lib.run_case(c64, "c", current_step_time=STEP_T + 3600)
    check({k: np.array(c32.lf.field[k], dtype=np.float64) for k in c32.outputs}, ref, f"{variant} fused fp32")
