"""Seeded random configurations of the flux path against the oracle (GPU).

The hand-picked cases of test_gpu_parity.py cover one axis at a time; here every case draws
all of them at once: the method of every (flux, surface type) from the reference's method
set (calc:25-385: CCLM / MOM5 / RCO / water / ice / StBo / zero, and copy for the types
after the first, prepare:36-38), 1-4 surface types with their averages (calc:368-385), the
u/v grids shared with the t grid or separate, bias on or off, RSDR bound or not, one phase
or early then normal, and grid sizes from 1 cell to a few thousand (partial wave tiles and
layout tiles).  Each case: the fused step's outputs within the SURVEY 8d tolerance
(tests/parity.py) of the C oracle, itself pinned to the reference flux_lib.
"""
import os

import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu

fcx = pytest.importorskip("fcx")
from fcx.basic import PHASE_ALL, PHASE_EARLY, PHASE_NORMAL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.synthetic import build_case  # noqa: E402

STEP_T = 3600 * 24 * 31  # February 1961: the month-2 bias slice
# FCX_RANDOM_SEED_BASE: other seeds for a longer search (the committed runs use 0)
SEED_BASE = int(os.environ.get("FCX_RANDOM_SEED_BASE", "0"))

FLUX_METHODS = {
    "which_flux_mass_evap": ("CCLM", "MOM5", "RCO", "zero"),
    "which_flux_heat_latent": ("water", "ice", "zero"),
    "which_flux_heat_sensible": ("CCLM", "MOM5", "RCO", "zero"),
    "which_flux_momentum": ("CCLM", "MOM5", "RCO", "zero"),
    "which_flux_radiation_blackbody": ("StBo", "zero"),
}
QSUR_TABLES = ("which_spec_vapor_surface_t", "which_spec_vapor_surface_u", "which_spec_vapor_surface_v")


def draw_case(seed):
    r = np.random.default_rng([seed, 20231015])
    T = int(r.integers(1, 5))
    n = int(r.choice([1, 2, 3, 127, 128, 129, 4095, 4097, int(r.integers(1, 6000))]))
    sep = None
    if r.random() < 0.4:
        sep = (max(1, n + int(r.integers(-5, 6))), max(1, n + int(r.integers(-5, 6))))
    variant = str(r.choice(["CCLM", "MOM5", "RCO"]))
    per_type = {}
    for s in range(1, T + 1):
        # the RCO variant computes no QSUR (RCO formulas do not read it): with CCLM / MOM5
        # methods drawn for other fluxes the types need it, so QSUR is computed (CCLM) there
        m = {t: "CCLM" for t in QSUR_TABLES} if variant == "RCO" else {}
        for table, choices in FLUX_METHODS.items():
            if r.random() < 0.5:  # else the variant's own method
                pool = choices + (("copy",) if s >= 2 else ())
                m[table] = str(r.choice(pool))
        if s >= 2 and r.random() < 0.3:  # QSUR of the first type (alias)
            for t in QSUR_TABLES:
                m[t] = "copy"
        if m:
            per_type[s] = m
    return dict(variant=variant, n=n, T=T, bias=bool(r.random() < 0.5),
                sep_grids=sep, rsdr=bool(r.random() < 0.3), per_type=per_type or None, seed=1000 + seed,
                two_phases=bool(r.random() < 0.4))


def conditioned_parity(make_case, got, ref, label, tol=1e-10, ulps=16, trials=8, regrid=False,
                       eps=float(np.finfo(np.float64).eps), normwise=False):
    """The SURVEY 8d gate (tests/parity.py: |x - ref| <= 1e-10 max(|ref|, 1e-6 |ref|_inf)),
    with one allowance for ill-conditioned cells.  Where a flux cancels -- HSEN = F c_p (T_s -
    T_a EF) with T_s ~ T_a EF, MEVA = F (q_s - q_a) with q_s ~ q_a -- one ulp of a
    transcendental (the device's pow / exp against the host libm's) moves the result by more
    than the gate: seed 19 of the transport test, one HSEN cell of 7,068 at 1.5e-10 where
    T_s - T_a EF = -2.4e-4 K.  Such a cell passes if the GPU agrees with the oracle within
    twice the oracle's own movement when every input array is perturbed by `ulps` ulps (eight
    seeded perturbations, random signs per cell: with two, T_s and T_a drew the same signs in
    both at fp32 seed 170026, the cancellation did not show, and a cell whose movement is 0.012
    was held to 2.8e-5); an error no input rounding explains still fails, and every other
    cell is held to the gate.  fp32 (normwise, eps = 2^-23): the norm-wise fp32 gate
    (|x - ref| <= 1e-5 |ref|_inf), the inputs perturbed by 16 fp32 ulps."""
    delta = {k: np.zeros(np.shape(v)) for k, v in ref.items()}
    for t in range(trials):
        c = make_case()
        outs = {id(c.lf.field[k]) for k in c.outputs}
        r = np.random.default_rng([t, 99])
        seen = set()
        for a in c.lf.field.values():
            if id(a) in outs or id(a) in seen or not isinstance(a, np.ndarray) or a.dtype != np.float64:
                continue
            seen.add(id(a))
            a *= 1.0 + ulps * eps * r.choice([-1.0, 1.0], a.shape)
        rp = oracle_lib.run_case(c, "c", current_step_time=STEP_T, regrid=regrid)
        for k in ref:
            with np.errstate(invalid="ignore"):
                d = np.abs(np.asarray(rp[k], dtype=np.float64) - np.asarray(ref[k], dtype=np.float64))
            delta[k] = np.fmax(delta[k], d)
    bad = []
    for k, rv in ref.items():
        x, rv = np.asarray(got[k], dtype=np.float64), np.asarray(rv, dtype=np.float64)
        fin = np.isfinite(rv)
        top = np.max(np.abs(rv[fin])) if fin.any() else 1.0
        scale = np.full(rv.shape, top) if normwise else np.maximum(np.abs(rv), 1e-6 * top)
        with np.errstate(invalid="ignore"):
            err = np.abs(x - rv)
            ok = (err <= tol * scale) | (err <= 2.0 * delta[k]) | (np.isnan(x) & np.isnan(rv))
        if not ok.all():
            i = np.nonzero(~ok)[0]
            bad.append(f"{k}: {i.size} cells, first {i[:4].tolist()} got {x[i[:4]].tolist()} want "
                       f"{rv[i[:4]].tolist()} (input-rounding movement {delta[k][i[:4]].tolist()})")
    assert not bad, f"{label}: " + "; ".join(bad)


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 64))
def test_random_configuration(seed):
    spec = draw_case(seed)
    two = spec.pop("two_phases")
    case = build_case(**spec)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, regrid=case.regrid)
    for ph in ((PHASE_EARLY, PHASE_NORMAL) if two else (PHASE_ALL,)):
        eng.step(ph, STEP_T)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    conditioned_parity(lambda: build_case(**spec), got, ref, label=f"seed {seed}: {spec} two_phases={two}")


def draw_transport(seed):
    """Random host transport and launch-shape options (include/fcx.h FCX_OPT_*): zero-copy
    never / always / auto, the staging arena or one runtime copy per array, the chunk pipeline
    from 2 x 1024-4096 cells, one cell per lane, a grid-stride cap, the plain layout, deferred
    host copies."""
    r = np.random.default_rng([seed, 7])
    opts = {"zero_copy": int(r.choice([0, 1, 2]))}
    if r.random() < 0.5:
        opts["host_staging"] = int(r.integers(0, 2))
    if r.random() < 0.6:
        opts.update(pipeline_chunks=int(r.choice([2, 3, 4, 8])), pipeline_min_chunk=1024 * int(r.integers(1, 5)))
    if r.random() < 0.3:
        opts["cells_per_thread"] = 1
    if r.random() < 0.3:
        opts["max_blocks"] = int(r.choice([1, 7, 64]))
    if r.random() < 0.3:
        opts["tiled_layout"] = 0
    if r.random() < 0.3:
        opts["deferred_scatter"] = 1
    return opts


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 48))
def test_random_configuration_and_transport(seed):
    """A random configuration (draw_case) through random transport options: every transport
    and launch shape gives the oracle's results."""
    spec = draw_case(100 + seed)
    two = spec.pop("two_phases")
    spec["n"] = max(spec["n"], int(np.random.default_rng(seed).integers(1, 12_000)))
    if spec["sep_grids"]:
        spec["sep_grids"] = (spec["n"] + 3, max(1, spec["n"] - 2))
    opts = draw_transport(seed)
    case = build_case(**spec)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, regrid=case.regrid, options=opts)
    for ph in ((PHASE_EARLY, PHASE_NORMAL) if two else (PHASE_ALL,)):
        eng.step(ph, STEP_T)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    conditioned_parity(lambda: build_case(**spec), got, ref, label=f"seed {seed}: {spec} {opts} two_phases={two}")


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 32))
def test_random_configuration_fp32(seed):
    """The fp32 engine on a random configuration, against the fp64 oracle on the same
    (fp32-rounded) inputs: the norm-wise fp32 gate of tests/parity.py."""
    from parity import FP32_NORM_GATE
    from fcx.synthetic import as_dtype

    spec = draw_case(200 + seed)
    spec.pop("two_phases")
    c32 = as_dtype(build_case(**spec), "float32")
    c64 = as_dtype(c32, "float64")  # exactly the inputs the fp32 kernel saw
    ref = oracle_lib.run_case(c64, "c", current_step_time=STEP_T)
    eng = Engine(c32.lf, c32.num_surface_types, c32.methods, corrections=c32.corrections,
                 averages=c32.averages)
    eng.step(PHASE_ALL, STEP_T)
    got = {k: np.array(c32.lf.field[k], dtype=np.float64) for k in c32.outputs}
    eng.close()
    # (a few cells of 1-3 with HSEN cancelling in fp32 exceed the norm-wise gate: seed 24)
    conditioned_parity(lambda: as_dtype(as_dtype(build_case(**spec), "float32"), "float64"), got, ref,
                       label=f"seed {seed}: {spec} (fp32)", tol=FP32_NORM_GATE, eps=2.0 ** -23, normwise=True)


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 32))
def test_random_fused_accumulation(seed):
    """The exchange -> atmosphere accumulation fused into the flux pass, one surface type (the
    fluxes) or two (the type-0 averages), on random run-length maps (0..5 up to 1..400 cells
    per atmosphere cell: halo tiles, crossing records, atmos_kernel, empty atmosphere cells)
    with random launch options: bit-identical to the sequential sum of the GPU's own values."""
    import torch
    from fcx.parallel import local_atmos
    from test_gpu_multirank import random_run_map

    r = np.random.default_rng([seed, 11])
    T = int(r.integers(1, 3))
    n = int(r.integers(1, 40_000))
    lengths = [(1, 5), (1, 9), (1, 10), (20, 64), (1, 400), (0, 5)][int(r.integers(0, 6))]
    opts = {}
    if r.random() < 0.4:
        opts["atmos_halo"] = 0
    if r.random() < 0.3:
        opts["max_blocks"] = int(r.choice([1, 16, 64]))
    if r.random() < 0.3:
        opts.update(pipeline_chunks=4, pipeline_min_chunk=4096, zero_copy=0)
    variant = str(r.choice(["CCLM", "MOM5", "RCO"]))
    case = build_case(variant, n=n, T=T, bias=bool(r.random() < 0.5), seed=3000 + seed)
    amap = random_run_map(n, lengths, seed=4000 + seed)
    la = local_atmos(amap, 0, 1)
    fields = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))
    s_out = 1 if T == 1 else 0
    outs = {k: torch.full((la.n_atmos,), float("nan"), dtype=torch.float64, device="cuda:0") for k, _ in fields}
    phase_of = {"RBBR": 1}  # the early phase's field; the others are the normal phase's
    atmos = {"local": la, "fields": [(phase_of.get(k, 2), s_out, g, k, outs[k]) for k, g in fields]}
    eng = Engine(case.lf, T, case.methods, corrections=case.corrections, averages=case.averages, atmos=atmos,
                 options=opts)
    for step in range(2):
        for o in outs.values():
            o.fill_(float("nan"))
        eng.step(PHASE_ALL, STEP_T + 3600 * step)
        torch.cuda.synchronize()
        for k, g in fields:
            src = np.asarray(case.lf.field[(s_out, g, k)])
            # (the rank's atmosphere range starts at its first exchange cell's atmosphere
            # cell: leading atmosphere cells without exchange cells are no rank's)
            want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, src, amap.n_atmos)
            want = want[la.atmos_offset: la.atmos_offset + la.n_atmos]
            np.testing.assert_array_equal(outs[k].cpu().numpy(), want,
                                          err_msg=f"seed {seed}: {variant} T={T} n={n} {lengths} {opts} {k} step {step}")
    eng.close()


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 16))
def test_random_regridding(seed):
    """do_regridding (basic:463-522) inside the step, on random separate t/u/v grids with all
    four matrices in use (build_regrid_case: QSUR t->u, t->v; UMOM u->t; VMOM v->t), random
    method sets, types, bias and phases, against the oracle's staged sequence."""
    from fcx.synthetic import build_regrid_case

    r = np.random.default_rng([seed, 13])
    n = int(r.integers(1, 3000))
    kw = dict(variant=str(r.choice(["CCLM", "MOM5", "RCO"])), n=n,
              sep_grids=(max(1, n + int(r.integers(-40, 41))), max(1, n + int(r.integers(-40, 41)))),
              T=int(r.integers(1, 4)), bias=bool(r.random() < 0.5), seed=5000 + seed)
    two = bool(r.random() < 0.5)
    case = build_regrid_case(**kw)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T, regrid=True)
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, regrid=case.regrid)
    for ph in ((PHASE_EARLY, PHASE_NORMAL) if two else (PHASE_ALL,)):
        eng.step(ph, STEP_T)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    conditioned_parity(lambda: build_regrid_case(**kw), got, ref, label=f"seed {seed}: {kw} two_phases={two}",
                       regrid=True)


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 12))
def test_random_group_launch(seed):
    """fcx_run_group over a random member list (1-4 engines, repeats allowed), grid size,
    precision, surface types and map: every flux and atmosphere value the bits of each
    engine's own fcx_run (test_gpu_group.run_both)."""
    from test_gpu_group import run_both, same_bits

    r = np.random.default_rng([seed, 17])
    variants = tuple(str(v) for v in r.choice(["CCLM", "MOM5", "RCO"], int(r.integers(1, 5))))
    precision = "f32" if r.random() < 0.4 else "f64"
    types = 1 if precision == "f32" else int(r.integers(1, 3))
    n = int(r.integers(1_000, 200_000))
    opts = {"atmos_halo": 0} if r.random() < 0.3 else None
    a, b = run_both(n, variants, str(r.choice(["random", "periodic"])), precision, types=types, options=opts)
    same_bits(a, b)


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 12))
def test_random_sharded_accumulation(seed):
    """The APPLE-sharded step (decomp_def.F90:23-31) on a random map: 2-6 engines in one
    process, each its rank's cells, the boundary slots summed as the all-reduce would
    (fused or separate accumulation).  Every atmosphere cell one rank owns is bit-identical to
    the sequential sum of the GPU's own fluxes; a cell two ranks share is the sum of their two
    partial sums, within 4 eps of the sum of the products' magnitudes."""
    import torch
    from fcx.parallel import local_atmos
    from test_gpu_multirank import FIELDS, make_engine, random_run_map, shard_case

    r = np.random.default_rng([seed, 19])
    n = int(r.integers(2_000, 50_000))
    world = int(r.integers(2, 7))
    variant = str(r.choice(["CCLM", "MOM5", "RCO"]))
    fused = bool(r.random() < 0.7)
    lengths = [(1, 5), (1, 10), (20, 64), (0, 5)][int(r.integers(0, 4))]
    full = build_case(variant, n=n, T=1, bias=True, seed=911)
    amap = random_run_map(n, lengths, seed=6000 + seed)
    stride = len(FIELDS)
    engines = []
    for rank in range(world):
        la = local_atmos(amap, rank, world)
        shared = torch.zeros(max(world - 1, 1) * stride, dtype=torch.float64, device="cuda:0")
        case = shard_case(full, la.offset, la.offset + la.size, variant)
        eng, outs = make_engine(case, la, shared, stride, fused=fused)
        engines.append((la, shared, eng, outs, case))
    for la, shared, eng, outs, case in engines:
        eng.step(PHASE_ALL, 7200)
    total = sum(e[1] for e in engines)  # the all-reduce (sum) of the boundary slots
    for la, shared, eng, outs, case in engines:
        shared.copy_(total)
        eng.atmos_finish()
        eng.synchronize()
    owner = np.zeros(amap.n_atmos, np.int32)  # ranks holding part of each atmosphere cell
    got = {name: np.full(amap.n_atmos, np.nan) for name, _ in FIELDS}
    flux = {name: np.empty(n) for name, _ in FIELDS}
    for la, shared, eng, outs, case in engines:
        sl = slice(la.atmos_offset, la.atmos_offset + la.n_atmos)
        owner[sl] += 1
        for name, g in FIELDS:
            got[name][sl] = outs[name].cpu().numpy()[: la.n_atmos]
            flux[name][la.offset: la.offset + la.size] = np.asarray(case.lf.field[(1, g, name)])
        eng.close()
    eps = np.finfo(np.float64).eps
    for name, _ in FIELDS:
        want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, flux[name], amap.n_atmos)
        mag = oracle_lib.atmos_accumulate(amap.atmos_index, np.abs(amap.weight), np.abs(flux[name]), amap.n_atmos)
        one, two = owner == 1, owner >= 2
        np.testing.assert_array_equal(got[name][one], want[one], err_msg=f"seed {seed}: {name} (owned cells)")
        assert np.all(np.abs(got[name][two] - want[two]) <= 4 * eps * mag[two]), f"seed {seed}: {name} shared"


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 16))
def test_random_per_call_sequence(seed):
    """The reference subroutines one by one (calc:25-385, in flux_calculator.F90:902-1008's
    order) through the C ABI on a random configuration: the drop-in's level-0 path."""
    from fcx import flux_calculator_calculate as fcc

    spec = draw_case(300 + seed)
    spec.pop("two_phases")
    case = build_case(**spec)
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
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    fcc.release(lf)
    conditioned_parity(lambda: build_case(**spec), got, ref, label=f"seed {seed}: {spec} (per call)")


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 16))
def test_random_async_and_hand_over(seed):
    """fcx_step_async + fcx_synchronize, and fields handed over one by one (fcx_upload_field,
    a random subset, in random order) before fcx_step, on a random configuration and random
    transport: the bits of the plain fcx_step, over two steps."""
    spec = draw_case(400 + seed)
    spec.pop("two_phases")
    opts = draw_transport(400 + seed)
    r = np.random.default_rng([seed, 23])
    mode = str(r.choice(["async", "hand_over"]))

    def run(special):
        case = build_case(**spec)
        outs = {id(case.lf.field[k]) for k in case.outputs}
        slots, seen = [], set()
        for key, a in case.lf.field.items():
            if id(a) not in outs and id(a) not in seen:
                seen.add(id(a))
                slots.append(key)
        eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                     averages=case.averages, options=opts)
        res = []
        for step in range(2):
            for k in case.outputs:
                case.lf.field[k][:] = np.nan
            if special and mode == "async":
                eng.step_async(PHASE_ALL, STEP_T + 3600 * step)
                eng.synchronize()
            else:
                if special:
                    pick = r.permutation(len(slots))[: int(r.integers(0, len(slots) + 1))]
                    for i in pick:
                        eng.upload_field(*slots[i])
                eng.step(PHASE_ALL, STEP_T + 3600 * step)
            res.append({k: np.array(case.lf.field[k], copy=True) for k in case.outputs})
        eng.close()
        return res

    for a, b in zip(run(False), run(True)):
        assert a.keys() == b.keys()
        for k in a:
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"seed {seed}: {mode} {spec} {opts} {k}")


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 16))
def test_random_remaps(seed):
    """Exchange -> model remaps (fcx_add_remap) on random model grids,
    link counts, surface types (type 1 fields, or the type-0 averages at T >= 2), packing
    and transport: bit-identical to the sequential weight application on the GPU's own
    fields."""
    from fcx.parallel import synthetic_model_map

    r = np.random.default_rng([seed, 29])
    T = int(r.integers(1, 4))
    n = int(r.integers(10, 60_000))
    variant = str(r.choice(["CCLM", "MOM5", "RCO"]))
    case = build_case(variant, n=n, T=T, bias=bool(r.random() < 0.5), seed=7000 + seed)
    s = 0 if T >= 2 else 1
    fields = (("MEVA", 1), ("HSEN", 1), ("UMOM", 2), ("VMOM", 3), ("HLAT", 1), ("RBBR", 1))
    fields = tuple(fields[i] for i in sorted(r.choice(len(fields), int(r.integers(1, 7)), replace=False)))
    maps, outs = [], []
    for k in range(int(r.integers(1, 3))):
        n_model = int(r.integers(1, max(2, n // 3)))
        links = int(r.integers(1, 3))  # (a second link needs a second model cell)
        mm = synthetic_model_map(n, max(n_model, links), links_per_cell=links, seed=8000 + 10 * seed + k)
        oo = {name: np.full(mm.n_model, np.nan) for name, _ in fields}
        maps.append(mm)
        outs.append(oo)
    remaps = [{"n_dst": mm.n_model, "src": mm.src, "dst": mm.dst, "w": mm.weight,
               "fields": [(1 if name == "RBBR" else 2, s, g, name, oo[name]) for name, g in fields]}
              for mm, oo in zip(maps, outs)]
    opts = draw_transport(500 + seed)
    opts["remap_pack"] = int(r.integers(0, 3))
    eng = Engine(case.lf, T, case.methods, corrections=case.corrections, averages=case.averages, remaps=remaps,
                 options=opts)
    for step in range(2):
        eng.step(PHASE_ALL, STEP_T + 3600 * step)
        for mm, oo in zip(maps, outs):
            for name, g in fields:
                want = oracle_lib.remap_apply(mm.src, mm.dst, mm.weight, np.asarray(case.lf.field[(s, g, name)]),
                                              mm.n_model)
                np.testing.assert_array_equal(oo[name], want, err_msg=f"seed {seed}: {variant} T={T} {opts} {name}")
    eng.close()


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 12))
def test_random_fortran_dropin(seed, tmp_path):
    """The Fortran drop-in module in a Fortran host (tests/fortran/dropin_host.F90, a process
    without torch: the system HIP runtime) on a random configuration, each mode of
    test_fortran.py (per call, fused phases, async phases, fields handed over)."""
    import os
    import subprocess

    from test_fortran import DROPIN, write_manifest

    if not os.path.exists(DROPIN):
        pytest.skip("Fortran drop-in host not built")
    spec = draw_case(600 + seed)
    spec.pop("two_phases")
    mode = ("percall", "fused", "async", "handover")[seed % 4]
    case = build_case(**spec)
    outs = write_manifest(case, str(tmp_path), STEP_T)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    r = subprocess.run([DROPIN, str(tmp_path), mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "DROPIN_HOST OK" in r.stdout, r.stdout + r.stderr
    got = {key: np.fromfile(os.path.join(tmp_path, f"o{i}.bin"), dtype=np.float64) for i, key in enumerate(outs)}
    conditioned_parity(lambda: build_case(**spec), got, {k: ref[k] for k in outs},
                       label=f"seed {seed}: {spec} ({mode})")


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 16))
def test_random_fused_accumulation_fp32(seed):
    """The fp32 engine's fused accumulation (4 cells per lane, products and sums in fp64,
    outputs rounded once) on random maps, sizes and launch options: bit-identical to the
    sequential fp64 sum of the GPU's own fp32 fluxes, rounded once."""
    from fcx.parallel import local_atmos
    from fcx.synthetic import as_dtype
    from test_gpu_multirank import random_run_map

    r = np.random.default_rng([seed, 31])
    n = int(r.integers(1, 60_000))
    lengths = [(1, 5), (1, 9), (1, 10), (40, 64), (1, 400), (0, 5)][int(r.integers(0, 6))]
    opts = {}
    if r.random() < 0.4:
        opts["atmos_halo"] = 0
    if r.random() < 0.3:
        opts["max_blocks"] = int(r.choice([1, 16, 64]))
    if r.random() < 0.3:
        opts.update(pipeline_chunks=4, pipeline_min_chunk=4096, zero_copy=0)
    variant = str(r.choice(["CCLM", "MOM5", "RCO"]))
    c32 = as_dtype(build_case(variant, n=n, T=1, bias=bool(r.random() < 0.5), seed=9000 + seed), "float32")
    amap = random_run_map(n, lengths, seed=9500 + seed)
    la = local_atmos(amap, 0, 1)
    fields = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))
    outs = {k: np.full(la.n_atmos, np.nan, np.float32) for k, _ in fields}
    eng = Engine(c32.lf, 1, c32.methods, corrections=c32.corrections,
                 atmos={"local": la, "fields": [(2, 1, g, k, outs[k]) for k, g in fields]}, options=opts)
    for step in range(2):
        for o in outs.values():
            o[:] = np.nan
        eng.step(PHASE_ALL, STEP_T + 3600 * step)
        for k, g in fields:
            flux = np.asarray(c32.lf.field[(1, g, k)], dtype=np.float64)
            want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, flux, amap.n_atmos).astype(np.float32)
            want = want[la.atmos_offset: la.atmos_offset + la.n_atmos]
            np.testing.assert_array_equal(outs[k], want, err_msg=f"seed {seed}: {variant} n={n} {lengths} {opts} {k}")
    eng.close()


def draw_case_with_none(seed):
    """draw_case with 'none' methods (the flux not computed for that type, its array not
    allocated, prepare:36-42) for the independent fluxes: HSEN, momentum, RBBR, and MEVA with
    HLAT (HLAT water / ice needs its type's MEVA)."""
    spec = draw_case(seed)
    r = np.random.default_rng([seed, 43])
    per_type = dict(spec["per_type"] or {})
    for s in range(1, spec["T"] + 1):
        m = dict(per_type.get(s, {}))
        for table in ("which_flux_heat_sensible", "which_flux_momentum", "which_flux_radiation_blackbody"):
            if r.random() < 0.25:
                m[table] = "none"
        if r.random() < 0.2:
            m["which_flux_mass_evap"] = "none"
            m["which_flux_heat_latent"] = str(r.choice(["none", "zero"]))
        per_type[s] = m
    # 'copy' aliases the first type's array: none there, none here (prepare:36-38)
    first = per_type.get(1, {})
    for s in range(2, spec["T"] + 1):
        for table, method in list(per_type[s].items()):
            if method == "copy" and first.get(table) == "none":
                per_type[s][table] = "none"
    # HLAT water / ice needs its type's MEVA (prepare rejects it, the engine too): no MEVA, no HLAT
    for s in range(1, spec["T"] + 1):
        if per_type[s].get("which_flux_mass_evap") == "none" and \
                per_type[s].get("which_flux_heat_latent") not in ("none", "zero"):
            per_type[s]["which_flux_heat_latent"] = "none"
    spec["per_type"] = per_type
    return spec


@pytest.mark.parametrize("seed", range(SEED_BASE, SEED_BASE + 32))
def test_random_configuration_with_none(seed):
    """Random configurations in which some fluxes of some types are not computed at all."""
    spec = draw_case_with_none(700 + seed)
    two = spec.pop("two_phases")
    case = build_case(**spec)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, regrid=case.regrid, options=draw_transport(700 + seed))
    for ph in ((PHASE_EARLY, PHASE_NORMAL) if two else (PHASE_ALL,)):
        eng.step(ph, STEP_T)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    conditioned_parity(lambda: build_case(**spec), got, ref, label=f"seed {seed}: {spec} two_phases={two}")
