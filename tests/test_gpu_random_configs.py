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
import numpy as np
import pytest

import oracle_lib
from parity import assert_parity

pytestmark = pytest.mark.gpu

fcx = pytest.importorskip("fcx")
from fcx.basic import PHASE_ALL, PHASE_EARLY, PHASE_NORMAL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.synthetic import build_case  # noqa: E402

STEP_T = 3600 * 24 * 31  # February 1961: the month-2 bias slice

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


@pytest.mark.parametrize("seed", range(32))
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
    assert_parity(got, ref, label=f"seed {seed}: {spec} two_phases={two}")
