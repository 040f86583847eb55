"""The planner against the kernels' load predicates, on the host (no GPU): fcx_plan_check
builds every launch plan an engine can take (whole phases, the per-call subroutines, the
regridding sequence, the explicit averages) and audits each -- a flux the plan computes
must have every input the kernel loads for it bound ('zero' momentum loaded an
unbound wind).  Random method tables over the reference's method set (calc:25-385,
prepare:19-301), 1-4 surface types, shared or separate u/v grids, bias, RSDR."""
import os
import subprocess
import sys

import numpy as np
import pytest

from fcx import _lib
from fcx.engine import Engine
from fcx.synthetic import VARIANTS, build_case

TABLES = {
    "which_spec_vapor_surface_t": ("CCLM", "none"),
    "which_spec_vapor_surface_u": ("CCLM", "none"),
    "which_spec_vapor_surface_v": ("CCLM", "none"),
    "which_flux_mass_evap": ("CCLM", "MOM5", "RCO", "zero", "none"),
    "which_flux_heat_latent": ("water", "ice", "zero", "none"),
    "which_flux_heat_sensible": ("CCLM", "MOM5", "RCO", "zero", "none"),
    "which_flux_momentum": ("CCLM", "MOM5", "RCO", "zero", "none"),
    "which_flux_radiation_blackbody": ("StBo", "zero", "none"),
}
# what validate() may legitimately reject (prepare's rules); never the audit's FCX_E_STATE
VALIDATION = {1, 3, 5}


def draw(seed):
    r = np.random.default_rng([seed, 31337])
    T = int(r.integers(1, 5))
    n = int(r.choice([1, 7, 129, 4097]))
    sep = (max(1, n + int(r.integers(-3, 4))), max(1, n + int(r.integers(-3, 4)))) if r.random() < 0.4 else None
    variant = str(r.choice(["CCLM", "MOM5", "RCO"]))
    base = {k: VARIANTS[variant]["qsur"] for k in TABLES if k.startswith("which_spec")}
    per_type = {}
    for s in range(1, T + 1):
        m = {}
        for table, choices in TABLES.items():
            # 'copy' aliases the type-1 array (prepare:36-38): only where type 1 has one
            one = per_type.get(1, {}).get(table, base.get(table))
            pool = choices + (("copy",) if s >= 2 and one != "none" else ())
            if r.random() < 0.7:
                m[table] = str(r.choice(pool))
        per_type[s] = m
    return dict(variant=variant, n=n, T=T, bias=bool(r.random() < 0.5),
                sep_grids=sep, rsdr=bool(r.random() < 0.3), per_type=per_type, seed=7000 + seed)


OUTS = (("QSUR", (1, 2, 3)), ("MEVA", (1,)), ("HLAT", (1,)), ("HSEN", (1,)), ("RBBR", (1,)), ("UMOM", (2,)),
        ("VMOM", (3,)))


def complete(case):
    """Every flux array of every type associated, as on a host that receives or keeps them
    even where a type's method is 'none' (so that methods downstream read them as inputs):
    the tables then exercise the planner's input paths instead of prepare's rejections."""
    lf = case.lf
    for s in range(1, case.num_surface_types + 1):
        for name, grids in OUTS:
            for g in grids:
                if not lf.associated(s, g, name):
                    lf.allocate_localvar(name, s, g, value=0.0)


@pytest.mark.parametrize("seed", range(300))
def test_random_method_tables_pass_the_audit(seed):
    spec = draw(seed)
    case = build_case(**spec)
    complete(case)
    e = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
               averages=case.averages, commit=False)
    try:
        e.plan_check()
    except _lib.FcxError as ex:
        # prepare's own rejections are fine; an audit failure means the planner left an input
        # unbound that a kernel predicate would load
        assert ex.status in VALIDATION, f"{spec}: {ex}"
    finally:
        e.close()


def test_golden_like_cases_pass_the_audit():
    for v in ("CCLM", "MOM5", "RCO"):
        for T in (1, 2, 3):
            for sep in (None, (130, 127)):
                case = build_case(v, n=128, T=T, bias=True, sep_grids=sep, rsdr=True)
                e = Engine(case.lf, T, case.methods, corrections=case.corrections, averages=case.averages,
                           commit=False)
                e.plan_check()
                e.close()


@pytest.mark.parametrize("var,flux", [("UATM", "MEVA"), ("AMOI", "MEVA"), ("FICE", "QSUR(t)"), ("FARE", "average")])
def test_audit_names_an_unbound_input(var, flux):
    """With the planner told to forget one input (FCX_TEST_PLAN_UNBIND, tests only) the audit
    returns FCX_E_STATE naming the flux and the variable -- before any launch."""
    code = f"""
import sys
sys.path[:0] = {sys.path!r}
from fcx import _lib
from fcx.engine import Engine
from fcx.synthetic import build_case
case = build_case("CCLM", n=64, T=2, bias=True)
e = Engine(case.lf, 2, case.methods, corrections=case.corrections, averages=case.averages, commit=False)
try:
    e.plan_check()
except _lib.FcxError as ex:
    print("STATUS", ex.status, str(ex))
else:
    print("STATUS 0")
"""
    env = dict(os.environ, FCX_TEST_PLAN_UNBIND=var)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    line = [x for x in out.stdout.splitlines() if x.startswith("STATUS")]
    assert line, out.stderr[-2000:]
    assert line[0].startswith("STATUS 2 "), line[0]
    assert "plan audit" in line[0] and var in line[0] and flux in line[0], line[0]


def test_plan_check_after_commit_is_a_state_error():
    case = build_case("CCLM", n=16, T=1)
    e = Engine(case.lf, 1, case.methods, commit=False)
    e.plan_check()
    e.plan_check()  # repeatable: the dry plans are dropped
    e.close()
