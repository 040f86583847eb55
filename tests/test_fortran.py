"""The Fortran side of the boundary.

* the drop-in module flux_calculator_calculate (components.flux_calculator_amd/fortran)
  compiles against the reference's own flux_calculator_basic module and exports the
  reference subroutine names (checked on the built object);
* a Fortran host (tests/fortran/fcx_selftest.F90) drives libfcx through fcx_c_api on the
  GPU and matches the reference flux_lib called from Fortran (gpu)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM_O = os.path.join(ROOT, "components.flux_calculator_amd", "lib", "fortran", "flux_calculator_calculate.o")
SELFTEST = os.path.join(ROOT, "oracle", "_ref", "fcx_fortran_selftest")
REFERENCE_NAMES = ["calc_spec_vapor_surface", "calc_flux_mass_evap", "calc_flux_heat_latent",
                   "calc_flux_heat_sensible", "calc_flux_momentum_east", "calc_flux_momentum_north",
                   "calc_flux_radiation_blackbody", "distribute_shortwave_radiation_flux",
                   "average_across_surface_types"]


@pytest.mark.skipif(not os.path.exists(SHIM_O), reason="Fortran shim not built (needs flang + reference module)")
def test_dropin_module_exports_reference_subroutines():
    out = subprocess.run(["nm", SHIM_O], capture_output=True, text=True, check=True).stdout.lower()
    for name in REFERENCE_NAMES:
        assert f"_qmflux_calculator_calculatep{name}" in out, name
    for c in ("fcx_calc_flux_mass_evap", "fcx_average_across_surface_types", "fcx_bind_field"):
        assert f" u {c}" in out, c  # calls straight into the C ABI


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(SELFTEST), reason="Fortran self-test not built")
def test_fortran_host_selftest_on_gpu():
    r = subprocess.run([SELFTEST], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FCX_FORTRAN_SELFTEST OK" in r.stdout, r.stdout


DROPIN = os.path.join(ROOT, "oracle", "_ref", "fcx_dropin_host")
TABLES = ("which_spec_vapor_surface_t", "which_spec_vapor_surface_u", "which_spec_vapor_surface_v",
          "which_flux_mass_evap", "which_flux_heat_latent", "which_flux_heat_sensible", "which_flux_momentum",
          "which_flux_radiation_blackbody")  # fcx_attach's argument order


def write_manifest(case, d, step_time):
    """tests/fortran/dropin_host.F90's manifest of a synthetic case: every distinct array once
    (aliases share a buffer), the slot map, the method tables, corrections, type-0 outputs."""
    import numpy as np
    from fcx.basic import IDX

    bufs, lines, slots = {}, [], []
    for (s, g, name), a in case.lf.field.items():
        k = bufs.setdefault(id(a), (len(bufs) + 1, a))[0]
        slots.append(f"S {s} {g} {IDX[name]} {k} {int((s, g, name) in case.lf.allocated)}")
    nt, nu, nv = case.grid_size
    lines.append(f"N {len(bufs)} {case.num_surface_types} {nt} {nu} {nv}")
    for k, a in bufs.values():
        np.ascontiguousarray(a, dtype=np.float64).tofile(os.path.join(d, f"a{k}.bin"))
        lines.append(f"A {k} {a.shape[0]} a{k}.bin")
    lines += slots
    for t, table in enumerate(TABLES, start=1):
        for s, m in enumerate(case.methods[table], start=1):
            lines.append(f"M {t} {s} {m}")
    if case.corrections is not None:
        init_date, corr = case.corrections
        np.ascontiguousarray(corr, dtype=np.float64).tofile(os.path.join(d, "corr.bin"))  # [n][12] = (12, n)
        lines.append(f"C {init_date} corr.bin")
    for phase, g, name in case.averages:
        lines.append(f"V {phase} {g} {IDX[name]}")
    lines.append(f"R {step_time}")
    outs = list(dict.fromkeys(case.outputs))
    for i, (s, g, name) in enumerate(outs):
        lines.append(f"O {s} {g} {IDX[name]} o{i}.bin")
    with open(os.path.join(d, "manifest.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    return outs


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DROPIN), reason="Fortran drop-in host not built")
@pytest.mark.parametrize("mode", ["percall", "fused", "async", "handover", "libmem", "libmem_async"])
@pytest.mark.parametrize("variant,T", [("CCLM", 2), ("MOM5", 3), ("RCO", 1)])
def test_dropin_module_in_a_fortran_host(tmp_path, mode, variant, T):
    """The drop-in module flux_calculator_calculate driven by a Fortran host whose
    local_field is the reference's own flux_calculator_basic (tests/fortran/dropin_host.F90):
    the reference subroutines one by one (percall), the two fused phases (fused), or each
    phase started and finished in two calls (async: fcx_step_async + fcx_synchronize), or
    every input field handed over one by one before each phase (handover: fcx_upload_field,
    as after each oasis_get), against the oracle on the same inputs (tests/parity.py
    tolerance)."""
    import numpy as np

    import oracle_lib
    from fcx.synthetic import build_case
    from parity import assert_parity

    step_time = 3600 * 24 * 45  # February: the bias month changes from the init date's
    case = build_case(variant, n=5003, T=T, bias=True)
    outs = write_manifest(case, str(tmp_path), step_time)
    ref = oracle_lib.run_case(case, "c", current_step_time=step_time)
    r = subprocess.run([DROPIN, str(tmp_path), mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "DROPIN_HOST OK" in r.stdout, r.stdout
    got = {key: np.fromfile(os.path.join(tmp_path, f"o{i}.bin"), dtype=np.float64) for i, key in enumerate(outs)}
    assert_parity(got, {k: ref[k] for k in outs}, label=f"{variant} T={T} {mode}")


@pytest.mark.skipif(not os.path.exists(DROPIN), reason="Fortran drop-in host not built")
@pytest.mark.parametrize("mode,message", [
    ("noattach", "no flux engine attached"),
    ("badtable", "method table differs from the attached one: surface type 1"),
    ("badgrid", "grid_size"),
    ("badtypes", "num_surface_types 3 but the engine was attached with 2"),
])
def test_dropin_per_call_checks_its_arguments(tmp_path, mode, message):
    """The reference subroutines take my_bottom_model, num_surface_types, the method table and
    grid_size on every call (calc:25-385; called at flux_calculator.F90:902, 972-991).  The
    drop-in checks them against what fcx_attach bound and stops with a named error --
    the reference host loop without fcx_attach, a different method table, a different
    grid_size, a different type count.  Host-side only: no GPU work is reached."""
    from fcx.synthetic import build_case

    case = build_case("CCLM", n=257, T=2, bias=False)
    write_manifest(case, str(tmp_path), 3600)
    r = subprocess.run([DROPIN, str(tmp_path), mode], capture_output=True, text=True, timeout=120)
    out = r.stdout + r.stderr
    assert r.returncode != 0, out
    assert "flux engine contract violation" in out and message in out, out
    assert "DROPIN_HOST OK" not in out


@pytest.mark.skipif(not os.path.exists(DROPIN), reason="Fortran drop-in host not built")
@pytest.mark.parametrize("mode,message", [
    ("noattach", "no flux engine attached"),
    ("badtable", "method table differs from the attached one: surface type 1"),
])
def test_dropin_hands_errors_to_the_host_abort_routine(tmp_path, mode, message):
    """The reference ends a coupled run with oasis_abort(comp_id, comp_name, msg)
    (flux_calculator.F90:883-887), so the other components do not wait in their next
    exchange.  A host that registers its abort routine (fcx_register_abort -> the C ABI's
    fcx_set_abort_handler) gets the drop-in's contract-violation message there before the
    rank would stop: the test host's routine prints it and ends the run with code 3."""
    from fcx.synthetic import build_case

    case = build_case("CCLM", n=257, T=2, bias=False)
    write_manifest(case, str(tmp_path), 3600)
    r = subprocess.run([DROPIN, str(tmp_path), mode + "+abort"], capture_output=True, text=True, timeout=120)
    out = r.stdout + r.stderr
    assert r.returncode == 3, out
    line = [x for x in out.splitlines() if x.startswith("HOST ABORT ROUTINE: ")]
    assert line and "flux engine contract violation" in line[0] and message in line[0], out
    assert "DROPIN_HOST OK" not in out
