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
