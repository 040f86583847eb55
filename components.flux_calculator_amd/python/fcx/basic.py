"""Mirror of the reference data model constants (flux_calculator_basic.F90).

varnames / idx_* (basic:42-60, 526-568), limits (basic:27-32), grid names (basic:64) and
the method strings of the namelist which_* tables (flux_calculator.F90:99-107).
"""

MAX_BOTTOM_MODELS = 10  # basic:27
MAX_SURFACE_TYPES = 10  # basic:28
MAX_VARNAMES = 35  # basic:42

# basic:43-51, in order: idx_X == VARNAMES.index(X) + 1
VARNAMES = (
    "ALBE", "ALBA", "AMOI", "AMOM", "FARE", "FICE", "PATM", "PSUR",
    "QATM", "TATM", "TSUR", "UATM", "VATM", "U10M", "V10M",
    "CMOM", "CMOI", "CHEA",
    "QSUR",
    "HLAT", "HSEN",
    "MEVA", "MPRE", "MRAI", "MSNO",
    "RBBR", "RLWD", "RLWU", "RSID", "RSIU", "RSIN", "RSDD", "RSDR",
    "UMOM", "VMOM",
)
IDX = {name: i + 1 for i, name in enumerate(VARNAMES)}

GRID_NAME = ("t_grid", "u_grid", "v_grid")  # basic:64
T_GRID, U_GRID, V_GRID = 1, 2, 3

# include/fcx.h enum fcx_method
METHODS = ("none", "zero", "copy", "CCLM", "MOM5", "RCO", "water", "ice", "StBo")
METHOD_ID = {m: i for i, m in enumerate(METHODS)}

# include/fcx.h enum fcx_flux: the which_* namelist tables
FLUXES = (
    "which_spec_vapor_surface_t",
    "which_spec_vapor_surface_u",
    "which_spec_vapor_surface_v",
    "which_flux_mass_evap",
    "which_flux_heat_latent",
    "which_flux_heat_sensible",
    "which_flux_momentum",
    "which_flux_radiation_blackbody",
)
FLUX_ID = {f: i for i, f in enumerate(FLUXES)}

PHASE_EARLY, PHASE_NORMAL, PHASE_ALL = 1, 2, 3

# early fields (basic:154-156 inputs, basic:271-273 outputs)
EARLY_INPUTS = ("FARE", "TSUR", "ALBE", "CMOM", "CMOI", "CHEA")
EARLY_OUTPUTS = ("RBBR", "TSUR", "FICE", "ALBE")


def method_id(method: str) -> int:
    """trim(method) == '...' (calc:39-48); raises like prepare's 'Method ... is not known'."""
    m = method.rstrip()
    if m not in METHOD_ID:
        raise ValueError(f"Method {method!r} is not known.")
    return METHOD_ID[m]
