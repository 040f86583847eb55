"""Reference-named host interface: module flux_calculator_calculate
(/root/reference/src/flux_calculator_calculate.F90) over libfcx.

Same subroutine names and argument meaning as the reference:
    calc_spec_vapor_surface(my_bottom_model, num_surface_types, which_grid, methods, grid_size, local_field)
    calc_flux_mass_evap(my_bottom_model, num_surface_types, methods, grid_size, local_field)
    ...
    average_across_surface_types(which_grid, my_idx, num_surface_types, grid_size, local_field)
`methods` is the which_* table indexed [my_bottom_model][surface_type] (1-based, as in the
namelist).  The reference module keeps no state; libfcx needs the bindings up front, so
prepare() (the counterpart of flux_calculator_prepare + fcx_commit) attaches an engine to
the LocalFields once, and every call checks that the methods it is given are the ones the
engine was prepared with.  Like the reference calc_* routines, the calls return nothing and
leave their results in local_field; errors raise fcx._lib.FcxError.
"""
from . import _lib
from .basic import IDX, FLUXES
from .engine import Engine


class _Table:
    """methods(my_bottom_model, surface_type) with 1-based indexing."""

    def __init__(self, per_type, my_bottom_model=1):
        self.rows = {my_bottom_model: list(per_type)}

    def __getitem__(self, key):
        b, s = key
        return self.rows[b][s - 1]

    def row(self, b):
        return self.rows[b]


def methods_2d(methods, my_bottom_model=1):
    """{which_*: [per type]} -> {which_*: table[my_bottom_model, surface_type]}"""
    return {k: _Table(v, my_bottom_model) for k, v in methods.items()}


def prepare(local_field, my_bottom_model, num_surface_types, methods, corrections=None,
            averages=(), regrid=None, device=0):
    """Bind local_field to a committed engine (validation as flux_calculator_prepare.F90)."""
    release(local_field)
    eng = Engine(local_field, num_surface_types, methods, corrections=corrections,
                 averages=averages, regrid=regrid, device=device)
    local_field.engine = eng
    local_field.engine_methods = {k: list(v)[:num_surface_types] for k, v in methods.items()}
    local_field.my_bottom_model = my_bottom_model
    return eng


def release(local_field):
    eng = getattr(local_field, "engine", None)
    if eng is not None:
        eng.close()
        local_field.engine = None


def _engine(local_field, table, methods, my_bottom_model, num_surface_types):
    eng = getattr(local_field, "engine", None)
    if eng is None:
        raise _lib.FcxError(_lib.FCX_OK + 2, "local_field has no engine: call prepare() first")
    if methods is not None:
        given = [methods[my_bottom_model, i].rstrip() for i in range(1, num_surface_types + 1)]
        if given != [m.rstrip() for m in local_field.engine_methods[table]]:
            raise _lib.FcxError(1, f"{table}: methods {given} differ from the prepared "
                                   f"{local_field.engine_methods[table]}")
    return eng


def calc_spec_vapor_surface(my_bottom_model, num_surface_types, which_grid, methods, grid_size, local_field):
    """calc:25-50"""
    eng = _engine(local_field, FLUXES[which_grid - 1], methods, my_bottom_model, num_surface_types)
    _lib.check(eng.lib.fcx_calc_spec_vapor_surface(eng.h, which_grid))


def calc_flux_mass_evap(my_bottom_model, num_surface_types, methods, grid_size, local_field,
                        current_step_time=0):
    """calc:54-120; current_step_time is the module variable of basic:125."""
    eng = _engine(local_field, "which_flux_mass_evap", methods, my_bottom_model, num_surface_types)
    _lib.check(eng.lib.fcx_calc_flux_mass_evap(eng.h, int(current_step_time)))


def calc_flux_heat_latent(my_bottom_model, num_surface_types, methods, grid_size, local_field):
    """calc:124-154"""
    eng = _engine(local_field, "which_flux_heat_latent", methods, my_bottom_model, num_surface_types)
    _lib.check(eng.lib.fcx_calc_flux_heat_latent(eng.h))


def calc_flux_heat_sensible(my_bottom_model, num_surface_types, methods, grid_size, local_field):
    """calc:156-208"""
    eng = _engine(local_field, "which_flux_heat_sensible", methods, my_bottom_model, num_surface_types)
    _lib.check(eng.lib.fcx_calc_flux_heat_sensible(eng.h))


def calc_flux_momentum_east(my_bottom_model, num_surface_types, which_grid, methods, grid_size, local_field):
    """calc:212-263"""
    eng = _engine(local_field, "which_flux_momentum", methods, my_bottom_model, num_surface_types)
    _lib.check(eng.lib.fcx_calc_flux_momentum_east(eng.h, which_grid))


def calc_flux_momentum_north(my_bottom_model, num_surface_types, which_grid, methods, grid_size, local_field):
    """calc:265-316"""
    eng = _engine(local_field, "which_flux_momentum", methods, my_bottom_model, num_surface_types)
    _lib.check(eng.lib.fcx_calc_flux_momentum_north(eng.h, which_grid))


def calc_flux_radiation_blackbody(my_bottom_model, num_surface_types, methods, grid_size, local_field):
    """calc:320-345"""
    eng = _engine(local_field, "which_flux_radiation_blackbody", methods, my_bottom_model,
                  num_surface_types)
    _lib.check(eng.lib.fcx_calc_flux_radiation_blackbody(eng.h))


def distribute_shortwave_radiation_flux(my_bottom_model, num_surface_types, grid_size, local_field):
    """calc:347-364 (skipped when RSDD/RSDR are not associated: P6)"""
    eng = _engine(local_field, None, None, my_bottom_model, num_surface_types)
    _lib.check(eng.lib.fcx_distribute_shortwave_radiation_flux(eng.h))


def average_across_surface_types(which_grid, my_idx, num_surface_types, grid_size, local_field):
    """calc:368-385; my_idx is the idx_* value or the variable name."""
    eng = _engine(local_field, None, None, None, num_surface_types)
    idx = IDX[my_idx] if isinstance(my_idx, str) else int(my_idx)
    _lib.check(eng.lib.fcx_average_across_surface_types(eng.h, which_grid, idx))


def do_regridding(varidx, surface_type, local_field):
    """basic:463-522 with the matrices given to prepare(regrid=...)."""
    eng = _engine(local_field, None, None, None, 0)
    idx = IDX[varidx] if isinstance(varidx, str) else int(varidx)
    _lib.check(eng.lib.fcx_do_regridding(eng.h, idx, surface_type))
