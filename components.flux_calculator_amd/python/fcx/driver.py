"""The coupling time loop of the reference main program (flux_calculator.F90:859-1026,
STEP 2) for a Python host, on a set-up from fcx.setup and an fcx.Engine.

Per coupling step, in the reference order:
  2.1  oasis_get of the early received fields (grids t, u, v; list order), then
       do_regridding of each early received field (F90:874-897);
  2.2  the early calculations: RBBR and its regridding           -> engine phase EARLY;
  2.3  oasis_put of the early sent fields, each type-0 field averaged first when the
       put loop's trigger holds (F90:906-937)                    -> averages in phase EARLY;
  2.4  oasis_get of the normal received fields + their regridding (F90:943-958);
  2.5  QSUR, MEVA, HLAT, HSEN, UMOM, VMOM with their regriddings, the shortwave
       distribution (F90:964-988)                                -> engine phase NORMAL;
  2.6  oasis_put of the normal sent fields, averaged first as in 2.3 (F90:994-1022).
The coupler stands in for OASIS3-MCT: `get(name, time, out)` fills the received field's
array in place (oasis_get writes through the io_field pointer), `put(name, time, array)`
takes the sent field.  The engine's step(phase) uploads what the phase reads, runs it on
the GPU and downloads what it writes, so the arrays the coupler sees are the host
local_field arrays exactly as in the reference loop.
"""
from .basic import PHASE_EARLY, PHASE_NORMAL


def _regridded(lf, f):
    """Does do_regridding(f.var, f.surface_type) have any put_to flag to act on?"""
    types = range(1, 11) if f.surface_type == 0 else (f.surface_type,)
    return any(lf.put_to.get((s, g, f.var), 0) for s in types for g in (1, 2, 3))


def coupling_step(setup, engine, coupler, current_time):
    lf = setup.local_field
    for early, phase in ((True, PHASE_EARLY), (False, PHASE_NORMAL)):
        for f in setup.fields_in_put_order(setup.input_field, early):
            coupler.get(f.name, current_time, lf.field[f.slot])
        for f in setup.input_field:
            if f.early == early and _regridded(lf, f):
                engine.do_regridding(f.var, f.surface_type)
        engine.step(phase, current_time)
        for f in setup.fields_in_put_order(setup.output_field, early):
            coupler.put(f.name, current_time, lf.field[f.slot])


def run(setup, engine, coupler, num_timesteps=None, timestep=None):
    """DO n_timestep = 1, num_timesteps; current_time = (n_timestep - 1) * timestep."""
    n = setup.nml["num_timesteps"] if num_timesteps is None else num_timesteps
    dt = setup.nml["timestep"] if timestep is None else timestep
    for k in range(1, n + 1):
        coupling_step(setup, engine, coupler, (k - 1) * dt)


__all__ = ["coupling_step", "run"]
