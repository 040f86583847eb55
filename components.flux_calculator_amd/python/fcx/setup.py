"""Set-up of one flux_calculator instance from flux_calculator.nml: the reference main
program's STEP 1.3-1.7 (flux_calculator.F90:262-768), restated for a Python host.

`FluxCalculatorSetup(nml, mype, grid_size)` reproduces, in the reference's order:
  * which bottom model this rank serves (F90:262-310, the num_tasks_per_model walk);
  * STEP 1.4, the received fields (F90:337-578): per grid t, u, v first the bottom model's
    variables per surface type, then the atmosphere's; allocate_localvar / init_localvar
    (constant `val_*`) / distribute_input_field (`val_bottom_var = -2e20`: use surface
    type 1) / add_input_field -> input_field names R + letter + VAR + NN (basic:129-168);
  * STEP 1.5, prepare_regridding of every received field (F90:585-594, basic:362-459);
  * STEP 1.6, the prepare_* checks and output allocations (flux_calculator_prepare.F90),
    each followed by prepare_regridding(var, 0) (F90:596-667);
  * STEP 1.7, the sent fields (F90:668-768, add_output_field basic:170-284): uniform
    aliases, type-0 allocations, default-valued fallbacks with their warnings, and
    output_field names S + letter + VAR + NN.
The local_field pointer structure is a LocalFields: a slot holds an array and aliasing is
holding the same array object; `allocated` and `put_to` follow the reference's flags
(allocate_localvar resets put_to; pointer assignment leaves the flags alone).

Fatal reference errors (mpi_finalize(1) / oasis_abort with a message) raise SetupError
with the reference's message; WARNING lines go to `self.log`.

The result drives the engine directly (`engine()`), the coupling step in the reference
order (`fcx.driver`), and the namcouple generator (`fcx.namcouple`).  The reference
set-up needs MPI, OASIS3-MCT and NetCDF, none of which this image has: its behaviour is
restated from the source and pinned by tests/test_setup_namcouple.py case by case
(parity unpinned against a reference run).
"""
from dataclasses import dataclass

import numpy as np

from .basic import (EARLY_INPUTS, EARLY_OUTPUTS, FLUXES, GRID_NAME, IDX, MAX_SURFACE_TYPES,
                    PHASE_EARLY, PHASE_NORMAL)
from .local_field import LocalFields
from .namelist import MAX_VARS

GRIDS = "tuv"


class SetupError(RuntimeError):
    """A fatal set-up error of the reference (mpi_finalize(1) / oasis_abort)."""


@dataclass
class IOField:
    """io_fields_type (basic:106-114) without the pointer: the slot is
    (surface_type, which_grid, var) of the set-up's LocalFields."""
    name: str  # OASIS name, 8 characters
    which_grid: int
    surface_type: int
    var: str
    early: bool

    @property
    def slot(self):
        return (self.surface_type, self.which_grid, self.var)


def numtype(i):
    """numtype(i) = '(I0.2)' of i (F90:333-335)."""
    return f"{i:02d}"


def count_bottom_models(nml):
    """F90:262-273: leading non-blank name_bottom_model entries; a gap is an error."""
    n = 0
    for i, name in enumerate(nml["name_bottom_model"], start=1):
        if name.strip() != "":
            n += 1
            if n < i:
                raise SetupError("ERROR: Vector name_bottom_model in flux_calculator.nml must not contain gaps.")
    return n


def find_bottom_model(nml, mype, num_bottom_models):
    """F90:275-298: walk the ranks over num_tasks_per_model; returns my_bottom_model."""
    ntask = nml["num_tasks_per_model"]
    i, j, k = 0, 1, 1
    while i < mype:
        if k < ntask[j - 1]:
            k += 1
            i += 1
        elif k == ntask[j - 1]:
            k = 1
            j += 1
            i += 1
        if j > len(ntask) or ntask[j - 1] == 0:
            j, i = -1, mype
        elif j > num_bottom_models:
            j, i = -1, mype
    if j < 0:
        raise SetupError("Too many MPI instances of flux_calculator were started. "
                         "Check your num_tasks_per_model settings in flux_calculator.nml.")
    return j


class FluxCalculatorSetup:
    def __init__(self, nml, mype=0, grid_size=None, device=None, dtype="float64"):
        """nml: fcx.namelist.read_input(...) values.  grid_size: (t, u, v) local cell
        counts (the reference reads them from the exchange-grid files, fcx.io)."""
        self.nml = nml
        self.mype = mype
        self.log = []
        self.num_bottom_models = count_bottom_models(nml)
        self.my_bottom_model = b = find_bottom_model(nml, mype, self.num_bottom_models)
        self.log.append(f"I am calculating fluxes for bottom model {b}")
        letter = nml["letter_bottom_model"][b - 1]
        if letter.strip() == "":
            raise SetupError(f"ERROR: letter_bottom_model({b}) must not be empty.")
        if letter in ("A", "R", "S"):
            raise SetupError(f"ERROR: letter_bottom_model({b}) has value {letter} which is reserved "
                             "(A=atmosphere, R=receive, S=send).")
        self.my_bottom_letter = letter
        if grid_size is None:
            raise SetupError("grid_size (t, u, v) is required (read it with fcx.io.read_scrip_grid)")
        self.grid_size = [int(x) for x in grid_size]
        self.local_field = LocalFields(self.grid_size, device=device, dtype=dtype)
        self.input_field = []
        self.output_field = []
        self._inputs()
        for f in self.input_field:  # STEP 1.5
            self.prepare_regridding(f.var, f.surface_type)
        self._prepares()
        self._outputs()

    # ------------------------------------------------------------- local_field helpers
    @property
    def num_surface_types(self):
        return self._T

    def _assoc(self, s, g, var):
        return (s, g, var) in self.local_field.field

    def _allocate(self, s, g, var, value=None, reset_put_to=True):
        """allocate_localvar (basic:288-309; resets put_to) or a bare ALLOCATE."""
        if var not in IDX:
            raise SetupError(f"Could not allocate local variable {var} because flux_calculator "
                             "does not know this variable.")
        lf = self.local_field
        lf.field[(s, g, var)] = lf._new(self.grid_size[g - 1], value)
        lf.allocated.add((s, g, var))
        if reset_put_to:
            lf.put_to.pop((s, g, var), None)

    def _point(self, dst, src):
        """dst => src (pointer assignment; a disassociated source disassociates dst)."""
        lf = self.local_field
        if src in lf.field:
            lf.field[dst] = lf.field[src]
        else:
            lf.field.pop(dst, None)

    def distribute_input_field(self, var, g, from_s, to_s):
        """basic:334-358."""
        if var not in IDX:
            raise SetupError(f"Could not distribute local variable {var} to other surface_types "
                             "because flux_calculator does not know this variable.")
        for j in range(1, self._T + 1):
            if j == to_s or (j != from_s and to_s == 0):
                self._point((j, g, var), (from_s, g, var))

    # ------------------------------------------------------------------ STEP 1.4
    def _inputs(self):
        nml, b = self.nml, self.my_bottom_model
        T = 0
        for g in GRIDS:  # F90:350-394: number of surface types
            names = nml[f"name_bottom_var_{g}"][b - 1]
            for i in range(1, MAX_SURFACE_TYPES + 1):
                if any(names[i - 1, j].rstrip() != "none" for j in range(MAX_VARS)):
                    T = max(T, i)
        self._T = T
        for gi, g in enumerate(GRIDS, start=1):
            names = nml[f"name_bottom_var_{g}"][b - 1]
            vals = nml[f"val_bottom_var_{g}"][b - 1]
            for i in range(1, MAX_SURFACE_TYPES + 1):
                for j in range(MAX_VARS):
                    name = names[i - 1, j]
                    if name.rstrip() == "none":
                        continue
                    self._allocate(i, gi, name)
                    v = vals[i - 1, j]
                    if v > -0.99e20:
                        self.local_field.field[(i, gi, name)][:] = v  # init_localvar
                    elif v < -1.99e20:
                        self.distribute_input_field(name, gi, 1, 0)
                    else:
                        self.add_input_field(name, self.my_bottom_letter, i, gi)
            names = nml[f"name_atmos_var_{g}"]
            vals = nml[f"val_atmos_var_{g}"]
            for j in range(MAX_VARS):
                name = names[j]
                if name.rstrip() == "none":
                    continue
                self._allocate(0, gi, name)
                v = vals[j]
                if v > -0.99e20:
                    self.local_field.field[(0, gi, name)][:] = v
                else:
                    self.add_input_field(name, "A", 0, gi)
                self.distribute_input_field(name, gi, 0, 0)

    def add_input_field(self, var, letter, s, g):
        """basic:129-168."""
        if var not in IDX:
            raise SetupError(f"Could not add input field for variable {var} because flux_calculator "
                             "does not know this variable.")
        self.input_field.append(IOField("R" + letter + var + numtype(s), g, s, var, var in EARLY_INPUTS))

    # ------------------------------------------------------------------ STEP 1.5
    def prepare_regridding(self, var, s):
        """basic:362-459: allocate the destination of every requested regrid and set the
        source's put_to flag.  s = 0: all surface types."""
        nml, b = self.nml, self.my_bottom_model
        lf = self.local_field
        for table, from_g, to_g, bit in (("u_to_t", 2, 1, 1), ("v_to_t", 3, 1, 1),
                                          ("t_to_u", 1, 2, 2), ("t_to_v", 1, 3, 4)):
            rows = nml[f"regrid_{table}"][b - 1]
            for j in range(1, MAX_SURFACE_TYPES + 1):
                if not (j == s or s == 0):
                    continue
                for k in range(MAX_VARS):
                    if rows[j - 1, k].rstrip() != var:
                        continue
                    if (j, to_g, var) in lf.allocated:
                        raise SetupError(f"Could not regrid local variable {var} from {GRID_NAME[from_g - 1]} "
                                         f"to {GRID_NAME[to_g - 1]} as requested in the namelist, because "
                                         "it already exists on that grid.")
                    self._allocate(j, to_g, var, reset_put_to=False)
                    lf.put_to[(j, from_g, var)] = lf.put_to.get((j, from_g, var), 0) | bit
                    self.log.append(f"    {GRID_NAME[from_g - 1]} -> {GRID_NAME[to_g - 1]}: {var} for surface type {j}")

    # ------------------------------------------------------------------ STEP 1.6
    # prepare_*: (method -> [(checked var, name in the message)]), 'copy' checks the type-1
    # array of `copy_var` -- the literal checks of flux_calculator_prepare.F90, including its
    # slips (HLAT 'copy' checks HSEN, several 'TSUR' messages test TATM, ...)
    _PREPARE = {
        "QSUR": ("QSUR", {"CCLM": [("FICE", "FICE"), ("PSUR", "PSUR"), ("TSUR", "TSUR")]}, False),
        "MEVA": ("MEVA", {
            "CCLM": [("AMOI", "AMOI"), ("PSUR", "PSUR"), ("QATM", "QATM"), ("QSUR", "QSUR"),
                     ("TATM", "TATM"), ("UATM", "UATM"), ("VATM", "VATM")],
            "MOM5": [("CMOI", "CMOI"), ("PSUR", "PSUR"), ("QATM", "QATM"), ("QSUR", "QSUR"),
                     ("TATM", "TATM"), ("UATM", "UATM"), ("VATM", "VATM")],
            "RCO": [("QATM", "QATM"), ("QSUR", "TSUR"), ("UATM", "UATM"), ("VATM", "VATM")]}, True),
        "HLAT": ("HSEN", {"water": [("MEVA", "MEVA")], "ice": [("MEVA", "MEVA")]}, True),
        "HSEN": ("HSEN", {
            "CCLM": [("AMOI", "AMOI"), ("PATM", "PATM"), ("PSUR", "PSUR"), ("QSUR", "QSUR"),
                     ("TATM", "TATM"), ("TATM", "TSUR"), ("UATM", "UATM"), ("VATM", "VATM")],
            "MOM5": [("CHEA", "CHEA"), ("PATM", "PATM"), ("PSUR", "PSUR"), ("QSUR", "QSUR"),
                     ("TATM", "TATM"), ("TATM", "TSUR"), ("UATM", "UATM"), ("VATM", "VATM")],
            "RCO": [("TATM", "TATM"), ("TATM", "TSUR"), ("UATM", "UATM"), ("VATM", "VATM")]}, True),
        "UMOM": ("UMOM", {
            "CCLM": [("AMOM", "AMOM"), ("PSUR", "PSUR"), ("QSUR", "QSUR"), ("TATM", "TATM"),
                     ("TATM", "TSUR"), ("UATM", "UATM")],
            "MOM5": [("CMOM", "CMOM"), ("PSUR", "PSUR"), ("QSUR", "QSUR"), ("TATM", "TATM"),
                     ("TATM", "TSUR"), ("UATM", "UATM")],
            "RCO": [("UATM", "UATM"), ("VATM", "VATM")]}, True),
        "VMOM": ("VMOM", {
            "CCLM": [("AMOM", "AMOM"), ("PSUR", "PSUR"), ("QSUR", "QSUR"), ("TATM", "TATM"),
                     ("TATM", "TSUR"), ("UATM", "VATM")],
            "MOM5": [("CMOM", "CMOM"), ("PSUR", "PSUR"), ("QSUR", "QSUR"), ("TATM", "TATM"),
                     ("TATM", "TSUR"), ("UATM", "VATM")],
            "RCO": [("UATM", "UATM"), ("VATM", "VATM")]}, True),
        "RBBR": ("RBBR", {"StBo": [("TSUR", "TSUR")]}, True),
    }

    def prepare(self, var, s, g, method):
        """prepare_<var> + do_prepare_calculation (prepare:19-44 and the per-flux routines)."""
        m = method.rstrip()
        if m == "none":
            return
        copy_var, checks, has_zero = self._PREPARE[var]
        where = f"{var} for surface_type {s} on the grid {GRID_NAME[g - 1]}"
        missing = ""
        if m == "copy":
            if not self._assoc(1, g, copy_var):
                missing = f"{var} for surface_type=1 "
        elif m == "zero" and has_zero:
            pass
        elif m in checks:
            for need, label in checks[m]:
                if not self._assoc(s, g, need):
                    missing = missing.rstrip() + " " + label
        else:
            raise SetupError(f"Error calculating {where}:    Method {method} is not known. ")
        if missing.strip():
            raise SetupError(f"Error calculating {where}:    For method {method} we are lacking "
                             f"the following variables: {missing.rstrip()}")
        if m == "copy":
            self._point((s, g, var), (1, g, var))
        else:
            self._allocate(s, g, var, reset_put_to=False)

    def _prepares(self):
        nml, b, T = self.nml, self.my_bottom_model, self._T
        row = lambda key: nml[key][b - 1]  # noqa: E731
        for i in range(1, T + 1):
            for gi, g in enumerate(GRIDS, start=1):
                self.prepare("QSUR", i, gi, row(f"which_spec_vapor_surface_{g}")[i - 1])
        self.prepare_regridding("QSUR", 0)
        for var, g, key in (("MEVA", 1, "which_flux_mass_evap"), ("HLAT", 1, "which_flux_heat_latent"),
                            ("HSEN", 1, "which_flux_heat_sensible"),
                            ("RBBR", 1, "which_flux_radiation_blackbody"),
                            ("UMOM", 2, "which_flux_momentum"), ("VMOM", 3, "which_flux_momentum")):
            for i in range(1, T + 1):
                self.prepare(var, i, g, row(key)[i - 1])
            self.prepare_regridding(var, 0)

    # ------------------------------------------------------------------ STEP 1.7
    def _outputs(self):
        nml, b, letter = self.nml, self.my_bottom_model, self.my_bottom_letter
        T = self._T
        for j in range(MAX_VARS):
            for gi, g in enumerate(GRIDS, start=1):
                name = nml[f"name_send_{g}"][j]
                if name.rstrip() == "none":
                    continue
                to_bottom = nml[f"send_to_bottom_{g}"][b - 1, j]
                uniform = nml[f"send_uniform_{g}"][b - 1, j]
                default = nml[f"val_flux_{g}"][j]
                if nml[f"send_to_atmos_{g}"][j]:
                    # F90:694-700 / 717-723 / 740-746: with no bottom send, t uses
                    # uniform=.FALSE. but u and v use .TRUE.
                    u = uniform if to_bottom else (g != "t")
                    self.add_output_field(name, "A", 0, gi, u, default)
                if to_bottom:
                    if uniform:
                        self.add_output_field(name, letter, 1, gi, True, default)
                    else:
                        for i in range(1, T + 1):
                            self.add_output_field(name, letter, i, gi, False, default)

    def add_output_field(self, var, letter, s, g, uniform, default_value):
        """basic:170-284."""
        append = numtype(s)
        if any(f.name.rstrip() == "R" + letter + var + append for f in self.input_field):
            return  # received already: no output field
        if var not in IDX:
            raise SetupError(f"Could not add output field for variable {var} because flux_calculator "
                             "does not know this variable.")
        T = self._T
        if s == 0:
            if uniform:
                for j in range(1, T + 1):
                    if self._assoc(j, g, var) and not self._assoc(0, g, var):
                        self._point((0, g, var), (j, g, var))
            else:
                all_fluxes = all(self._assoc(j, g, var) for j in range(1, T + 1))
                all_areas = all(self._assoc(j, g, "FARE") for j in range(1, T + 1))
                if not all_areas:
                    raise SetupError(f"ERROR: Output field {var} has not been defined as uniform "
                                     "(flux_?_uniform=.FALSE.). To calculate its average value across "
                                     "different surface_types, their fractional area (FARE) must be "
                                     "given but is missing.")
                if all_fluxes and not self._assoc(0, g, var):
                    self._allocate(0, g, var, reset_put_to=False)
            if not self._assoc(0, g, var):
                self.log.append(f"WARNING: Flux {var} cannot be calculated for surface_type=0  =>  set to {default_value}")
                self._allocate(0, g, var, value=default_value, reset_put_to=False)
        else:
            if uniform and not self._assoc(s, g, var):
                for j in range(1, T + 1):  # basic:245-249: the alias lands in type 0
                    if self._assoc(j, g, var) and not self._assoc(0, g, var):
                        self._point((0, g, var), (j, g, var))
            if not self._assoc(s, g, var):
                self.log.append(f"WARNING: Flux {var} cannot be calculated for surface_type={s}  =>  set to {default_value}")
                self._allocate(s, g, var, value=default_value, reset_put_to=False)
        self.output_field.append(IOField("S" + letter + var + append, g, s, var, var in EARLY_OUTPUTS))

    # ------------------------------------------------------------------ products
    @property
    def methods(self):
        """{which_*: [method per surface type 1..T]} for the engine (the namelist rows of
        my_bottom_model)."""
        b, T = self.my_bottom_model, self._T
        out = {}
        for key in FLUXES:
            out[key] = [self.nml[key][b - 1, i].rstrip() for i in range(T)]
        return out

    def averages(self):
        """(phase, grid, var) of the type-0 outputs the put loops average before sending:
        ASSOCIATED(local_field(0)) .AND. ASSOCIATED(local_field(2)) (F90:913-914,
        1003-1004) and local_field(0)%allocated (calc:376), in put order (grids t, u, v;
        output list order)."""
        lf = self.local_field
        out = []
        for early, phase in ((True, PHASE_EARLY), (False, PHASE_NORMAL)):
            for g in (1, 2, 3):
                for f in self.output_field:
                    if f.which_grid != g or f.early != early or f.surface_type != 0:
                        continue
                    if (self._assoc(0, g, f.var) and self._assoc(2, g, f.var)
                            and (0, g, f.var) in lf.allocated):
                        if (phase, g, f.var) not in out:
                            out.append((phase, g, f.var))
        return out

    def fields_in_put_order(self, fields, early):
        """The get/put loops' order: grid t, u, v, then list order (F90:878-889, 905-932)."""
        return [f for g in (1, 2, 3) for f in fields if f.which_grid == g and f.early == early]

    def computed_slots(self):
        """(s, g, var) slots written by the step: outputs of the calculations, regrid
        destinations and averaged type-0 fields."""
        out = set()
        for (s, g, var) in self.local_field.field:
            if var in ("QSUR", "MEVA", "HLAT", "HSEN", "RBBR", "UMOM", "VMOM") and s >= 1:
                out.add((s, g, var))
        for _, g, var in self.averages():
            out.add((0, g, var))
        return sorted(out)

    def engine(self, corrections=None, regrid=None, **kw):
        """An fcx.Engine over the set-up's local_field (methods, averages, put_to)."""
        from .engine import Engine

        return Engine(self.local_field, self._T, self.methods, corrections=corrections,
                      averages=self.averages(), regrid=regrid, **kw)


def setup_from_namelist(path_or_text, mype=0, grid_size=None, **kw):
    """Read flux_calculator.nml (&input) and set the instance up."""
    from .namelist import read_input

    text = path_or_text
    if "\n" not in text and not text.lstrip().startswith("&"):
        with open(text) as f:
            text = f.read()
    return FluxCalculatorSetup(read_input(text), mype=mype, grid_size=grid_size, **kw)


__all__ = ["SetupError", "IOField", "numtype", "count_bottom_models", "find_bottom_model",
           "FluxCalculatorSetup", "setup_from_namelist"]
