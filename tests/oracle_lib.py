"""ctypes access to the CPU oracles (TEST INFRASTRUCTURE ONLY).

  libfco.so      oracle/fco.c, the plain-C restatement (always built by build())
  libfco_ref.so  the reference flux_lib compiled from /root/reference + ref_harness.F90
                 (built only where /root/reference exists; travels to the GPU box)

run_case() executes one coupling step of a synthetic Case in the reference order
(flux_calculator.F90:902-1008) on a private deep copy of the case's arrays (aliasing kept)
and returns {(s, g, name): ndarray} for every output.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libfco.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libfco_ref.so")
REF_REGRID_SO = os.path.join(ROOT, "oracle", "_ref", "libfco_ref_regrid.so")

NV, MT = 35, 10
c_int32, c_void_p, c_uint8 = ctypes.c_int32, ctypes.c_void_p, ctypes.c_uint8


class FcoMatrix(ctypes.Structure):
    _fields_ = [("num_elements", c_int32), ("pad", c_int32), ("src_index", c_void_p),
                ("dst_index", c_void_p), ("weight", c_void_p)]


class FcoState(ctypes.Structure):
    _fields_ = [
        ("num_surface_types", c_int32),
        ("grid_size", c_int32 * 3),
        ("method", (c_int32 * MT) * 8),
        ("lcorrections", c_int32),
        ("current_month", c_int32),
        ("corrections", c_void_p),
        ("field", ((c_void_p * NV) * 3) * (MT + 1)),
        ("allocated", ((c_uint8 * NV) * 3) * (MT + 1)),
        ("put_to", ((c_uint8 * NV) * 3) * (MT + 1)),
        ("regrid", FcoMatrix * 4),
    ]


_libs = {}


def load(kind="c"):
    """kind "c": the C restatement; "ref": the reference flux_lib + ref_harness.F90;
    "ref_regrid": the reference do_regridding (flux_calculator_basic.F90:463-522)."""
    if kind == "ref_regrid":
        if kind not in _libs:
            if not os.path.exists(REF_REGRID_SO):
                return None
            lib = ctypes.CDLL(REF_REGRID_SO)
            lib.ref_do_regridding.argtypes = [ctypes.POINTER(FcoState), ctypes.c_int, ctypes.c_int]
            _libs[kind] = (lib, "ref_")
        return _libs[kind]
    if kind not in _libs:
        path = ORACLE_SO if kind == "c" else REF_SO
        if not os.path.exists(path):
            return None
        lib = ctypes.CDLL(path)
        p = "fco_" if kind == "c" else "ref_"
        for name in ("calc_flux_mass_evap", "calc_flux_heat_latent", "calc_flux_heat_sensible",
                     "calc_flux_radiation_blackbody", "distribute_shortwave_radiation_flux"):
            getattr(lib, p + name).argtypes = [ctypes.POINTER(FcoState)]
        for name in ("calc_spec_vapor_surface", "calc_flux_momentum_east", "calc_flux_momentum_north"):
            getattr(lib, p + name).argtypes = [ctypes.POINTER(FcoState), ctypes.c_int]
        getattr(lib, p + "average_across_surface_types").argtypes = [
            ctypes.POINTER(FcoState), ctypes.c_int, ctypes.c_int]
        if kind == "c":
            lib.fco_do_regridding.argtypes = [ctypes.POINTER(FcoState), ctypes.c_int, ctypes.c_int]
            lib.fco_current_month.argtypes = [ctypes.c_int32, ctypes.c_int64]
            lib.fco_current_month.restype = ctypes.c_int
            lib.fco_step_threads.argtypes = [ctypes.POINTER(FcoState), ctypes.c_int]
            lib.fco_step.argtypes = [ctypes.POINTER(FcoState)]
            lib.fco_remap_apply.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
            lib.fco_atmos_accumulate.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        _libs[kind] = (lib, p)
    return _libs[kind]


def current_month(init_date, seconds):
    lib, _ = load("c")
    return lib.fco_current_month(int(init_date), int(seconds))


FLUX_ORDER = ("which_spec_vapor_surface_t", "which_spec_vapor_surface_u",
              "which_spec_vapor_surface_v", "which_flux_mass_evap", "which_flux_heat_latent",
              "which_flux_heat_sensible", "which_flux_momentum", "which_flux_radiation_blackbody")
METHODS = ("none", "zero", "copy", "CCLM", "MOM5", "RCO", "water", "ice", "StBo")
VARNAMES = (
    "ALBE", "ALBA", "AMOI", "AMOM", "FARE", "FICE", "PATM", "PSUR", "QATM", "TATM", "TSUR", "UATM",
    "VATM", "U10M", "V10M", "CMOM", "CMOI", "CHEA", "QSUR", "HLAT", "HSEN", "MEVA", "MPRE", "MRAI",
    "MSNO", "RBBR", "RLWD", "RLWU", "RSID", "RSIU", "RSIN", "RSDD", "RSDR", "UMOM", "VMOM")
IDX0 = {n: i for i, n in enumerate(VARNAMES)}


class OracleState:
    """A private copy of a case's LocalFields (aliasing preserved) wired into FcoState."""

    def __init__(self, case, current_step_time=0, copy=True):
        """copy=False: work in place on the case's own float64 host arrays (the way the
        Fortran works on local_field), for OracleEngine."""
        self.case = case
        self.arrays = {}
        copies = {}
        for key, a in case.lf.field.items():
            if not copy:
                if not (isinstance(a, np.ndarray) and a.dtype == np.float64 and a.flags.c_contiguous):
                    raise TypeError(f"{key}: in-place oracle needs contiguous float64 host arrays")
                self.arrays[key] = a
                continue
            a = np.asarray(a) if isinstance(a, np.ndarray) else a.detach().cpu().numpy()
            if id(a) not in copies:
                copies[id(a)] = np.array(a, dtype=np.float64, copy=True)
            self.arrays[key] = copies[id(a)]
        st = FcoState()
        st.num_surface_types = case.num_surface_types
        for g in range(3):
            st.grid_size[g] = case.lf.grid_size[g]
        for f, table in enumerate(FLUX_ORDER):
            for s, m in enumerate(case.methods[table], start=1):
                st.method[f][s - 1] = METHODS.index(m.rstrip())
        for (s, g, name), a in self.arrays.items():
            st.field[s][g - 1][IDX0[name]] = a.ctypes.data
            st.allocated[s][g - 1][IDX0[name]] = 1 if (s, g, name) in case.lf.allocated else 0
        for (s, g, name), mask in case.lf.put_to.items():
            st.put_to[s][g - 1][IDX0[name]] = mask
        self._keep = []
        if case.regrid:
            for which, (src, dst, w) in case.regrid.get("matrices", {}).items():
                src = np.ascontiguousarray(src, dtype=np.int32)
                dst = np.ascontiguousarray(dst, dtype=np.int32)
                w = np.ascontiguousarray(w, dtype=np.float64)
                self._keep += [src, dst, w]
                st.regrid[which].num_elements = src.shape[0]
                st.regrid[which].src_index = src.ctypes.data
                st.regrid[which].dst_index = dst.ctypes.data
                st.regrid[which].weight = w.ctypes.data
        if case.corrections is not None:
            init_date, corr = case.corrections
            corr = np.ascontiguousarray(corr, dtype=np.float64)
            self._keep.append(corr)
            st.lcorrections = 1
            st.corrections = corr.ctypes.data
            st.current_month = current_month(init_date, current_step_time)
        self.st = st

    def outputs(self):
        return {k: self.arrays[k].copy() for k in self.case.outputs}


def run_case(case, kind="c", current_step_time=0, phases=(1, 2), regrid=False):
    """One coupling step in the order of flux_calculator.F90:902-1008 on an oracle."""
    o = OracleState(case, current_step_time)
    run_state(o, kind, phases, regrid)
    return o.outputs()


def host_threads():
    """Threads for the oracle on this host: the process's CPU share, capped at 16 (the GPU
    box's per-GPU share; os.cpu_count() there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def run_case_threads(case, current_step_time=0, nthreads=None):
    """run_case over the WHOLE grid with fco_step_threads: APPLE ranges over host threads,
    bit-identical to fco_step (test_oracle_golden.py::test_oracle_threads_equal_single_thread).
    No regridding; the type-0 averages follow serially, in the reference put order."""
    o = OracleState(case, current_step_time)
    lib, _ = load("c")
    lib.fco_step_threads(ctypes.byref(o.st), int(nthreads or host_threads()))
    for ph, g, name in case.averages:
        lib.fco_average_across_surface_types(ctypes.byref(o.st), g, IDX0[name])
    out = o.outputs()
    del o
    return out


class OracleEngine:
    """The fcx.driver engine interface (step / do_regridding) on the C oracle, in place on
    a set-up's LocalFields: the reference time loop with the oracle doing the arithmetic."""

    def __init__(self, setup, corrections=None, regrid=None):
        from fcx.synthetic import Case

        self.case = Case(name="setup", lf=setup.local_field, num_surface_types=setup.num_surface_types,
                         methods=setup.methods, corrections=corrections, averages=setup.averages(),
                         regrid=regrid)
        self.o = OracleState(self.case, 0, copy=False)
        self.lib, _ = load("c")

    def do_regridding(self, name, surface_type=0):
        self.lib.fco_do_regridding(ctypes.byref(self.o.st), IDX0[name], int(surface_type))

    def step(self, phase, current_step_time=0):
        if self.case.corrections is not None:
            self.o.st.current_month = current_month(self.case.corrections[0], current_step_time)
        run_state(self.o, "c", (1, 2) if phase == 3 else (phase,), regrid=True)


def run_state(o, kind="c", phases=(1, 2), regrid=False):
    """The coupling step on an existing OracleState (its arrays are updated in place)."""
    case = o.case
    lib, p = load(kind)
    sp = ctypes.byref(o.st)
    fn = lambda name: getattr(lib, p + name)  # noqa: E731
    if kind == "ref":  # the reference's own do_regridding next to its flux_lib (1-based varidx)
        rlib, _ = load("ref_regrid")
        rg1 = lambda v: rlib.ref_do_regridding(sp, IDX0[v] + 1, 0)  # noqa: E731
    else:  # fco_do_regridding takes the 0-based variable index
        rg1 = lambda v: load("c")[0].fco_do_regridding(sp, IDX0[v], 0)  # noqa: E731
    rg = rg1 if regrid else (lambda v: None)

    def averages(phase):
        for ph, g, name in case.averages:
            if ph == phase:
                fn("average_across_surface_types")(sp, g, IDX0[name])

    if 1 in phases:
        fn("calc_flux_radiation_blackbody")(sp)
        rg("RBBR")
        averages(1)
    if 2 in phases:
        for g in (1, 2, 3):
            fn("calc_spec_vapor_surface")(sp, g)
        rg("QSUR")
        fn("calc_flux_mass_evap")(sp)
        rg("MEVA")
        fn("calc_flux_heat_latent")(sp)
        rg("HLAT")
        fn("calc_flux_heat_sensible")(sp)
        rg("HSEN")
        fn("calc_flux_momentum_east")(sp, 2)
        rg("UMOM")
        fn("calc_flux_momentum_north")(sp, 3)
        rg("VMOM")
        fn("distribute_shortwave_radiation_flux")(sp)
        averages(2)


def atmos_accumulate(atmos_index, weight, x_field, n_atmos):
    """fco_atmos_accumulate: sequential SCRIP weight application (parity unpinned)."""
    lib, _ = load("c")
    idx = np.ascontiguousarray(atmos_index, dtype=np.int32)
    w = np.ascontiguousarray(weight, dtype=np.float64)
    x = np.ascontiguousarray(x_field, dtype=np.float64)
    out = np.empty(int(n_atmos))
    lib.fco_atmos_accumulate(idx.shape[0], idx.ctypes.data, w.ctypes.data, x.ctypes.data,
                             int(n_atmos), out.ctypes.data)
    return out


def remap_apply(src, dst, w, x_field, n_dst):
    """fco_remap_apply: sequential SCRIP weight application in link order (parity unpinned)."""
    lib, _ = load("c")
    src = np.ascontiguousarray(src, dtype=np.int32)
    dst = np.ascontiguousarray(dst, dtype=np.int32)
    w = np.ascontiguousarray(w, dtype=np.float64)
    x = np.ascontiguousarray(x_field, dtype=np.float64)
    out = np.empty(int(n_dst))
    lib.fco_remap_apply(src.shape[0], src.ctypes.data, dst.ctypes.data, w.ctypes.data, x.ctypes.data,
                        int(n_dst), out.ctypes.data)
    return out
