"""Synthetic exchange-grid inputs and coupling configurations.

The real MOM5_Baltic-CCLM_Eurocordex exchange grid is not available (zenodo set-up,
Readme.md:49), so every benchmark and test runs on seeded synthetic data with the value
distributions of SURVEY.md 8d: numpy PCG64, base seed 20231015, one stream per variable.

A Case is one flux_calculator configuration: a LocalFields laid out the way
flux_calculator.F90:347-558 and flux_calculator_prepare.F90 would lay it out for the
given namelist (atmosphere fields distributed to every surface type by pointer, per-type
bottom fields, allocated outputs, 'copy' aliases), plus the which_* method tables, the
bias corrections and the registered type-0 averages.
"""
from dataclasses import dataclass, field

import numpy as np

from .basic import PHASE_EARLY, PHASE_NORMAL
from .local_field import LocalFields

BASE_SEED = 20231015
ATMOS_VARS = ("PATM", "PSUR", "QATM", "TATM", "UATM", "VATM", "AMOI", "AMOM", "RSDD", "ALBA")
BOTTOM_VARS = ("TSUR", "FICE", "FARE", "ALBE", "CMOI", "CHEA", "CMOM")
_VAR_STREAM = {v: i for i, v in enumerate(ATMOS_VARS + BOTTOM_VARS + ("CORR", "EDGE"))}


def _rng(var, seed, stype=0):
    return np.random.Generator(np.random.PCG64([seed, _VAR_STREAM[var], stype]))


def atmos_fields(n, seed=BASE_SEED, tsur=None):
    """Atmosphere-side fields on the exchange grid (type 0)."""
    out = {}
    ps = _rng("PSUR", seed).uniform(95000.0, 105000.0, n)
    out["PSUR"] = ps
    out["PATM"] = ps - _rng("PATM", seed).uniform(50.0, 1500.0, n)
    base_t = tsur if tsur is not None else _rng("TSUR", seed).uniform(271.0, 303.0, n)
    rt = _rng("TATM", seed)
    ta = np.clip(base_t + rt.normal(0.0, 3.0, n), 240.0, 310.0)
    if n >= 200:  # 0.5 % cells with T_a == T_s exactly (RCO stability switch, heat:153)
        eq = rt.permutation(n)[: n // 200]
        ta[eq] = base_t[eq]
    out["TATM"] = ta
    out["QATM"] = _rng("QATM", seed).uniform(5e-4, 2e-2, n)
    r = _rng("UATM", seed)
    u = r.normal(0.0, 7.0, n)
    v = _rng("VATM", seed).normal(0.0, 7.0, n)
    # 1 % calm cells (|vel| < u_min = 0.01), 1 % exactly at the RCO switch vel = 11
    k = max(n // 100, 1) if n >= 100 else 0
    if k:
        idx = r.permutation(n)
        calm, at11 = idx[:k], idx[k:2 * k]
        u[calm] = r.uniform(-0.007, 0.007, k)
        v[calm] = r.uniform(-0.007, 0.007, k)
        sgn = np.where(r.random(k) < 0.5, -1.0, 1.0)
        half = k // 2
        u[at11[:half]], v[at11[:half]] = 11.0 * sgn[:half], 0.0
        u[at11[half:]], v[at11[half:]] = 6.6 * sgn[half:], 8.8  # |vel| within an ulp of 11
    out["UATM"], out["VATM"] = u, v
    out["AMOI"] = _rng("AMOI", seed).uniform(5e-4, 3e-3, n)
    out["AMOM"] = _rng("AMOM", seed).uniform(5e-4, 3e-3, n)
    out["RSDD"] = _rng("RSDD", seed).uniform(-1000.0, 0.0, n)
    out["ALBA"] = _rng("ALBA", seed).uniform(0.05, 0.3, n)
    return out


def bottom_fields(n, stype, seed=BASE_SEED, ice=None):
    """Bottom-model fields of one surface type.  ice: None = Bernoulli(0.2), True/False = all."""
    out = {}
    r = _rng("FICE", seed, stype)
    if ice is None:
        fice = (r.random(n) < 0.2).astype(np.float64)
    else:
        fice = np.full(n, 1.0 if ice else 0.0)
    ts = _rng("TSUR", seed, stype).uniform(271.0, 303.0, n)
    ts = np.where(fice == 1.0, _rng("TSUR", seed + 1, stype).uniform(255.0, 273.15, n), ts)
    out["FICE"], out["TSUR"] = fice, ts
    out["ALBE"] = _rng("ALBE", seed, stype).uniform(0.05, 0.8, n)
    out["CMOI"] = _rng("CMOI", seed, stype).uniform(8e-4, 2.5e-3, n)
    out["CHEA"] = _rng("CHEA", seed, stype).uniform(8e-4, 2.5e-3, n)
    out["CMOM"] = _rng("CMOM", seed, stype).uniform(8e-4, 2.5e-3, n)
    return out


def fare(n, T, seed=BASE_SEED):
    """FARE ~ Dirichlet(1,...,1) over the T surface types."""
    if T == 1:
        return [np.ones(n)]
    f = _rng("FARE", seed).dirichlet(np.ones(T), n)
    return [np.ascontiguousarray(f[:, i]) for i in range(T)]


def corrections(n, seed=BASE_SEED + 5):
    """corr ~ N(0, 1e-5) kg m-2 s-1 per (month, cell); Fortran corrections(1,12,n) = [n][12]."""
    return np.ascontiguousarray(_rng("CORR", seed).normal(0.0, 1e-5, (n, 12)))


VARIANTS = {
    # which_* per variant for a water surface type (ice types take HLAT 'ice')
    "CCLM": dict(qsur="CCLM", meva="CCLM", hlat="water", hsen="CCLM", mom="CCLM", rbbr="StBo"),
    "MOM5": dict(qsur="CCLM", meva="MOM5", hlat="water", hsen="MOM5", mom="MOM5", rbbr="StBo"),
    "RCO": dict(qsur="none", meva="RCO", hlat="water", hsen="RCO", mom="RCO", rbbr="StBo"),
}


@dataclass
class Case:
    name: str
    lf: LocalFields
    num_surface_types: int
    methods: dict
    corrections: tuple = None  # (init_date, corr[n][12])
    averages: list = field(default_factory=list)
    regrid: dict = None
    outputs: list = field(default_factory=list)  # (s, g, name) written by the path

    @property
    def grid_size(self):
        return self.lf.grid_size


def build_case(variant="CCLM", n=4096, T=1, bias=False, sep_grids=None, rsdr=False,
               per_type=None, seed=BASE_SEED, init_date=19610101, device=None, data=None):
    """One configuration.

    variant   : CCLM | MOM5 | RCO (the method set of every surface type)
    T         : surface types; type 2 is ice (HLAT 'ice'), FARE Dirichlet over types
    sep_grids : None -> u/v grids ARE the t grid (aliased arrays);
                (n_u, n_v) -> separate u and v grids with their own arrays
    per_type  : {surface_type: {which_*: method}} overrides ('zero', 'copy', 'none', ...)
    data      : pre-generated {name: array} to reuse (bench: inputs shared by variants)
    """
    nu, nv = (n, n) if sep_grids is None else sep_grids
    lf = LocalFields([n, nu, nv], device=device)
    grids = (1,) if sep_grids is None else (1, 2, 3)
    gsize = {1: n, 2: nu, 3: nv}
    put = lf.set_array if device is None else (lambda name, s, g, a, allocated=True: lf.set_array(
        name, s, g, _to_dev(a, device), allocated))

    # bottom fields per surface type
    bottom = {}
    for s in range(1, T + 1):
        for g in grids:
            if data is not None and g == 1 and T == 1:
                bottom[(s, g)] = data
            else:
                bottom[(s, g)] = bottom_fields(gsize[g], s, seed + 10 * (g - 1),
                                               ice=(s == 2) if T >= 2 else None)
    # atmosphere fields: type 0, distributed to every surface type (flux_calculator.F90:474)
    for g in grids:
        if data is not None and g == 1:
            src = data
        else:
            src = atmos_fields(gsize[g], seed + 10 * (g - 1), tsur=bottom[(1, g)]["TSUR"])
        for name in ATMOS_VARS:
            put(name, 0, g, src[name])
            lf.distribute_input_field(name, g, 0, 0, T)
    fa = {g: fare(gsize[g], T, seed + 10 * (g - 1)) for g in grids}
    for s in range(1, T + 1):
        for g in grids:
            b = bottom[(s, g)]
            for name in ("TSUR", "FICE", "ALBE", "CMOI", "CHEA", "CMOM"):
                put(name, s, g, b[name])
            put("FARE", s, g, fa[g][s - 1])
    if sep_grids is None:  # u/v grids are the t grid: every slot aliases the t-grid array
        for (s, g, name), a in list(lf.field.items()):
            if g == 1:
                for gg in (2, 3):
                    lf.field[(s, gg, name)] = a
                    lf.allocated.discard((s, gg, name))

    meth = VARIANTS[variant]
    methods = {k: [] for k in ("which_spec_vapor_surface_t", "which_spec_vapor_surface_u",
                               "which_spec_vapor_surface_v", "which_flux_mass_evap",
                               "which_flux_heat_latent", "which_flux_heat_sensible",
                               "which_flux_momentum", "which_flux_radiation_blackbody")}
    for s in range(1, T + 1):
        m = dict(which_spec_vapor_surface_t=meth["qsur"], which_spec_vapor_surface_u=meth["qsur"],
                 which_spec_vapor_surface_v=meth["qsur"], which_flux_mass_evap=meth["meva"],
                 which_flux_heat_latent="ice" if (T >= 2 and s == 2) else meth["hlat"],
                 which_flux_heat_sensible=meth["hsen"], which_flux_momentum=meth["mom"],
                 which_flux_radiation_blackbody=meth["rbbr"])
        if per_type and s in per_type:
            m.update(per_type[s])
        for k, v in m.items():
            methods[k].append(v)

    # outputs, as do_prepare_calculation would allocate them (prepare:36-42)
    outputs = []

    def out(name, s, g, table):
        mth = methods[table][s - 1]
        if mth == "none":
            return
        if mth == "copy":
            lf.alias(name, s, g, 1)
            return
        if sep_grids is None and g != 1 and lf.associated(s, 1, name):
            lf.field[(s, g, name)] = lf.field[(s, 1, name)]  # the u/v grid is the t grid
            lf.allocated.discard((s, g, name))
            outputs.append((s, 1, name))
            return
        if not lf.associated(s, g, name) or (s, g, name) not in lf.allocated:
            lf.allocate_localvar(name, s, g, value=np.nan if device is None else float("nan"))
        outputs.append((s, g, name))

    for s in range(1, T + 1):
        for g, t in ((1, "which_spec_vapor_surface_t"), (2, "which_spec_vapor_surface_u"),
                     (3, "which_spec_vapor_surface_v")):
            if methods[t][s - 1] == "none" and methods["which_flux_mass_evap"][s - 1] in ("RCO",):
                # prepare:107 asks for QSUR even for RCO: keep an (unused) array associated
                if not lf.associated(s, g, "QSUR"):
                    if sep_grids is None and g != 1:
                        lf.field[(s, g, "QSUR")] = lf.field[(s, 1, "QSUR")]
                    else:
                        lf.allocate_localvar("QSUR", s, g, value=0.0)
                continue
            out("QSUR", s, g, t)
    for s in range(1, T + 1):
        out("MEVA", s, 1, "which_flux_mass_evap")
        out("HLAT", s, 1, "which_flux_heat_latent")
        out("HSEN", s, 1, "which_flux_heat_sensible")
        out("RBBR", s, 1, "which_flux_radiation_blackbody")
        out("UMOM", s, 2, "which_flux_momentum")
        out("VMOM", s, 3, "which_flux_momentum")
        if rsdr:
            lf.allocate_localvar("RSDR", s, 1, value=np.nan if device is None else float("nan"))
            outputs.append((s, 1, "RSDR"))

    averages = []
    if T >= 2:  # type-0 outputs averaged over surface types (add_output_field, basic:222-227)
        for name, g, phase in (("RBBR", 1, PHASE_EARLY), ("TSUR", 1, PHASE_EARLY),
                               ("MEVA", 1, PHASE_NORMAL), ("HLAT", 1, PHASE_NORMAL),
                               ("HSEN", 1, PHASE_NORMAL), ("UMOM", 2, PHASE_NORMAL),
                               ("VMOM", 3, PHASE_NORMAL)):
            if all(lf.associated(s, g, name) for s in range(1, T + 1)):
                lf.allocate_localvar(name, 0, g, value=np.nan if device is None else float("nan"))
                averages.append((phase, g, name))
                outputs.append((0, g, name))

    corr = (init_date, corrections(n, seed + 5)) if bias else None
    return Case(name=f"{variant}_T{T}{'_bias' if bias else ''}{'_sep' if sep_grids else ''}",
                lf=lf, num_surface_types=T, methods=methods, corrections=corr, averages=averages,
                outputs=outputs)


def regrid_links(n_src, n_dst, seed, max_links=4):
    """A sparse_regridding_matrix (basic:117-122) in COO file order: every destination gets
    0..max_links links (empty rows included, repeated (src, dst) pairs possible), the links
    shuffled so that a row's links are scattered through the list; 1-based indices."""
    r = np.random.Generator(np.random.PCG64([seed, 97]))
    per = r.integers(0, max_links + 1, n_dst)
    dst = np.repeat(np.arange(1, n_dst + 1, dtype=np.int32), per)
    src = r.integers(1, n_src + 1, dst.shape[0]).astype(np.int32)
    w = r.uniform(0.0, 1.0, dst.shape[0])
    order = r.permutation(dst.shape[0])
    return (np.ascontiguousarray(src[order]), np.ascontiguousarray(dst[order]), np.ascontiguousarray(w[order]))


def build_regrid_case(variant="CCLM", n=300, sep_grids=(310, 290), T=2, bias=False, seed=BASE_SEED):
    """A case on separate t/u/v grids with all four regridding matrices in use
    (flux_calculator.F90:330-337, do_regridding basic:463-522): QSUR computed on t and put to
    the u and v grids (t->u, t->v; QSUR(u/v) methods 'none'), UMOM computed on u and put to t
    (u->t), VMOM on v put to t (v->t)."""
    case = build_case(variant, n=n, T=T, bias=bias, sep_grids=sep_grids, seed=seed)
    nt, nu, nv = case.grid_size
    case.regrid = {"matrices": {0: regrid_links(nu, nt, seed + 1), 1: regrid_links(nv, nt, seed + 2),
                                2: regrid_links(nt, nu, seed + 3), 3: regrid_links(nt, nv, seed + 4)}}
    lf = case.lf
    for s in range(1, T + 1):
        if case.methods["which_spec_vapor_surface_t"][s - 1] == "CCLM":
            case.methods["which_spec_vapor_surface_u"][s - 1] = "none"
            case.methods["which_spec_vapor_surface_v"][s - 1] = "none"
            lf.put_to[(s, 1, "QSUR")] = 2 | 4
        lf.put_to[(s, 2, "UMOM")] = 1
        lf.put_to[(s, 3, "VMOM")] = 1
        for name in ("UMOM", "VMOM"):
            lf.allocate_localvar(name, s, 1, value=np.nan)
            case.outputs.append((s, 1, name))
    case.name = f"{case.name}_regrid"
    return case


def as_dtype(case, dtype):
    """The same case with every field array rounded once to dtype (aliases kept): the fp32
    variant of SURVEY.md 8d config 5, and (as_dtype(c32, 'float64')) the exactly widened
    inputs its fp64 oracle runs on."""
    import copy

    new = copy.copy(case)
    new.lf = case.lf.astype(dtype)
    new.name = f"{case.name}_{dtype}"
    return new


def _to_dev(a, device):
    import torch

    return torch.as_tensor(a, dtype=torch.float64).to(device)


def inputs_for_bench(n, seed=BASE_SEED):
    """One set of input arrays (T=1) shared by the CCLM, MOM5 and RCO cases."""
    d = bottom_fields(n, 1, seed)
    d.update(atmos_fields(n, seed, tsur=d["TSUR"]))
    return d


class SyntheticCoupler:
    """A stand-in for OASIS3-MCT in fcx.driver: get() fills a received field with the
    seeded synthetic values of its variable (SURVEY.md 8d distributions) for the field's
    grid, surface type and time; put() records a copy of every sent field.

    Names are the reference's R/S + letter + VAR + NN (basic:150, 267)."""

    def __init__(self, grid_size, num_surface_types, seed=BASE_SEED):
        self.grid_size = list(grid_size)
        self.T = max(int(num_surface_types), 1)
        self.seed = seed
        self.sent = {}  # (name, time) -> ndarray
        self.grid_of = {}  # received name -> which_grid
        self._cache = {}

    def _values(self, g, time):
        key = (g, time)
        if key not in self._cache:
            n = self.grid_size[g - 1]
            s = self.seed + 7919 * g + (time // 60)
            bottom = [bottom_fields(n, st, s) for st in range(1, self.T + 1)]
            atm = atmos_fields(n, s, tsur=bottom[0]["TSUR"])
            fa = fare(n, self.T, s)
            for st in range(self.T):
                bottom[st]["FARE"] = fa[st]
            self._cache[key] = (atm, bottom)
        return self._cache[key]

    def get(self, name, time, out, which_grid=None):
        var, st = name[2:6], int(name[6:8])
        g = which_grid or self.grid_of.get(name, 1)
        atm, bottom = self._values(g, time)
        src = atm if st == 0 else bottom[min(st, self.T) - 1]
        if var in src:
            vals = src[var]
        elif var in atm:
            vals = atm[var]
        else:
            vals = bottom[min(max(st, 1), self.T) - 1].get(var)
        if vals is None:
            raise KeyError(f"synthetic coupler has no values for {name}")
        if hasattr(out, "copy_"):
            import torch

            out.copy_(torch.as_tensor(vals, dtype=out.dtype))
        else:
            out[:] = vals

    def put(self, name, time, array):
        a = array if isinstance(array, np.ndarray) else array.detach().cpu().numpy()
        self.sent[(name, time)] = np.array(a, copy=True)

    @classmethod
    def for_setup(cls, setup, seed=BASE_SEED):
        c = cls(setup.grid_size, setup.num_surface_types, seed)
        c.grid_of = {f.name: f.which_grid for f in setup.input_field}
        return c
