#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run in the build container only).

The reference has no tests, fixtures or golden files, so the pins
are produced here from the reference itself:

  flux_*.npz   inputs and outputs of one coupling step, outputs computed by the REFERENCE
               flux_lib compiled unmodified from /root/reference/src/flux_lib with -r8
               semantics (oracle/_ref/libfco_ref.so, recipe in oracle/Makefile), driven in
               the call order of flux_calculator.F90:902-1008.  Cases with regridding
               matrices ("builder": "regrid") call the REFERENCE do_regridding
               (flux_calculator_basic.F90:463-522, compiled unmodified; oracle/_ref/
               libfco_ref_regrid.so via oracle/ref_regrid.F90) after each calc, as
               flux_calculator.F90:972-991 does; their matrices are stored as well.
  months.json  calendar months from the reference's own Python helper
               /root/reference/src/pyfort/datetime_helpers.py:get_current_date, imported
               by path (no bytecode written) -- the only Python in the reference path.

Usage:  python tests/golden/make_golden.py [stem ...]   (needs /root/reference and built
        oracles; with stems, only those fixtures are (re)written and the manifest is merged)
"""
import importlib.util
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "components.flux_calculator_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.dont_write_bytecode = True

from fcx.synthetic import build_case, build_regrid_case  # noqa: E402
import oracle_lib  # noqa: E402

STEP_T = 3600 * 24 * 31 + 7200  # 1961-02-01 02:00 -> February bias slice

# (file stem, build_case kwargs)
CASES = [
    ("cclm_t1", dict(variant="CCLM", n=512, T=1)),
    ("mom5_t1", dict(variant="MOM5", n=512, T=1)),
    ("rco_t1", dict(variant="RCO", n=512, T=1)),
    ("cclm_t1_bias", dict(variant="CCLM", n=512, T=1, bias=True)),
    ("mom5_t3_bias", dict(variant="MOM5", n=384, T=3, bias=True)),
    ("rco_t3", dict(variant="RCO", n=384, T=3)),
    ("cclm_t2_sep", dict(variant="CCLM", n=300, T=2, sep_grids=(310, 290))),
    ("cclm_t3_copy_bias", dict(variant="CCLM", n=256, T=3, bias=True, per_type={
        2: dict(which_flux_mass_evap="copy", which_flux_heat_latent="water"),
        3: dict(which_flux_mass_evap="zero", which_flux_heat_sensible="zero",
                which_flux_momentum="zero", which_flux_radiation_blackbody="zero")})),
    ("mixed_t2", dict(variant="CCLM", n=256, T=2, per_type={
        1: dict(which_flux_mass_evap="RCO", which_flux_momentum="RCO"),
        2: dict(which_flux_heat_sensible="RCO", which_flux_mass_evap="MOM5")})),
    # distribute_shortwave_radiation_flux (calc:347-364): RSDD/ALBA bound, RSDR per type
    ("cclm_t1_rsdr", dict(variant="CCLM", n=512, T=1, rsdr=True)),
    ("mom5_t3_rsdr_bias", dict(variant="MOM5", n=384, T=3, bias=True, rsdr=True)),
    ("rco_t2_rsdr", dict(variant="RCO", n=384, T=2, rsdr=True)),
]
# do_regridding after each calc, all four matrices (u->t, v->t, t->u, t->v)
REGRID_CASES = [
    ("cclm_t2_regrid", dict(variant="CCLM", n=300, sep_grids=(310, 290), T=2, bias=True)),
    ("mom5_t1_regrid", dict(variant="MOM5", n=257, sep_grids=(263, 251), T=1)),
]

MONTH_PROBES = [(19610101, 0), (19610101, 2678399), (19610101, 2678400), (20000228, 86400),
                (19991231, 86400), (19991231, 86399), (19000228, 86400), (20040229, 86400 * 366),
                (19610101, 3600 * 24 * 365 * 10), (20231015, 3600 * 17), (19701231, 2**31 - 1)]


def case_arrays(case):
    """Distinct arrays of a case keyed 's:g:NAME' (first slot that holds each array)."""
    seen, out, alias = {}, {}, {}
    for (s, g, name), a in sorted(case.lf.field.items()):
        key = f"{s}:{g}:{name}"
        if id(a) in seen:
            alias[key] = seen[id(a)]
        else:
            seen[id(a)] = key
            out[key] = np.asarray(a)
    return out, alias


def main():
    if oracle_lib.load("ref") is None or oracle_lib.load("ref_regrid") is None:
        raise SystemExit("oracle/_ref not built: make -C oracle ref basic-mod ref-regrid")
    only = set(sys.argv[1:])
    path = os.path.join(HERE, "manifest.json")
    manifest = json.load(open(path)) if only and os.path.exists(path) else {"step_time": STEP_T, "cases": {}}
    assert manifest["step_time"] == STEP_T
    for stem, kw, builder in ([(s, k, "case") for s, k in CASES] + [(s, k, "regrid") for s, k in REGRID_CASES]):
        if only and stem not in only:
            continue
        case = build_regrid_case(**kw) if builder == "regrid" else build_case(**kw)
        ref = oracle_lib.run_case(case, "ref", current_step_time=STEP_T, regrid=builder == "regrid")
        arrays, alias = case_arrays(case)
        payload = {f"in:{k}": v for k, v in arrays.items()}
        payload.update({f"out:{s}:{g}:{n}": v for (s, g, n), v in ref.items()})
        if case.corrections is not None:
            payload["corrections"] = case.corrections[1]
        for which, (src, dst, w) in (case.regrid or {}).get("matrices", {}).items():
            payload[f"regrid:{which}:src"], payload[f"regrid:{which}:dst"], payload[f"regrid:{which}:w"] = src, dst, w
        np.savez_compressed(os.path.join(HERE, f"flux_{stem}.npz"), **payload)
        manifest["cases"][stem] = {"build_case": kw, "builder": builder, "aliases": alias,
                                   "outputs": [f"{s}:{g}:{n}" for (s, g, n) in ref]}
        print(stem, len(arrays), "arrays,", len(ref), "outputs")
    if only:
        with open(path, "w") as f:
            json.dump(manifest, f, indent=1)
        return

    spec = importlib.util.spec_from_file_location(
        "datetime_helpers", "/root/reference/src/pyfort/datetime_helpers.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    months = []
    for init_date, secs in MONTH_PROBES:
        state = {"init_date": [init_date], "seconds": [secs]}
        mod.get_current_date(state)
        months.append({"init_date": init_date, "seconds": secs, "current_month": state["current_month"],
                       "current_date": state["current_date"]})
    manifest["months"] = months
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("months:", [(m["init_date"], m["seconds"], m["current_month"]) for m in months])


if __name__ == "__main__":
    main()
