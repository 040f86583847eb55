"""Parity metric of SURVEY.md 8d (fp64): per field
    max_j |x - x_ref| / max(|x_ref[j]|, 1e-6 * ||x_ref||_inf)  <=  1e-10
(mixed abs/rel, normalised per field: pure elementwise relative error is ill-posed where
q_s - q_a or T_s - T_a*EF cancel).  Integer/index results are compared bit-exactly.
"""
import numpy as np

FP64_TOL = 1e-10
# fp32 variant ("fp32: report only").  Its error is reported against
# the fp64 oracle on the same (float32-rounded) inputs; the gate below is a sanity bound on
# the norm-wise error max|x - ref| / ||ref||_inf, not a parity claim.
FP32_NORM_GATE = 1e-5


def mixed_error(x, ref):
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    if x.shape != ref.shape:
        raise AssertionError(f"shape {x.shape} != {ref.shape}")
    if ref.size == 0:
        return 0.0
    if not np.all(np.isfinite(x) == np.isfinite(ref)):
        return np.inf
    fin = np.isfinite(ref)
    if not fin.any():
        return 0.0
    scale = np.maximum(np.abs(ref[fin]), 1e-6 * np.max(np.abs(ref[fin])))
    scale = np.where(scale == 0.0, 1.0, scale)
    return float(np.max(np.abs(x[fin] - ref[fin]) / scale))


def assert_parity(got: dict, ref: dict, tol=FP64_TOL, label=""):
    worst = {}
    for key, r in ref.items():
        e = mixed_error(got[key], r)
        worst[key] = e
    bad = {k: v for k, v in worst.items() if not v <= tol}
    assert not bad, f"{label}: fields over tolerance {tol}: {bad}; " + "; ".join(
        _where(got[k], ref[k], tol, k) for k in bad)
    return worst


def _where(x, ref, tol, key):
    """the failing cells of one field (count, first indices and values) for the message"""
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    fin = np.isfinite(ref)
    top = np.max(np.abs(ref[fin])) if fin.any() else 1.0
    scale = np.maximum(np.abs(ref), 1e-6 * top)
    with np.errstate(invalid="ignore"):
        off = ~(np.abs(x - ref) <= tol * np.where(scale == 0.0, 1.0, scale)) & ~(np.isnan(x) & np.isnan(ref))
    idx = np.nonzero(off)[0]
    return (f"{key}: {idx.size} of {x.size} cells, first {idx[:8].tolist()}, "
            f"got {x[idx[:4]].tolist()} want {ref[idx[:4]].tolist()}")


def norm_error(x, ref):
    """max_j |x - x_ref| / ||x_ref||_inf (norm-wise; the fp32 report)."""
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    if ref.size == 0:
        return 0.0
    if not np.all(np.isfinite(x) == np.isfinite(ref)):
        return np.inf
    fin = np.isfinite(ref)
    top = np.max(np.abs(ref[fin])) if fin.any() else 0.0
    return float(np.max(np.abs(x[fin] - ref[fin])) / (top if top > 0 else 1.0))


def cell_report(got: dict, ref: dict):
    """Per field, over every cell: the mixed error (the gate), the plain elementwise max
    relative error, the counts of cells above 1e-10 by either measure, the bit-identical
    cells.  {"s:g:NAME": {...}}"""
    rep = {}
    for key, r in ref.items():
        g = np.asarray(got[key], dtype=np.float64)
        r = np.asarray(r, dtype=np.float64)
        fin = np.isfinite(r)
        top = float(np.max(np.abs(r[fin]))) if fin.any() else 0.0
        d = np.abs(g - r)
        nz = np.abs(r) > 0
        rel = np.zeros_like(r)
        np.divide(d, np.abs(r), out=rel, where=nz)
        rel[~nz & (d > 0)] = np.inf
        scale = np.maximum(np.abs(r), 1e-6 * top)
        mixed = np.divide(d, scale, out=np.zeros_like(r), where=scale > 0)
        rep["%d:%d:%s" % key] = {
            "cells": int(r.size), "mixed": mixed_error(g, r), "max_rel": float(rel.max(initial=0.0)),
            "cells_rel_gt_1e-10": int((rel > FP64_TOL).sum()),
            "cells_mixed_gt_1e-10": int((mixed > FP64_TOL).sum()),
            "bit_identical_cells": int((g == r).sum())}
    return rep


def write_report(name, rep):
    """gpurun_out/<name>.json (copied into profiles/ by the round's evidence scripts)."""
    import json
    import os

    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "parity")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, name + ".json"), "w") as f:
        json.dump(rep, f, indent=1)


def error_report(got: dict, ref: dict):
    """{field: (norm-wise error, mixed error, elementwise max relative error)}"""
    out = {}
    for key, r in ref.items():
        g = np.asarray(got[key], dtype=np.float64)
        r = np.asarray(r, dtype=np.float64)
        nz = np.abs(r) > 0
        rel = float(np.max(np.abs(g[nz] - r[nz]) / np.abs(r[nz]))) if nz.any() else 0.0
        out[key] = (norm_error(g, r), mixed_error(g, r), rel)
    return out


def sample_case(case, idx):
    """The case restricted to the cells idx (aliasing kept, the bias corrections sliced): for
    re-running the oracle on a few cells of a large grid.  u/v grids = t grid only."""
    from fcx.synthetic import build_case

    idx = np.asarray(idx)
    small = build_case(case.name.split("_")[0], n=idx.size, T=case.num_surface_types)
    remap = {}
    for key, a in case.lf.field.items():
        if id(a) not in remap:
            remap[id(a)] = np.ascontiguousarray(np.asarray(a)[idx])
        small.lf.field[key] = remap[id(a)]
    small.methods = {k: list(v) for k, v in case.methods.items()}
    if case.corrections is not None:
        init_date, corr = case.corrections
        corr = np.asarray(corr)
        small.corrections = (init_date, np.ascontiguousarray(corr[idx] if corr.shape[0] != 12 else corr[:, idx]))
    else:
        small.corrections = None
    return small


def conditioned_full(case, got, ref, t, label, tol=FP64_TOL, ulps=16, trials=8):
    """The SURVEY 8d gate over every cell, with the allowance of
    tests/test_gpu_random_configs.py::conditioned_parity for ill-conditioned cells: a cell
    over the gate (where HSEN = F c_p (T_s - T_a EF) or MEVA = F (q_s - q_a) cancel, one ulp of
    the device's pow / exp against the host libm's moves it by more than 1e-10 of its value)
    passes if the GPU is within twice the oracle's own movement when the cell's inputs are
    perturbed by `ulps` ulps (eight seeded perturbations, random signs per cell); any other
    error fails.  Returns {field: {"cells_over_gate", "max_err_over_movement"}}."""
    import oracle_lib

    bad = {}
    for key, r in ref.items():
        g = np.asarray(got[key], dtype=np.float64)
        r = np.asarray(r, dtype=np.float64)
        if not np.all(np.isfinite(g) == np.isfinite(r)):
            raise AssertionError(f"{label}: {key} finite/non-finite cells differ")
        fin = np.isfinite(r)
        top = float(np.max(np.abs(r[fin]))) if fin.any() else 0.0
        scale = np.maximum(np.abs(r), 1e-6 * top)
        with np.errstate(invalid="ignore", divide="ignore"):
            off = fin & (np.abs(g - r) > tol * np.where(scale == 0.0, 1.0, scale))
        if off.any():
            bad[key] = np.nonzero(off)[0]
    out = {"%d:%d:%s" % k: {"cells_over_gate": int(v.size)} for k, v in bad.items()}
    if not bad:
        return out
    idx = np.unique(np.concatenate(list(bad.values())))
    if idx.size > 10_000:
        raise AssertionError(f"{label}: {idx.size} cells over the gate")
    small = sample_case(case, idx)
    base = oracle_lib.run_case(small, "c", current_step_time=t)
    move = {k: np.zeros(idx.size) for k in bad}
    eps = float(np.finfo(np.float64).eps)
    outs = {id(small.lf.field[k]) for k in small.outputs}
    for trial in range(trials):
        c = sample_case(case, idx)
        rng = np.random.default_rng([trial, 99])
        seen = set()
        for a in c.lf.field.values():
            if id(a) in outs or id(a) in seen or not isinstance(a, np.ndarray) or a.dtype != np.float64:
                continue
            seen.add(id(a))
            a *= 1.0 + ulps * eps * rng.choice([-1.0, 1.0], a.shape)
        rp = oracle_lib.run_case(c, "c", current_step_time=t)
        for k in bad:
            move[k] = np.fmax(move[k], np.abs(np.asarray(rp[k]) - np.asarray(base[k])))
    pos = {int(j): i for i, j in enumerate(idx)}
    problems = []
    for k, cells in bad.items():
        sel = np.array([pos[int(j)] for j in cells])
        assert np.array_equal(np.asarray(base[k])[sel], np.asarray(ref[k])[cells]), (label, k, "oracle on the sample")
        err = np.abs(np.asarray(got[k])[cells] - np.asarray(ref[k])[cells])
        allow = 2.0 * move[k][sel]
        ratio = float(np.max(err / np.where(allow > 0, allow, np.inf))) if cells.size else 0.0
        out["%d:%d:%s" % k]["max_err_over_movement"] = ratio
        out["%d:%d:%s" % k]["cells"] = [int(x) for x in cells[:16]]
        if np.any(err > allow):
            problems.append(f"{k}: {int(np.sum(err > allow))} of {cells.size} cells over the gate are not explained "
                            f"by input rounding (first {cells[err > allow][:4].tolist()})")
    if problems:
        raise AssertionError(f"{label}: " + "; ".join(problems))
    return out
