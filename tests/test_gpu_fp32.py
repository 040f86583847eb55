"""fp32 variant of the cell pass ("fp32 and fp64 kernels ... report
max/percentile error vs oracle").  The fp32 engine (FCX_PRECISION_F32) stores and computes
in float; its outputs are compared with the fp64 oracle run on the SAME inputs (the float32
arrays widened exactly), so the reported error is the error of fp32 arithmetic alone.
Gate: tests/parity.py FP32_NORM_GATE on the norm-wise error (report, not a parity claim);
fp64 parity is tests/test_gpu_parity.py."""
import json
import os

import numpy as np
import pytest

import oracle_lib
from parity import FP32_NORM_GATE, error_report

pytestmark = pytest.mark.gpu

from fcx.basic import PHASE_ALL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.synthetic import as_dtype, build_case  # noqa: E402

STEP_T = 3600 * 24 * 31
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def run_fp32(case, options=None):
    c32 = as_dtype(case, "float32")
    c64 = as_dtype(c32, "float64")  # exactly the inputs the fp32 kernel saw
    ref = oracle_lib.run_case(c64, "c", current_step_time=STEP_T)
    eng = Engine(c32.lf, c32.num_surface_types, c32.methods, corrections=c32.corrections,
                 averages=c32.averages, options=options)
    eng.step(PHASE_ALL, STEP_T)
    got = {k: np.array(c32.lf.field[k], dtype=np.float64) for k in c32.outputs}
    eng.close()
    for k in c32.outputs:
        assert c32.lf.field[k].dtype == np.float32
    return got, ref


def check(got, ref, label):
    rep = error_report(got, ref)
    bad = {k: v for k, v in rep.items() if not v[0] <= FP32_NORM_GATE}
    assert not bad, f"{label}: fp32 norm-wise error over {FP32_NORM_GATE}: {bad}"
    return rep


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
@pytest.mark.parametrize("n", [1, 3, 4099, 32_768])
def test_fp32_t1_bias(variant, n):
    """T=1 specialised fp32 kernels (4 cells per lane, 16-B loads), ragged tails."""
    case = build_case(variant, n=n, T=1, bias=True)
    got, ref = run_fp32(case)
    rep = check(got, ref, f"{variant} n={n}")
    if n == 32_768:  # the config-5 report (merged into profiles/ by the bench tooling)
        os.makedirs(OUT, exist_ok=True)
        with open(os.path.join(OUT, f"fp32_error_{variant}.json"), "w") as f:
            json.dump({f"{s}:{g}:{name}": {"norm": e[0], "mixed": e[1], "max_rel": e[2]}
                       for (s, g, name), e in rep.items()}, f, indent=1)


@pytest.mark.parametrize("variant", ["CCLM", "RCO"])
def test_fp32_generic_t3_averages(variant):
    """Generic (VAR 0) fp32 kernel with surface types and type-0 averages."""
    got, ref = run_fp32(build_case(variant, n=3001, T=3, bias=True))
    check(got, ref, f"{variant} T=3")


def test_fp32_separate_grids():
    got, ref = run_fp32(build_case("MOM5", n=2003, T=2, sep_grids=(1999, 2011), bias=True))
    check(got, ref, "MOM5 separate u/v grids")


def test_fp32_one_cell_per_lane():
    got, ref = run_fp32(build_case("CCLM", n=1001, T=1, bias=True), options={"cells_per_thread": 1})
    check(got, ref, "CCLM cells_per_thread=1")


def test_fp32_device_resident_bytes_halved():
    """The fp32 engine moves half the bytes of the fp64 one for the same case."""
    torch = pytest.importorskip("torch")
    case = build_case("CCLM", n=10_000, T=1, bias=True, device="cuda:0")
    e64 = Engine(case.lf, 1, case.methods, corrections=case.corrections)
    b64 = e64.algorithmic_bytes(PHASE_ALL)
    e64.close()
    c32 = as_dtype(case, "float32")
    assert c32.lf.field[(1, 1, "TSUR")].dtype == torch.float32
    e32 = Engine(c32.lf, 1, c32.methods, corrections=c32.corrections)
    b32 = e32.algorithmic_bytes(PHASE_ALL)
    e32.run(PHASE_ALL, STEP_T)
    e32.synchronize()
    e32.close()
    assert b32 * 2 == b64
    assert torch.isfinite(c32.lf.field[(1, 1, "MEVA")]).all()
