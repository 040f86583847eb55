"""The host-bound fcx_step: caller arrays page-locked at commit (FCX_OPT_PIN_HOST) and the
step pipelined over cell chunks (FCX_OPT_PIPELINE_CHUNKS: H2D of chunk k+1, kernel of chunk k,
D2H of chunk k-1 on three streams).  Every chunking must give the bits of the sequential
upload/run/download step, and those are within tests/parity.py of the oracle."""
import numpy as np
import pytest

import oracle_lib
from parity import assert_parity

pytestmark = pytest.mark.gpu

from fcx.basic import PHASE_ALL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.parallel import local_atmos, synthetic_atmos_map  # noqa: E402
from fcx.synthetic import build_case  # noqa: E402

STEP_T = 3600 * 24 * 40


def run(case, options, atmos_n=None):
    """One fcx_step on fresh copies of the case's outputs; returns the outputs (and the
    atmosphere fields when atmos_n is given)."""
    for k in case.outputs:
        case.lf.field[k][:] = np.nan
    atmos, outs = None, None
    if atmos_n is not None:
        amap = synthetic_atmos_map(atmos_n)
        outs = {name: np.full(amap.n_atmos, np.nan) for name in ("MEVA", "HSEN", "UMOM")}
        atmos = {"local": local_atmos(amap, 0, 1),
                 "fields": [(2, 1, 1, "MEVA", outs["MEVA"]), (2, 1, 1, "HSEN", outs["HSEN"]),
                            (2, 1, 2, "UMOM", outs["UMOM"])]}
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, atmos=atmos, options=options)
    eng.step(PHASE_ALL, STEP_T)
    got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
    eng.close()
    if outs is not None:
        got.update({("atm", name): v.copy() for name, v in outs.items()})
    return got


def same_bits(a, b):
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=str(k))


@pytest.mark.parametrize("variant", ["CCLM", "RCO"])
def test_pipeline_chunkings_bit_identical(variant):
    case = build_case(variant, n=100_003, T=1, bias=True)
    seq = run(case, {"pipeline_chunks": 1, "pin_host": 0})
    for chunks in (2, 3, 8, 97):
        same_bits(run(case, {"pipeline_chunks": chunks}), seq)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(seq, ref, label=variant)


def test_pipeline_with_fused_atmosphere_accumulation():
    """Chunk boundaries cut atmosphere segments: carries + the fix-up after the last chunk."""
    n = 50_001
    case = build_case("MOM5", n=n, T=1, bias=True)
    seq = run(case, {"pipeline_chunks": 1}, atmos_n=n)
    for chunks in (4, 7):
        same_bits(run(case, {"pipeline_chunks": chunks}, atmos_n=n), seq)


def test_pipeline_generic_kernel_separate_grids_and_averages():
    case = build_case("CCLM", n=20_011, T=3, sep_grids=(19_997, 20_101), bias=True)
    seq = run(case, {"pipeline_chunks": 1})
    same_bits(run(case, {"pipeline_chunks": 5}), seq)
    same_bits(run(case, {"pipeline_chunks": 5, "pin_host": 0}), seq)
    ref = oracle_lib.run_case(case, "c", current_step_time=STEP_T)
    assert_parity(seq, ref, label="T3 sep")


def test_pinned_small_arrays_sharing_pages():
    """Many small arrays (several per page): merged page ranges are registered once."""
    case = build_case("CCLM", n=3_000, T=2, bias=True)
    a = run(case, {"pipeline_chunks": 2})
    b = run(case, {"pipeline_chunks": 1, "pin_host": 0})
    same_bits(a, b)
