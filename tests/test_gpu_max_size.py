"""The largest grid the suite holds: one MOM5 engine over 200,000,017 cells (a ragged count)
through the bench's path (fcx.workload.Workload: engine-owned tile-blocked mirrors, the
exchange -> atmosphere accumulation fused in, random runs crossing the wave tiles).  MOM5
reads 11 arrays, so its read pool holds 2.2e9 elements (17.6 GB): element offsets past 2^31
and byte offsets past 2^34 inside one allocation, tile strides in the tens of GB -- where a
32-bit index anywhere on the path would wrap.

The inputs are a 4,000,037-cell draw repeated with a different rotation per copy (drawing
200M cells of every field would take minutes of host time): every copy's cells differ, so a
result landing at an offset of whole copies is caught.  Checked: every output cell finite;
1,000,000 cells sampled over the grid plus the first and last 20,000 cells and the cells
around every 2^28-element boundary of the read pool against the C oracle run on those cells
(1e-10 mixed with the conditioning allowance, tests/parity.py); every atmosphere cell bit-identical to the sequential SCRIP
sum of the GPU's own fluxes.  Reference: flux_calculator_calculate.F90:25-385.
"""
import numpy as np
import pytest

import oracle_lib
from parity import conditioned_full, sample_case

pytestmark = pytest.mark.gpu

from fcx.synthetic import inputs_for_bench  # noqa: E402
from fcx.workload import ATM_FIELDS, Workload  # noqa: E402

N = 200_000_017
BASE = 4_000_037
T_STEP = 3600


def rotated_inputs(n, m):
    base = inputs_for_bench(m)
    out = {}
    copies = -(-n // m)
    for key, b in base.items():
        a = np.empty(n, dtype=b.dtype)
        for k in range(copies):  # copy k = the draw rotated by 7919 k cells (np.roll, in place)
            lo, hi = k * m, min(n, (k + 1) * m)
            r = (7919 * k) % m
            head = min(r, hi - lo)
            a[lo:lo + head] = b[m - r:m - r + head]
            a[lo + head:hi] = b[:hi - lo - head]
        out[key] = a
    return out


@pytest.mark.timeout(600)
def test_mom5_200M_cells_offsets_past_int32():
    wl = Workload(N, variants=("MOM5",), atmos_map="random", inputs=rotated_inputs(N, BASE))
    try:
        assert wl.n == N
        wl.run(T_STEP)
        wl.download()
        case = wl.cases[0]
        got = {k: np.asarray(case.lf.field[k]) for k in case.outputs}
        for k, x in got.items():
            assert np.isfinite(x).all(), k
        rng = np.random.default_rng(5)
        pool = 11 * N  # read-pool elements; cell offsets where the pool crosses 2^28-element marks
        marks = [(j << 28) // 11 for j in range(1, pool >> 28)]
        near = np.concatenate([np.arange(max(0, c - 200), min(N, c + 200)) for c in marks])
        idx = np.unique(np.concatenate([rng.integers(0, N, 1_000_000), np.arange(20_000),
                                        np.arange(N - 20_000, N), near]))
        small = sample_case(case, idx)
        ref = oracle_lib.run_case_threads(small, current_step_time=T_STEP)
        # (the gate with the conditioning allowance of the full-grid tests: a cell where HSEN or
        # MEVA cancels may sit above 1e-10 within twice the oracle's own input-rounding movement)
        conditioned_full(small, {k: v[idx] for k, v in got.items()}, ref, T_STEP, "MOM5 200M sampled")
        outs = wl.atm_outs[0]
        for name, g in ATM_FIELDS:
            want = oracle_lib.atmos_accumulate(wl.la.atmos_index, wl.la.weight, got[(1, g, name)], wl.la.n_atmos)
            np.testing.assert_array_equal(outs[name][: wl.la.n_atmos], want, err_msg=name)
    finally:
        wl.close()
