"""The whole reference time loop on the GPU: flux_calculator.nml -> set-up (fcx.setup,
flux_calculator.F90 STEP 1.3-1.7) -> engine -> coupling steps in the reference order
(fcx.driver, F90 STEP 2) against a synthetic coupler, compared put by put with the same
loop driven by the C oracle (tests/oracle_lib.OracleEngine) on an identical set-up.
Covers received-field regridding (t -> u, t -> v), calculated-field regridding (u -> t,
v -> t), constant and -2e20 inputs, 'copy' methods, uniform aliases, averaged and
default-valued sends, and the monthly bias corrections across steps."""
import numpy as np
import pytest

import namelists
from namelists import regrid_matrices
import oracle_lib
from parity import FP64_TOL, mixed_error

pytestmark = pytest.mark.gpu

from fcx import driver  # noqa: E402
from fcx.setup import setup_from_namelist  # noqa: E402
from fcx.synthetic import SyntheticCoupler, corrections  # noqa: E402

GRIDS = (3001, 2999, 3011)


@pytest.mark.parametrize("which, mype, bias", [("MOM5_BALTIC", 0, True), ("CCLM_REGRID", 1, False)])
def test_time_loop_matches_oracle(which, mype, bias):
    text = getattr(namelists, which)
    regrid = regrid_matrices(GRIDS)
    corr = (20000101, corrections(GRIDS[0])) if bias else None
    # t = 0, 600, 1200 s (MOM5) / 0, 3600 s: the month comes from init_date + time

    s_gpu = setup_from_namelist(text, mype=mype, grid_size=GRIDS)
    eng = s_gpu.engine(corrections=corr, regrid=regrid)
    c_gpu = SyntheticCoupler.for_setup(s_gpu)
    try:
        driver.run(s_gpu, eng, c_gpu)
    finally:
        eng.close()

    s_ref = setup_from_namelist(text, mype=mype, grid_size=GRIDS)
    c_ref = SyntheticCoupler.for_setup(s_ref)
    driver.run(s_ref, oracle_lib.OracleEngine(s_ref, corrections=corr, regrid=regrid), c_ref)

    assert c_gpu.sent.keys() == c_ref.sent.keys()
    steps = s_gpu.nml["num_timesteps"]
    assert len(c_ref.sent) == steps * len(s_ref.output_field)
    worst = {}
    for key, ref in c_ref.sent.items():
        got = c_gpu.sent[key]
        assert np.all(np.isfinite(ref)), key
        worst[key] = mixed_error(got, ref)
    bad = {k: v for k, v in worst.items() if not v <= FP64_TOL}
    assert not bad, f"{which}: puts over {FP64_TOL}: {bad}"
    # the loop really computed something: the averaged latent heat differs from each type's
    if which == "MOM5_BALTIC":
        t = 600
        assert not np.array_equal(c_ref.sent[("SAHLAT00", t)], c_ref.sent[("SMHLAT01", t)])
        assert np.all(c_ref.sent[("SMRLWU01", t)] == -5.0)
