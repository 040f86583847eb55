"""An empty task: a rank whose `task` range holds no exchange cells (io:101-104 sets
grid_size = 0 and grid_offset = 0 for it) still runs every per-step routine of the
reference (calc:25-385 loop over zero cells).  The engine must commit and step over a
zero-cell grid without launching a kernel and without touching memory, for one and several
surface types, on host arrays and through the drop-in per-call sequence."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

fcx = pytest.importorskip("fcx")
from fcx.basic import PHASE_ALL, PHASE_EARLY, PHASE_NORMAL  # noqa: E402
from fcx.engine import Engine  # noqa: E402
from fcx.synthetic import build_case  # noqa: E402

STEP_T = 3600 * 24 * 31


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
@pytest.mark.parametrize("T", [1, 3])
def test_empty_task_steps(variant, T):
    case = build_case(variant, n=0, T=T, bias=True)
    assert all(case.lf.field[k].size == 0 for k in case.outputs)
    eng = Engine(case.lf, case.num_surface_types, case.methods, corrections=case.corrections,
                 averages=case.averages, regrid=case.regrid)
    for ph in (PHASE_EARLY, PHASE_NORMAL, PHASE_ALL):
        eng.step(ph, STEP_T)
    eng.close()


def test_empty_and_one_cell_tasks_side_by_side():
    """An empty rank's engine next to a live one in the same process: the live engine's
    results are those it gives alone (the empty engine shares no state with it)."""
    live = build_case("MOM5", n=1, T=1, bias=True)
    e_live = Engine(live.lf, live.num_surface_types, live.methods, corrections=live.corrections,
                    averages=live.averages)
    e_live.step(PHASE_ALL, STEP_T)
    alone = {k: np.array(live.lf.field[k], copy=True) for k in live.outputs}
    for k in live.outputs:
        live.lf.field[k][:] = np.nan
    empty = build_case("MOM5", n=0, T=1, bias=True)
    e_empty = Engine(empty.lf, empty.num_surface_types, empty.methods,
                     corrections=empty.corrections, averages=empty.averages)
    e_empty.step(PHASE_ALL, STEP_T)
    e_live.step(PHASE_ALL, STEP_T)
    for k in live.outputs:
        np.testing.assert_array_equal(live.lf.field[k], alone[k], err_msg=str(k))
    e_empty.close()
    e_live.close()
