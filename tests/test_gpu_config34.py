"""BASELINE.json configs 3 and 4 at their real sizes, through exactly the bench's path
(fcx.workload.Workload: the three variants over one set of inputs, engine-owned
tile-blocked mirrors uploaded once, the exchange -> atmosphere accumulation fused into the
flux kernels, HBM-resident steps).

* config 3: 10M cells, CCLM + MOM5 + RCO: EVERY output cell against the C oracle run over
  the whole grid on the host cores (fco_step_threads; 1e-10 mixed, tests/parity.py), every
  cell finite, and every atmosphere cell bit-identical to the sequential SCRIP sum of the
  GPU's own fluxes.
* config 4: the 40M-cell grid as 8 APPLE shards (decomp_def.F90:23-31) in one process, the
  shards' boundary slots summed (what the RCCL all-reduce does) and finished: every flux
  cell of every shard against the oracle; every atmosphere cell against the sequential sum
  over the global grid -- interior cells bit-identical, the shared boundary cells (two
  partial sums) within 1e-12 mixed.

Each full-grid comparison writes its per-field report (mixed error, plain max relative
error, cells above 1e-10 by either measure, bit-identical cells) to gpurun_out/parity/.
Reference: flux_calculator_calculate.F90:25-385.
"""
import numpy as np
import pytest

import oracle_lib
from parity import cell_report, conditioned_full, write_report

pytestmark = pytest.mark.gpu

from fcx.workload import ATM_FIELDS, VARIANTS, Workload  # noqa: E402
from fcx.synthetic import build_case  # noqa: E402

T_STEP = 3600


def check_full(case, got, label, report):
    """Every cell of every output against the oracle over the whole grid; the report is
    accumulated under `label` and the gate (1e-10 mixed) applied, with the conditioning
    allowance of parity.conditioned_full for the cells over it."""
    ref = oracle_lib.run_case_threads(case, current_step_time=T_STEP)
    rep = cell_report(got, ref)
    cond = conditioned_full(case, got, ref, T_STEP, label)
    for k, v in cond.items():
        rep[k]["conditioned"] = v
    report[label] = rep
    del ref


@pytest.mark.timeout(300)
@pytest.mark.parametrize("path", ["run_group", "run"])
@pytest.mark.parametrize("atmos_map", ["random", "periodic"])
def test_config3_bench_path_10M(atmos_map, path):
    """The bench's exact path at config 3's size: the random-run atmosphere map (segments
    cross the wave tiles: halo tiles complete them) and the periodic one (none do).
    run_group is the bench's timed step -- the three variants in ONE
    cells_atmos_group_kernel launch (fcx_run_group) -- checked here against the oracle
    directly, not only against the per-engine launches; run is one launch per engine."""
    wl = Workload(10_000_000, variants=VARIANTS, atmos_map=atmos_map)
    try:
        if path == "run_group":
            wl.run_group(T_STEP)
            assert [e.last_group_size() for e in wl.engines] == [len(VARIANTS)] * len(VARIANTS)
        else:
            wl.run(T_STEP)
            assert [e.last_group_size() for e in wl.engines] == [0] * len(VARIANTS)
        wl.download()
        report = {}
        for v, case, outs in zip(wl.variants, wl.cases, wl.atm_outs):
            got = {k: np.array(case.lf.field[k], copy=True) for k in case.outputs}
            for k, x in got.items():
                assert np.isfinite(x).all(), (v, k)
            check_full(case, got, f"config3 {v}", report)
            for name, g in ATM_FIELDS:
                flux = got[(1, g, name)] if (1, g, name) in got else np.asarray(case.lf.field[(1, g, name)])
                want = oracle_lib.atmos_accumulate(wl.la.atmos_index, wl.la.weight, flux, wl.la.n_atmos)
                np.testing.assert_array_equal(outs[name][: wl.la.n_atmos], want, err_msg=f"{v} {name}")
        write_report(f"config3_{atmos_map}_{path}", report)
    finally:
        wl.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("atmos_map", ["random", "periodic"])
def test_config4_40M_eight_shards(atmos_map):
    import torch
    from fcx.parallel import BlockedRandomAtmosMap, PeriodicAtmosMap

    # 40M + 40 cells: shards of 5,000,005 cells, so the shard ends fall inside atmosphere cells
    # of the periodic map (16 exchange cells = 4 atmosphere cells) and the boundary exchange
    # has work to do (with 5M-cell shards every boundary would coincide with a cell edge)
    n_global, world = 40_000_040, 8
    shards = [Workload(n_global, r, world, variants=VARIANTS, atmos_map=atmos_map) for r in range(world)]
    try:
        for wl in shards:
            wl.run(T_STEP)
        total = sum(wl.shared for wl in shards)  # the all-reduce (sum) of the boundary slots
        for wl in shards:
            wl.shared.copy_(total)
            wl.finish()
            wl.download()
        torch.cuda.synchronize()
        for wl in shards:
            assert float(wl.shared.abs().sum()) == 0.0
        gmap = (PeriodicAtmosMap() if atmos_map == "periodic" else BlockedRandomAtmosMap()).global_map(n_global)
        report = {}
        for i, v in enumerate(VARIANTS):
            fluxes = {name: np.empty(n_global) for name, _ in ATM_FIELDS}
            atm = {name: np.full(gmap.n_atmos, np.nan) for name, _ in ATM_FIELDS}
            for r, wl in enumerate(shards):
                case, la = wl.cases[i], wl.la
                got = {k: np.asarray(case.lf.field[k]) for k in case.outputs}
                check_full(case, got, f"config4 {v} shard {r}", report)
                for name, g in ATM_FIELDS:
                    fluxes[name][wl.offset: wl.offset + wl.n] = np.asarray(case.lf.field[(1, g, name)])
                    part = wl.atm_outs[i][name][: la.n_atmos]
                    seg = atm[name][la.atmos_offset: la.atmos_offset + la.n_atmos]
                    both = ~np.isnan(seg)  # a boundary cell both neighbours hold: the same value
                    np.testing.assert_array_equal(seg[both], part[both], err_msg=f"{v} {name} boundary r{r}")
                    seg[:] = part
            shared_cells = np.array(sorted({wl.la.atmos_offset for wl in shards if wl.la.left >= 0}), dtype=np.int64)
            assert shared_cells.size >= world // 2, "the shard boundaries must cut atmosphere cells"
            for name, _ in ATM_FIELDS:
                want = oracle_lib.atmos_accumulate(gmap.atmos_index, gmap.weight, fluxes[name], gmap.n_atmos)
                got = atm[name]
                assert np.isfinite(got).all(), (v, name)
                interior = np.ones(gmap.n_atmos, bool)
                interior[shared_cells] = False
                np.testing.assert_array_equal(got[interior], want[interior], err_msg=f"{v} {name} interior")
                if shared_cells.size:
                    scale = max(np.abs(want).max(), 1e-300)
                    err = np.abs(got[shared_cells] - want[shared_cells]) / np.maximum(
                        np.abs(want[shared_cells]), 1e-6 * scale)
                    assert err.max() <= 1e-12, (v, name, err.max())
        write_report(f"config4_{atmos_map}", report)
    finally:
        for wl in shards:
            wl.close()
