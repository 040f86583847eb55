"""fcx_run_group: several engines' fused T = 1 flux passes (one per bottom-model variant) as
ONE launch (cells_atmos_group_kernel).  Each tile runs the same code as the engine's own
launch, so every flux and every atmosphere value must be the bits of fcx_run of each engine;
engines that cannot join (several surface types, a grid cap) run as fcx_run inside the call."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from fcx.basic import PHASE_ALL  # noqa: E402
from fcx.workload import ATM_FIELDS, Workload  # noqa: E402


def outputs(wl):
    wl.download()
    got = {}
    for i, (case, outs) in enumerate(zip(wl.cases, wl.atm_outs)):
        for k in case.outputs:
            got[(i,) + k] = np.array(case.lf.field[k], copy=True)
        for name, _ in ATM_FIELDS:
            got[(i, "atm", name)] = np.array(outs[name], copy=True)
    return got


def run_both(n, variants, atmos_map, precision="f64", types=1, options=None, steps=2):
    import torch

    res = []
    for grouped in (False, True):
        wl = Workload(n, 0, 1, variants, types=types, precision=precision, atmos=True, atmos_map=atmos_map,
                      engine_options=options)
        for k in range(steps):
            if grouped:
                wl.run_group(3600 * k)
            else:
                wl.run(3600 * k)
        torch.cuda.synchronize()
        res.append(outputs(wl))
        wl.close()
    return res


def same_bits(a, b):
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=str(k))


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("atmos_map", ["random", "periodic"])
def test_group_launch_bit_identical(precision, atmos_map):
    """CCLM + MOM5 + RCO in one launch: random map (segments cross the wave tiles: halo
    tiles), periodic map (no crossing)."""
    a, b = run_both(300_007, ("CCLM", "MOM5", "RCO"), atmos_map, precision)
    same_bits(a, b)


@pytest.mark.parametrize("variants", [("RCO", "CCLM"), ("MOM5", "MOM5", "CCLM", "RCO")])
def test_group_orders_and_sizes(variants):
    """Any order, repeated variants, four members (the most one launch takes)."""
    a, b = run_both(70_001, variants, "random")
    same_bits(a, b)


def test_group_without_halo_uses_crossing_records():
    """Halo tiles off (FCX_OPT_ATMOS_HALO 0): the members' crossing records and fix-ups."""
    a, b = run_both(130_003, ("CCLM", "MOM5", "RCO"), "random", options={"atmos_halo": 0})
    same_bits(a, b)


@pytest.mark.parametrize("types", [2, 3])
def test_group_of_multi_type_launches(types):
    """Several surface types: the members' multi-type kernels (type-0 averages in registers,
    accumulated on the fly) in one launch."""
    a, b = run_both(50_021, ("CCLM", "MOM5", "RCO"), "random", types=types)
    same_bits(a, b)


def test_group_falls_back_for_engines_that_cannot_join():
    """A grid cap (not a one-trip fused launch) and fp32 at two surface types (no fused
    multi-type fp32 kernel): every engine runs as fcx_run inside fcx_run_group."""
    a, b = run_both(50_021, ("CCLM", "RCO"), "random", options={"max_blocks": 32})
    same_bits(a, b)
    a, b = run_both(50_021, ("CCLM", "RCO"), "random", precision="f32", types=2)
    same_bits(a, b)


def test_group_of_engines_on_different_streams_runs_them_apart():
    """Engines on different streams are not merged (each keeps its stream order)."""
    import torch
    from fcx.engine import Engine, run_group
    from fcx.synthetic import build_case

    n = 40_003
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    cases = [build_case(v, n=n, T=1, bias=True) for v in ("CCLM", "MOM5")]
    engines = [Engine(c.lf, 1, c.methods, corrections=c.corrections, stream=s.cuda_stream)
               for c, s in zip(cases, streams)]
    for e in engines:
        e.upload(PHASE_ALL)
    run_group(engines, PHASE_ALL, 7200)
    for e in engines:
        e.download(PHASE_ALL)
        e.synchronize()
    got = [{k: np.array(c.lf.field[k], copy=True) for k in c.outputs} for c in cases]
    for e in engines:
        e.run(PHASE_ALL, 7200)
        e.download(PHASE_ALL)
        e.synchronize()
    for c, g in zip(cases, got):
        for k in c.outputs:
            np.testing.assert_array_equal(g[k], np.asarray(c.lf.field[k]), err_msg=str(k))
    for e in engines:
        e.close()


def test_group_with_empty_atmosphere_cells():
    """A map with atmosphere cells that no exchange cell maps to (runs of 0..5 cells): the
    grouped launch stores their zero sums for every member, as fcx_run does, and matches the
    sequential SCRIP application of each member's own fluxes."""
    import torch
    import oracle_lib
    from fcx.engine import Engine, run_group
    from fcx.parallel import local_atmos
    from fcx.synthetic import build_case
    from test_gpu_multirank import random_run_map

    n = 60_013
    amap = random_run_map(n, (0, 5), seed=41)
    la = local_atmos(amap, 0, 1)
    fields = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))
    cases, engines, outs = [], [], []
    for v in ("CCLM", "MOM5", "RCO"):
        c = build_case(v, n=n, T=1, bias=True, seed=5)
        o = {name: torch.full((la.n_atmos,), float("nan"), dtype=torch.float64, device="cuda:0")
             for name, _ in fields}
        atmos = {"local": la, "fields": [(2, 1, g, name, o[name]) for name, g in fields]}
        engines.append(Engine(c.lf, 1, c.methods, corrections=c.corrections, atmos=atmos))
        cases.append(c)
        outs.append(o)
    for e in engines:
        e.upload(PHASE_ALL)
    run_group(engines, PHASE_ALL, 3600)
    for e in engines:
        e.download(PHASE_ALL)
        e.synchronize()
    for c, o in zip(cases, outs):
        for name, g in fields:
            if (1, g, name) not in c.outputs:
                continue
            want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, np.asarray(c.lf.field[(1, g, name)]),
                                               amap.n_atmos)
            np.testing.assert_array_equal(o[name].cpu().numpy(), want, err_msg=name)
    for e in engines:
        e.close()


@pytest.mark.parametrize("types", [1, 2])
def test_group_launch_captured_in_a_hip_graph(types):
    """fcx_run_group captured into one HIP graph (the engines switched to the capture stream
    with fcx_set_stream) and replayed on new inputs: the group launch and its fix-up launch
    (random map) recompute everything, so a replay gives the bits of a direct call."""
    import torch

    wl = Workload(40_009, 0, 1, ("CCLM", "MOM5", "RCO"), types=types, atmos=True, atmos_map="random")
    wl.run_group(7200)
    torch.cuda.synchronize()
    before = outputs(wl)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            cap = torch.cuda.current_stream().cuda_stream
            for e in wl.engines:
                e.set_stream(cap)
            wl.run_group(7200)
    for e in wl.engines:
        e.set_stream(wl.stream.cuda_stream)
    seen = set()
    for case in wl.cases:  # new air temperatures, uploaded into the same device mirrors
        for key, arr in case.lf.field.items():
            if key[2] == "TATM" and id(arr) not in seen:
                seen.add(id(arr))
                arr *= 1.001
    for e in wl.engines:
        e.upload(PHASE_ALL)
    g.replay()
    torch.cuda.synchronize()
    got = outputs(wl)
    wl.run_group(7200)
    torch.cuda.synchronize()
    want = outputs(wl)
    same_bits(got, want)
    assert any(not np.array_equal(got[k], before[k]) for k in got)  # the replay did the work
    wl.close()
