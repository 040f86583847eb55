"""libfcx's own collective (fcx_comm_*, include/fcx.h) on the GPU box: a real RCCL
communicator through the C ABI, world size 1 (one GPU per box; RCCL refuses two ranks on one
device -- libfcx's exchange with 2 and 3 ranks runs through a librccl stand-in in
test_gpu_exchange_ranks.py, and the 8-GPU run is bench.py's).

With one rank the all-reduce is the identity, so an engine given a boundary slot for its
last atmosphere cell must come out bit-identical to the sequential SCRIP sum after the
exchange, with the slots re-zeroed."""
import dataclasses

import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu

from fcx.basic import PHASE_ALL, PHASE_NORMAL  # noqa: E402
from fcx.parallel import local_atmos, synthetic_atmos_map  # noqa: E402
from fcx.synthetic import build_case  # noqa: E402

FIELDS = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))


def test_comm_allreduce_world1():
    import torch
    from fcx.comm import Comm, unique_id

    c = Comm(0, 1, 0, unique_id())
    x = torch.arange(1000, dtype=torch.float64, device="cuda:0") * 0.5
    want = x.clone()
    s = torch.cuda.current_stream()
    c.allreduce_sum(x, s.cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(x, want)
    c.close()


@pytest.mark.parametrize("variant", ["CCLM", "MOM5", "RCO"])
@pytest.mark.parametrize("fused", [True, False])
def test_engine_with_attached_comm(variant, fused):
    """fcx_set_atmos_boundaries + fcx_set_comm: the engine owns its slots and runs the
    all-reduce and the finish itself inside fcx_step."""
    import torch
    from fcx.comm import Comm, unique_id
    from fcx.engine import Engine

    n = 50_001
    case = build_case(variant, n=n, T=1, bias=True, seed=5)
    amap = synthetic_atmos_map(n)
    la = dataclasses.replace(local_atmos(amap, 0, 1), right=0, n_boundaries=1)
    c = Comm(0, 1, 0, unique_id())
    outs = {name: torch.full((la.n_atmos,), float("nan"), dtype=torch.float64, device="cuda:0")
            for name, _ in FIELDS}
    atmos = {"local": la, "fields": [(PHASE_NORMAL, 1, g, name, outs[name]) for name, g in FIELDS],
             "own_boundaries": True, "comm": c}
    eng = Engine(case.lf, 1, case.methods, corrections=case.corrections, atmos=atmos,
                 options=None if fused else {"specialize": 0})
    for step in range(2):
        for o in outs.values():
            o.fill_(float("nan"))
        eng.step(PHASE_ALL, 3600 * step)
        torch.cuda.synchronize()
        for name, g in FIELDS:
            flux = np.asarray(case.lf.field[(1, g, name)])
            want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, flux, amap.n_atmos)
            np.testing.assert_array_equal(outs[name].cpu().numpy(), want, err_msg=f"{name} step {step}")
    eng.close()
    c.close()


def test_one_allreduce_for_three_variants():
    """The bench's layout: the three variants' slots adjacent in one buffer, completed by
    fcx_atmos_allreduce in ONE all-reduce, then each engine's finish."""
    import torch
    from fcx.comm import Comm, unique_id
    from fcx.engine import Engine

    n = 40_003
    amap = synthetic_atmos_map(n)
    la = dataclasses.replace(local_atmos(amap, 0, 1), right=0, n_boundaries=1)
    stride = len(FIELDS)
    shared = torch.zeros(3 * stride, dtype=torch.float64, device="cuda:0")
    c = Comm(0, 1, 0, unique_id())
    engines, cases, outs_all = [], [], []
    for i, v in enumerate(("CCLM", "MOM5", "RCO")):
        case = build_case(v, n=n, T=1, seed=9)
        outs = {name: torch.full((la.n_atmos,), float("nan"), dtype=torch.float64, device="cuda:0")
                for name, _ in FIELDS}
        atmos = {"local": la, "fields": [(PHASE_NORMAL, 1, g, name, outs[name]) for name, g in FIELDS],
                 "shared": (shared[i * stride:], stride)}
        e = Engine(case.lf, 1, case.methods, atmos=atmos, options={"atmos_in_run": 0})
        e.upload(PHASE_ALL)
        engines.append(e)
        cases.append(case)
        outs_all.append(outs)
    for e in engines:
        e.run(PHASE_ALL, 0)
        e.run_atmos(PHASE_ALL)
    c.atmos_allreduce(engines)
    torch.cuda.synchronize()
    assert float(shared.abs().sum()) == 0.0  # re-zeroed by the finish
    for e, case, outs in zip(engines, cases, outs_all):
        e.download(PHASE_ALL)
        e.synchronize()
        for name, g in FIELDS:
            flux = np.asarray(case.lf.field[(1, g, name)])
            want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, flux, amap.n_atmos)
            np.testing.assert_array_equal(outs[name].cpu().numpy(), want, err_msg=name)
        e.close()
    c.close()


@pytest.mark.parametrize("layout", ["separate_buffers", "gapped_buffer", "reversed_adjacent"])
@pytest.mark.parametrize("streams", ["one", "per_engine"])
def test_atmos_allreduce_regions_and_streams(layout, streams):
    """fcx_atmos_allreduce over three engines whose boundary-slot regions do not follow each
    other in list order in one buffer (separate buffers, one buffer with gaps, or adjacent in
    reverse engine order): the slots are packed through the communicator's scratch for the
    one all-reduce and copied back; with the engines on one stream or each on its own stream
    (the all-reduce on the first engine's stream waits for the others' accumulations, and each
    engine's finish waits for it).  One rank: every atmosphere cell bit-identical to the
    sequential sum, every slot re-zeroed.  (2 and 3 ranks: tests/test_gpu_exchange_ranks.py.)"""
    import torch
    from fcx.comm import Comm, unique_id
    from fcx.engine import Engine

    n = 40_003
    amap = synthetic_atmos_map(n)
    # both boundary slots in use: the first and the last atmosphere cell go through the exchange
    la = dataclasses.replace(local_atmos(amap, 0, 1), left=0, right=1, n_boundaries=2)
    stride, nb = len(FIELDS), 2
    region = nb * stride
    if layout == "separate_buffers":
        bufs = [torch.zeros(region, dtype=torch.float64, device="cuda:0") for _ in range(3)]
        slots = bufs
    elif layout == "gapped_buffer":
        big = torch.zeros(3 * region + 2 * 7, dtype=torch.float64, device="cuda:0")
        bufs = [big]
        slots = [big[i * (region + 7):] for i in range(3)]
    else:
        big = torch.zeros(3 * region, dtype=torch.float64, device="cuda:0")
        bufs = [big]
        slots = [big[(2 - i) * region:] for i in range(3)]
    own = [torch.cuda.Stream() for _ in range(3)] if streams == "per_engine" else [torch.cuda.current_stream()] * 3
    c = Comm(0, 1, 0, unique_id())
    engines, cases, outs_all = [], [], []
    for i, v in enumerate(("CCLM", "MOM5", "RCO")):
        case = build_case(v, n=n, T=1, seed=31 + i)
        outs = {name: torch.full((la.n_atmos,), float("nan"), dtype=torch.float64, device="cuda:0")
                for name, _ in FIELDS}
        atmos = {"local": la, "fields": [(PHASE_NORMAL, 1, g, name, outs[name]) for name, g in FIELDS],
                 "shared": (slots[i], stride)}
        e = Engine(case.lf, 1, case.methods, atmos=atmos, stream=own[i].cuda_stream,
                   options={"atmos_in_run": 0})
        e.upload(PHASE_ALL)
        engines.append(e)
        cases.append(case)
        outs_all.append(outs)
    torch.cuda.synchronize()
    for step in range(2):
        for outs in outs_all:
            for o in outs.values():
                o.fill_(float("nan"))
        torch.cuda.synchronize()
        for e in engines:
            e.run(PHASE_ALL, 3600 * step)
            e.run_atmos(PHASE_ALL)
        c.atmos_allreduce(engines)
        for e in engines:
            e.download(PHASE_ALL)
            e.synchronize()
        torch.cuda.synchronize()
        for b in bufs:
            assert float(b.abs().sum()) == 0.0  # every slot re-zeroed by the finishes
        for case, outs in zip(cases, outs_all):
            for name, g in FIELDS:
                flux = np.asarray(case.lf.field[(1, g, name)])
                want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, flux, amap.n_atmos)
                np.testing.assert_array_equal(outs[name].cpu().numpy(), want, err_msg=f"{name} step {step}")
    for e in engines:
        e.close()
    c.close()
