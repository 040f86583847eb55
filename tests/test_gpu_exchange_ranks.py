"""libfcx's own N > 1 boundary exchange (fcx_atmos_allreduce / fcx_set_comm -> atmos_exchange,
fcx_engine.hip) executed with 2 and 3 ranks on the one GPU of the box.

RCCL refuses two ranks on one device, so the ranks load a test-only stand-in for librccl.so
through FCX_RCCL_LIBRARY (tests/cpp/mock_rccl.cpp): every ncclAllReduce is a host-memory
all-reduce over a shared-memory segment that also checks that every rank issued the same
call (count, type, operation) and fails -- instead of hanging -- on a mismatch or a missing
rank.  Everything above it is the product path: the communicator, the signature agreement,
the in-place and packed all-reduce, the stream joins, fcx_atmos_finish.

This closes the accumulation OASIS performs on oasis_put of the 'S A xxxx 00' fields
(flux_calculator.F90:1015, create_namcouple.F90:92-98).  Checked against the sequential SCRIP
sum of the GPU's own fluxes over the global map: interior atmosphere cells bit-identical,
cells shared between ranks within 1e-12 (they are sums of partial sums); every rank's
collective call sequence identical (the mock's logs)."""
import os
import socket
import subprocess
import sys
import json

import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOCK = os.path.join(ROOT, "components.flux_calculator_amd", "lib", "test", "libmock_rccl.so")
FIELDS = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))
VARIANTS = ("CCLM", "MOM5", "RCO")
N = 24_012  # every APPLE cut of 2 and 3 ranks falls inside an atmosphere cell

# (name, slot layout, streams, special); run by every rank in this order
SCENARIOS = [
    ("adjacent_one_stream", "adjacent", "one", None),
    ("adjacent_engine_streams", "adjacent", "per_engine", None),
    ("reversed_one_stream", "reversed", "one", None),
    ("gapped_engine_streams", "gapped", "per_engine", None),
    ("separate_one_stream", "separate", "one", None),
    ("attached_comm", "own", "one", "attached"),
    ("signature_mismatch", "adjacent", "one", "mismatch"),
    ("stale_engine", "adjacent", "one", "stale"),
    # fcx_set_comm + fcx_run_group where the ranks merge different engines (rank 0's last
    # engine has a grid cap, so it runs as fcx_run): the per-engine exchanges must still go
    # in list order on every rank (solo engines used to exchange first)
    ("attached_group_differs", "own", "one", "attached_group"),
    # the signature agreement before every exchange (fcx_comm_verify): after an agreed
    # exchange, rank 1 passes a shorter engine list -- every rank gets the named error
    ("relisted_after_agreement", "adjacent", "one", "relist"),
]
SCENARIOS_3 = [
    ("empty_middle_rank", "adjacent", "one", "empty_middle"),
    ("rank_inside_one_cell", "adjacent", "one", "tiny_middle"),
    ("rank_inside_one_cell_separate", "separate", "per_engine", "tiny_middle"),
]


def _uid():
    name = f"/fcxmock-test-{os.getpid()}-{np.random.default_rng().integers(1 << 62):x}".encode()
    return name + b"\0" * (128 - len(name))


def _ranges(world, special, amap):
    from fcx.parallel import apple_range

    n = amap.atmos_index.shape[0]
    if special == "empty_middle":
        k = next(i for i in range(n // 2, n) if amap.atmos_index[i - 1] == amap.atmos_index[i])
        return [(0, k), (0, 0), (k, n - k)]
    if special == "tiny_middle":
        idx = amap.atmos_index
        starts = np.flatnonzero(np.diff(np.concatenate([[-1], idx])))  # first cell of each run
        lens = np.diff(np.concatenate([starts, [n]]))
        c0 = int(starts[np.flatnonzero(lens >= 4)[len(starts) // 3 // 2]])
        return [(0, c0 + 1), (c0 + 1, 2), (c0 + 3, n - c0 - 3)]
    return [apple_range(n, r, world) for r in range(world)]


def _scenario(rank, world, uid, name, layout, streams, special, log):
    import dataclasses

    import torch
    from fcx.basic import PHASE_ALL, PHASE_NORMAL
    from fcx.comm import Comm
    from fcx.engine import Engine, run_group
    from fcx.parallel import local_atmos, synthetic_atmos_map
    from test_gpu_multirank import shard_case
    from fcx.synthetic import build_case

    os.environ["FCX_MOCK_RCCL_LOG"] = log
    amap = synthetic_atmos_map(N)
    ranges = _ranges(world, special, amap)
    la = local_atmos(amap, rank, world, ranges=ranges)
    off, size = ranges[rank]
    stride, nb = len(FIELDS), world - 1
    region = nb * stride
    dev = "cuda:0"
    if layout in ("adjacent", "reversed"):
        big = torch.zeros(3 * region, dtype=torch.float64, device=dev)
        slots = [big[(i if layout == "adjacent" else 2 - i) * region:] for i in range(3)]
        bufs = [big]
    elif layout == "gapped":
        big = torch.zeros(3 * region + 2 * 5, dtype=torch.float64, device=dev)
        slots = [big[i * (region + 5):] for i in range(3)]
        bufs = [big]
    elif layout == "separate":
        bufs = slots = [torch.zeros(region, dtype=torch.float64, device=dev) for _ in range(3)]
    else:
        bufs, slots = [], [None] * 3
    own = [torch.cuda.Stream() for _ in range(3)] if streams == "per_engine" else [torch.cuda.current_stream()] * 3
    comm = Comm(0, world, rank, uid)
    if special == "relist":
        comm.verify(True)
    engines, cases, outs_all = [], [], []
    for i, v in enumerate(VARIANTS):
        full = build_case(v, n=N, T=1, bias=True, seed=41 + i)
        case = shard_case(full, off, off + size, v, seed=41 + i)
        outs = {f: torch.full((max(la.n_atmos, 1),), float("nan"), dtype=torch.float64, device=dev) for f, _ in FIELDS}
        atmos = {"local": la, "fields": [(PHASE_NORMAL, 1, g, f, outs[f]) for f, g in FIELDS]}
        if layout == "own":
            atmos.update(own_boundaries=True, comm=comm)
        else:
            atmos["shared"] = (slots[i], stride)
        if special == "attached_group":
            opts = {"max_blocks": 32} if (rank == 0 and i == 2) else None
        else:
            opts = {"atmos_in_run": 0} if i == 1 else None
        e = Engine(case.lf, 1, case.methods, corrections=case.corrections, atmos=atmos,
                   stream=own[i].cuda_stream, options=opts)
        e.upload(PHASE_ALL)
        engines.append(e)
        cases.append(case)
        outs_all.append(outs)
    torch.cuda.synchronize()
    result = {"name": name, "atmos_offset": la.atmos_offset, "n_atmos": la.n_atmos, "left": la.left,
              "right": la.right, "offset": off, "size": size, "steps": []}
    for step in range(2):
        for outs in outs_all:
            for o in outs.values():
                o.fill_(float("nan"))
        torch.cuda.synchronize()
        err, group = None, None
        if special == "attached_group":
            run_group(engines, PHASE_ALL, 3600 * step)  # every engine's exchange inside
            group = [e.last_group_size() for e in engines]
        for i, e in enumerate(engines):
            if special == "attached_group":
                break
            if special == "stale" and rank == world - 1 and step == 0 and i == 2:
                continue  # this rank never runs engine 2 before the first exchange
            e.run(PHASE_ALL, 3600 * step)
            if i == 1:
                e.run_atmos(PHASE_ALL)  # atmos_in_run 0: the accumulation on its own
        try:
            if layout != "own":
                short = (special == "mismatch" and rank == 1) or (special == "relist" and rank == 1 and step == 1)
                use = engines[:2] if short else engines
                comm.atmos_allreduce(use)
        except Exception as ex:  # noqa: BLE001 -- reported to the parent
            err = str(ex)
        for e in engines:
            e.download(PHASE_ALL)
            e.synchronize()
        torch.cuda.synchronize()
        rec = {"error": err, "group": group, "slots_zero": all(float(b.abs().sum()) == 0.0 for b in bufs),
               "out": [{f: outs[f].cpu().numpy()[: la.n_atmos].copy() for f, _ in FIELDS} for outs in outs_all],
               "flux": [{f: np.array(c.lf.field[(1, g, f)], copy=True) for f, g in FIELDS} for c in cases]}
        result["steps"].append(rec)
        if special in ("mismatch", "stale"):
            break
    for e in engines:
        e.close()
    comm.close()
    return result


def _child(rank, world, uids, scenarios, logdir, q):
    os.environ["FCX_RCCL_LIBRARY"] = MOCK
    os.environ["FCX_MOCK_RCCL_TIMEOUT_S"] = "30"
    try:
        import torch

        torch.cuda.set_device(0)
        out = []
        for (name, layout, streams, special), uid in zip(scenarios, uids):
            out.append(_scenario(rank, world, uid, name, layout, streams, special, os.path.join(logdir, name)))
        q.put((rank, None, out))
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((rank, traceback.format_exc() + repr(ex), None))


def _mixed_err(got, want):
    return float(np.max(np.abs(got - want) / np.maximum(np.abs(want), 1e-300))) if got.size else 0.0


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_ranks_through_libfcx(world, tmp_path):
    import torch.multiprocessing as mp

    assert os.path.exists(MOCK), "build() makes the mock RCCL (make -C components.flux_calculator_amd mock-rccl)"
    scenarios = SCENARIOS + (SCENARIOS_3 if world == 3 else [])
    uids = [_uid() for _ in scenarios]
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_child, args=(r, world, uids, scenarios, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, err, out = q.get()
        assert err is None, f"rank {rank}: {err}"
        res[rank] = out
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from fcx.parallel import synthetic_atmos_map

    amap = synthetic_atmos_map(N)
    problems = []
    for k, (name, layout, streams, special) in enumerate(scenarios):
        per = [res[r][k] for r in range(world)]
        logs = [open(os.path.join(tmp_path, name) + f".{r}").read() for r in range(world)]
        if special != "mismatch" and len(set(logs)) != 1:
            problems.append(f"{name}: call sequences differ: {logs}")
        if special == "mismatch":
            errs = [p["steps"][0]["error"] for p in per]
            if not all(e and "ranks disagree" in e for e in errs):
                problems.append(f"{name}: expected every rank to report the disagreement, got {errs}")
            continue
        if special == "stale":
            errs = [p["steps"][0]["error"] for p in per]
            want_err = [None] * (world - 1) + ["no accumulation"]
            if not (all(e is None for e in errs[:-1]) and errs[-1] and "no accumulation" in errs[-1]):
                problems.append(f"{name}: expected {want_err}, got {errs}")
            continue
        if special == "relist":
            errs = [p["steps"][1]["error"] for p in per]
            if not all(e and "ranks disagree" in e for e in errs):
                problems.append(f"{name}: step 1 expected every rank to report the disagreement, got {errs}")
        if special == "attached_group":
            for r, p in enumerate(per):
                want_g = [2, 2, 0] if r == 0 else [3, 3, 3]
                want_g = [want_g, want_g]
                if [st["group"] for st in p["steps"]] != want_g:
                    problems.append(f"{name} rank {r}: group sizes {[st['group'] for st in p['steps']]}, want {want_g}")
        for step in range(1 if special == "relist" else 2):
            for p in per:
                if p["steps"][step]["error"]:
                    problems.append(f"{name} rank step {step}: {p['steps'][step]['error']}")
                if not p["steps"][step]["slots_zero"]:
                    problems.append(f"{name} step {step}: slots not re-zeroed")
            for i, v in enumerate(VARIANTS):
                for f, _ in FIELDS:
                    flux = np.concatenate([p["steps"][step]["flux"][i][f] for p in per])
                    want = oracle_lib.atmos_accumulate(amap.atmos_index, amap.weight, flux, amap.n_atmos)
                    for r, p in enumerate(per):
                        got = p["steps"][step]["out"][i][f]
                        if p["n_atmos"] == 0:
                            continue
                        a0 = p["atmos_offset"]
                        w = want[a0: a0 + p["n_atmos"]]
                        inner = np.ones(p["n_atmos"], bool)
                        if p["left"] >= 0:
                            inner[0] = False
                        if p["right"] >= 0:
                            inner[-1] = False
                        if not np.array_equal(got[inner], w[inner]):
                            problems.append(f"{name} {v} {f} rank {r} step {step}: interior differs")
                        if _mixed_err(got[~inner], w[~inner]) > 1e-12:
                            problems.append(f"{name} {v} {f} rank {r} step {step}: boundary error "
                                            f"{_mixed_err(got[~inner], w[~inner]):.3g}")
        shared = sum(int(p["left"] >= 0) + int(p["right"] >= 0) for p in per)
        if shared == 0:
            problems.append(f"{name}: no shared boundary cell exercised")
        if special == "tiny_middle" and not (per[1]["n_atmos"] == 1 and per[1]["left"] == per[1]["right"] >= 0):
            problems.append(f"{name}: middle rank should hold one cell with one slot, got {per[1]}")
    assert not problems, "\n".join(problems[:40])


def test_bench_two_ranks_through_libfcx_exchange(tmp_path):
    """bench.py's own N > 1 path, the one the driver's 8-GPU run times, with libfcx's
    communicator (not torch's all-reduce): two ranks on GPU 0 over gloo for the rendezvous
    and the mock RCCL for the collective.  Its multi_gpu_check must pass and both ranks must
    issue the same collective sequence."""
    assert os.path.exists(MOCK)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, FCX_RCCL_LIBRARY=MOCK, FCX_MOCK_RCCL_LOG=str(tmp_path / "bench"),
               FCX_MOCK_RCCL_TIMEOUT_S="60")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--same-device", "--backend", "gloo", "--collective", "rccl", "--steps", "6",
           "--warmup", "2", "--cells", "1000000", "--config4", "2000000", "--no-cpu", "--e2e", "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    mg = line["multi_gpu_check"]
    assert "libfcx RCCL communicator" in line["config"]["atmos_accumulation"]
    assert mg["ranks_seen"] == 2 and mg["shared_cells"] > 0, mg
    assert mg["max_mixed_err"] <= 1e-12 and mg["interior_bit_identical"], mg
    logs = [open(str(tmp_path / "bench") + f".{r}").read() for r in range(2)]
    assert logs[0] == logs[1] and logs[0].count("\n") >= 6, logs
