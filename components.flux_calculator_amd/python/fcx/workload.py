"""The benchmark workload of BASELINE.json configs 3/4 as one object, shared by bench.py and
the tests that check exactly that path (tests/test_gpu_config34.py).

One rank's part of a synthetic exchange grid (SURVEY.md 8d distributions): its APPLE cell
range (decomp_def.F90:23-31), the CCLM / MOM5 / RCO cases over one set of input arrays,
one engine per variant with the exchange -> atmosphere accumulation of the six fluxes sent
to the atmosphere ('S A xxxx 00', create_namcouple.F90:92-98) fused into the flux kernel,
inputs resident in HBM (engine-owned tile-blocked mirrors uploaded once, or the caller's
device arrays).  A step is fcx_run of every engine; the boundary slots of the atmosphere
cells shared with the neighbour ranks are laid out contiguously for all variants, so ONE
all-reduce per step completes them.
"""
import numpy as np

from .basic import PHASE_ALL, PHASE_NORMAL
from .engine import Engine, run_group
from .parallel import BlockedRandomAtmosMap, PeriodicAtmosMap, apple_range
from .synthetic import BASE_SEED, as_dtype, build_case, inputs_for_bench

VARIANTS = ("CCLM", "MOM5", "RCO")
# fluxes OASIS sends to the atmosphere, with their grids
ATM_FIELDS = (("MEVA", 1), ("HLAT", 1), ("HSEN", 1), ("RBBR", 1), ("UMOM", 2), ("VMOM", 3))


class Workload:
    """n_global cells split over `world` ranks by APPLE ranges (this is rank `rank`'s part).

    caller_device: bind contiguous torch device arrays shared by the variants instead of
    host arrays whose engine-owned device mirrors are uploaded once.
    engine_options: extra fcx_set_option values for every engine (A/B tools).
    inputs: this rank's input arrays (inputs_for_bench's keys) instead of drawing them."""

    def __init__(self, n_global, rank=0, world=1, variants=VARIANTS, types=1, bias=False,
                 precision="f64", atmos=True, caller_device=False, device=0, stream=None,
                 engine_options=None, atmos_map="periodic", inputs=None):
        import torch

        self.n_global, self.rank, self.world = int(n_global), int(rank), int(world)
        self.offset, self.n = apple_range(self.n_global, self.rank, self.world)
        self.variants = tuple(variants)
        self.types, self.bias, self.precision = int(types), bool(bias), precision
        f32 = precision == "f32"
        dev = torch.device("cuda", device)
        self.dev = dev
        self.stream = stream if stream is not None else torch.cuda.current_stream(dev)
        host = inputs if inputs is not None else inputs_for_bench(self.n, seed=BASE_SEED + self.offset)
        if caller_device:
            data = {k: torch.as_tensor(v).to(dev) for k, v in host.items()}
            if f32:  # inputs rounded once; every variant's case shares them
                data = {k: v.float() for k, v in data.items()}
            case_dev = dev
            del host
        else:
            data, case_dev = host, None
        self.caller_device = caller_device
        # periodic: runs of 3, 4, 5, 4 cells that never cross a 16-cell period (nor a wave
        # tile); random: runs of 3..5 cells in random order (BlockedRandomAtmosMap), so that
        # segments cross wave tiles as on a real intersection grid
        if not atmos:
            self.la = None
        else:
            ranges = [apple_range(self.n_global, r, self.world) for r in range(self.world)]
            amap = BlockedRandomAtmosMap() if atmos_map == "random" else PeriodicAtmosMap()
            self.la = amap.local(self.offset, self.n, self.rank, self.world, self.n_global, ranges=ranges)
        self.atmos_map = atmos_map
        nb, stride = max(self.world - 1, 0), len(ATM_FIELDS)
        self.n_boundaries, self.stride = nb, stride
        # [variant][boundary][field]: the shared slots of every variant in one buffer
        self.shared = torch.zeros(max(len(self.variants) * nb * stride, 1), dtype=torch.float64, device=dev)
        self.cases, self.engines, self.atm_outs = [], [], []
        # inputs uploaded once, before any timed region: no staging arena (it would pin a host
        # image of every mirror pool for one copy)
        opts = {"atmos_in_run": 0, "timing": 0, "host_staging": 0}
        opts.update(engine_options or {})
        for i, v in enumerate(self.variants):
            c = build_case(v, n=self.n, T=self.types, bias=self.bias, device=case_dev,
                           data=data if self.types == 1 else None)
            if f32:
                c = as_dtype(c, "float32")
            atm = None
            if self.la is not None:
                outs = {name: (torch.empty(max(self.la.n_atmos, 1), dtype=torch.float32 if f32 else torch.float64,
                                           device=dev) if case_dev is not None
                               else np.empty(max(self.la.n_atmos, 1), dtype=np.float32 if f32 else np.float64))
                        for name, _ in ATM_FIELDS}
                self.atm_outs.append(outs)
                # the type-0 fields: with several surface types the averages over the types,
                # with one type the type-1 fluxes themselves
                s0 = 0 if self.types >= 2 else 1
                atm = {"local": self.la, "fields": [(PHASE_NORMAL, s0, g, name, outs[name]) for name, g in ATM_FIELDS],
                       "shared": (self.shared[i * nb * stride:], stride) if nb else None}
            # per-kernel times come from the caller's own events on the same stream; the
            # engine's internal ones would add a second event pair per launch (+2.5 % per
            # step, bench/event_probe.py)
            e = Engine(c.lf, c.num_surface_types, c.methods, corrections=c.corrections,
                       averages=c.averages, device=device, stream=self.stream.cuda_stream, atmos=atm,
                       options=opts)
            if case_dev is None:
                e.upload(PHASE_ALL)  # inputs resident in HBM before any timed region
            self.cases.append(c)
            self.engines.append(e)
        self.alg_bytes = [e.algorithmic_bytes(PHASE_ALL) for e in self.engines]

    def run(self, t, events=None):
        """One coupling step of every variant (no collective); events[i] = (start, end)
        recorded around engine i's launch (None: no events around that engine)."""
        for i, e in enumerate(self.engines):
            ev = events[i] if events is not None else None
            if ev is not None:
                ev[0].record(self.stream)
            e.run(PHASE_ALL, t)
            if ev is not None:
                ev[1].record(self.stream)
            if self.la is not None:
                e.run_atmos(PHASE_ALL)

    def run_group(self, t, event=None):
        """One coupling step of every variant with their flux passes merged into ONE launch
        (fcx_run_group); event = (start, end) recorded around it, or None."""
        if event is not None:
            event[0].record(self.stream)
        run_group(self.engines, PHASE_ALL, t)
        if event is not None:
            event[1].record(self.stream)
        if self.la is not None:
            for e in self.engines:
                e.run_atmos(PHASE_ALL)  # (a no-op where the accumulation rode in the launch)

    def finish(self):
        """After the all-reduce of `shared`: the completed boundary sums into the outputs."""
        for e in self.engines:
            e.atmos_finish()

    def download(self):
        """Host-bound workloads: every engine's outputs (fluxes and atmosphere fields) back
        into the cases' host arrays."""
        for e in self.engines:
            e.download(PHASE_ALL)
            e.synchronize()

    def close(self):
        for e in self.engines:
            e.close()
        self.engines = []
