#!/bin/bash
# bench.py's N > 1 path with EIGHT ranks on GPU 0 -- the shape of the driver's
# `bench.py --gpus 8` -- through libfcx's own exchange (the mock librccl stand-in: RCCL
# refuses several ranks on one device), with every sub-measurement that run takes (main,
# other_map, config4 = BASELINE config 4's strong-scaling object, the all-reduce timings),
# each with its own warm-up.  The mock's per-rank call logs must be identical.
set -euo pipefail
O=${1:-gpurun_out/r06/rehearsal8}; mkdir -p $O
FCX_RCCL_LIBRARY=$PWD/components.flux_calculator_amd/lib/test/libmock_rccl.so FCX_MOCK_RCCL_LOG=$PWD/$O/calls \
  FCX_MOCK_RCCL_TIMEOUT_S=90 \
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29548 bench.py --gpus 8 --backend gloo --same-device --collective rccl --steps 20 --warmup 5 \
  --cells 1000000 --config4 8000000 --no-cpu --e2e 0 > $O/bench_rehearsal_8ranks.json 2> $O/rehearsal.err
python3 - "$O" <<'PY'
import sys, hashlib, glob, json
o = sys.argv[1]
logs = sorted(glob.glob(o + "/calls.*"))
h = {p.rsplit("/", 1)[1]: hashlib.sha1(open(p, "rb").read()).hexdigest()[:12] for p in logs}
lines = {p.rsplit("/", 1)[1]: open(p).read().count("\n") for p in logs}
line = json.loads([x for x in open(o + "/bench_rehearsal_8ranks.json") if x.startswith("{")][-1])
res = {"call_logs": h, "calls_per_rank": lines, "identical": len(set(h.values())) == 1,
       "multi_gpu_check": line.get("multi_gpu_check"), "allreduce": line.get("allreduce"),
       "config4": {k: line.get("config4", {}).get(k) for k in ("baseline_config", "ranks_seen", "allreduce_us_per_step",
                                                               "value", "scaling", "multi_gpu_check")},
       "sub_objects": [k for k in ("other_map", "config4") if k in line]}
json.dump(res, open(o + "/call_logs_check.json", "w"), indent=1)
print(json.dumps(res))
assert res["identical"] and len(logs) == 8 and len(res["sub_objects"]) == 2, res
assert line["multi_gpu_check"]["ranks_seen"] == 8 and line["config4"]["ranks_seen"] == 8, res
PY
