#!/bin/bash
# bench.py's N > 1 path with FOUR ranks on GPU 0 through libfcx's own exchange (the mock
# librccl stand-in: RCCL refuses several ranks on one device), taking the same sub-measurements
# as the driver's `bench.py --gpus 8`: the main workload, other_map and config4, each with its
# own warm-up (the round-4 rehearsal skipped the two that failed).  The mock's
# per-rank call logs must be identical.
set -euo pipefail
O=${1:-gpurun_out/r05/rehearsal4}; mkdir -p $O
FCX_RCCL_LIBRARY=$PWD/components.flux_calculator_amd/lib/test/libmock_rccl.so FCX_MOCK_RCCL_LOG=$PWD/$O/calls \
  FCX_MOCK_RCCL_TIMEOUT_S=60 \
  timeout -k 10 500 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29544 bench.py --gpus 4 --backend gloo --same-device --collective rccl --steps 20 --warmup 5 \
  --cells 2000000 --config4 8000000 --no-cpu --e2e 0 > $O/bench_rehearsal_4ranks.json 2> $O/rehearsal.err
python3 - "$O" <<'PY'
import sys, hashlib, glob, json
o = sys.argv[1]
logs = sorted(glob.glob(o + "/calls.*"))
h = {p: hashlib.sha1(open(p, "rb").read()).hexdigest()[:12] for p in logs}
lines = {p: open(p).read().count("\n") for p in logs}
line = json.loads([x for x in open(o + "/bench_rehearsal_4ranks.json") if x.startswith("{")][-1])
res = {"call_logs": h, "calls_per_rank": lines, "identical": len(set(h.values())) == 1,
       "multi_gpu_check": line.get("multi_gpu_check"), "sub_objects": [k for k in ("other_map", "config4") if k in line]}
json.dump(res, open(o + "/call_logs_check.json", "w"), indent=1)
print(json.dumps(res))
assert res["identical"] and len(logs) == 4 and len(res["sub_objects"]) == 2, res
PY
