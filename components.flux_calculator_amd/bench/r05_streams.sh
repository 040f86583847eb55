#!/bin/bash
# engines on torch's pooled streams against streams of their own (as a Fortran host gets),
# at the Baltic size; and bench.py's link probe with streams of its own
set -euo pipefail
O=gpurun_out/r05/streams; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 300 python3 -u $B/baltic_probe.py --steps 300 --handover 0 --mode default: --mode own:own_stream=1 --mode dma:zero_copy=0 --mode dma_own:zero_copy=0,own_stream=1 > $O/baltic_probe.log 2>&1
timeout -k 10 120 python3 -u -c "
import sys, json; sys.path.insert(0, '$B'); import torch; torch.cuda.init()
from link_probe import link_rates
print(json.dumps(link_rates(6815744, 5242880)))" > $O/link_rates.json 2>&1
