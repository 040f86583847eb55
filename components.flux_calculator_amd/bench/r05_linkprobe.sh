#!/bin/bash
# bench.py's host-link probe with plain hipMalloc device buffers (libfcx's pools) in a torch
# process: do the two directions overlap as in the plain-HIP dma_probe?
set -euo pipefail
O=gpurun_out/r05/linkprobe; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 120 python3 -u -c "
import sys, json; sys.path.insert(0, '$B'); import torch; torch.cuda.init()
from link_probe import link_rates
print(json.dumps(link_rates(6815744, 5242880)))" > $O/link_rates.json 2> $O/link_rates.err
