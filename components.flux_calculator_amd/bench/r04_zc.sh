#!/bin/bash
set -euo pipefail
O=gpurun_out/r04/zc; mkdir -p $O
for v in CCLM RCO; do
  timeout -k 10 300 python3 components.flux_calculator_amd/bench/zc_cap_probe.py --variant $v > $O/caps_$v.json
done
