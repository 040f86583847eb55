#!/bin/bash
# round 6: the host-link schedules of span DMAs (span_probe, default and mapped host memory),
# then the whole GPU suite (full-grid oracle parity of configs 3/4 included; reports under
# gpurun_out/parity/)
set -euo pipefail
O=${1:-gpurun_out/r06/first}; mkdir -p $O
timeout -k 10 120 components.flux_calculator_amd/lib/probe/span_probe 32768 300 mapped > $O/span_probe_mapped.json
timeout -k 10 120 components.flux_calculator_amd/lib/probe/span_probe 32768 300 default > $O/span_probe_default.json
cat $O/span_probe_mapped.json $O/span_probe_default.json
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests \
  > $O/tests.log 2>&1
tail -5 $O/tests.log
