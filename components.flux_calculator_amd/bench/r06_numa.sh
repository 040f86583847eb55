#!/bin/bash
# round 6: the NUMA node of page-locked host memory against the host-link rates (numa_probe),
# twice (the second run in a fresh process), then the T = 2 occupancy counters
set -euo pipefail
O=${1:-gpurun_out/r06/numa}; mkdir -p $O
timeout -k 10 200 components.flux_calculator_amd/lib/probe/numa_probe 150 > $O/numa_probe_1.json
cat $O/numa_probe_1.json
timeout -k 10 200 components.flux_calculator_amd/lib/probe/numa_probe 150 > $O/numa_probe_2.json
cat $O/numa_probe_2.json
timeout -k 10 900 bash components.flux_calculator_amd/bench/r06_t2counters.sh gpurun_out/r06/t2counters
