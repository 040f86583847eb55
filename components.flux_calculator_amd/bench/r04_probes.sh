#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out/r04
timeout -k 10 200 components.flux_calculator_amd/bench/f32_probe > gpurun_out/r04/f32_probe.txt 2>&1
