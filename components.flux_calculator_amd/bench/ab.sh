#!/bin/bash
# In-process A/B of libfcx builds (bench/inproc_ab.py, random map, host-bound mirrors like
# the bench): ab.sh OUTDIR LABEL "INPROC ARGS" [LABEL "ARGS" ...]; one JSON per label.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
while [ $# -gt 1 ]; do
  timeout -k 10 400 python3 components.flux_calculator_amd/bench/inproc_ab.py --host --rounds 6 --steps 30 --warmup 60 $2 > $O/$1.json
  shift 2
done
