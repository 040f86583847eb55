#!/bin/bash
# HBM read bytes by request size (gfx950): one rocprofv3 pass of the four TCC read-request
# counters (32-B, 64-B and 128-B requests and their total; 4 TCC slots), so that
#   read bytes = 32 * RDREQ_32B + 64 * RDREQ_64B + 128 * RDREQ_128B
# needs no FETCH_SIZE calibration (FETCH_SIZE tallies 128-B requests at 64 B on gfx950).
#   pmc_bytes.sh OUTDIR -- python3 prog.py args...
set -euo pipefail
export TMPDIR=/tmp
O=$1; shift; [ "$1" = "--" ] && shift
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
  --kernel-trace --output-format csv -d $O/rdreq -o run -- "$@" > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- "$@" > /dev/null
