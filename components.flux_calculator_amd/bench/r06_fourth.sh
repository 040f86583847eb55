#!/bin/bash
# round 6: the host link by hipHostMalloc flags as kernels (zero-copy) and copy engines use it,
# then the Baltic-size library-memory step with portable slabs (the build) and with the
# pre-round-6 mapped slabs (ab/pinmap)
set -euo pipefail
O=${1:-gpurun_out/r06/fourth}; mkdir -p $O
timeout -k 10 200 components.flux_calculator_amd/lib/probe/zc_flags_probe 200 > $O/zc_flags.json
cat $O/zc_flags.json
timeout -k 10 300 python3 -u components.flux_calculator_amd/bench/libmem_probe.py > $O/libmem_portable.json 2> $O/libmem_portable.err
cat $O/libmem_portable.json
FCX_LIBRARY=$PWD/ab/pinmap/libfcx.so timeout -k 10 300 python3 -u components.flux_calculator_amd/bench/libmem_probe.py \
  > $O/libmem_mapped.json 2> $O/libmem_mapped.err
cat $O/libmem_mapped.json
