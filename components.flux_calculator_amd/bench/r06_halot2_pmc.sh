#!/bin/bash
# round 6: HBM bytes of the T = 2 group launch, halo-tile build (ab_t2/halo) against the
# product build -- request-size read counters and WRITE_SIZE, one --pmc pass each per build.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/halot2_pmc; mkdir -p $O
A="--types 2 --rounds 1 --steps 10"
for b in ref halo; do
  mkdir -p $O/$b
  if [ $b = ref ]; then L=""; else L="$PWD/ab_t2/halo/libfcx.so"; fi
  FCX_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \
    TCC_EA0_RDREQ_128B_sum --kernel-trace --output-format csv -d $O/$b/rdreq -o run -- \
    python3 components.flux_calculator_amd/bench/group_ab.py $A > /dev/null
  FCX_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/$b/write -o run -- \
    python3 components.flux_calculator_amd/bench/group_ab.py $A > /dev/null
done
echo done > $O/DONE
