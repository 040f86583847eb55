#!/bin/bash
# round 6, VERDICT r05 item 3: the T = 2 (water + ice) group launch at 3 waves per SIMD (the
# build: 168 VGPRs, next-type prefetch) against the 4-wave builds (ab/t2nopf4: no prefetch,
# capped at 128 VGPRs, 40-56 B/lane of spills; ab/t2pf4: prefetch kept, capped, 72-136 B of
# spills) -- kernel trace (VGPRs, scratch, duration) and SQ / TCC counters per build, each in
# its own process (bench/group_ab.py at 10M cells, T = 2, random map).
set -euo pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06/t2counters}; mkdir -p $O
A="--types 2 --rounds 2 --steps 10"
for b in ref t2nopf4 t2pf4; do
  mkdir -p $O/$b
  if [ $b = ref ]; then L=""; else L="$PWD/ab/$b/libfcx.so"; fi
  FCX_LIBRARY=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$b/trace -o run -- \
    python3 components.flux_calculator_amd/bench/group_ab.py $A > $O/$b/group_ab.json
  FCX_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
    SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/$b/sq -o run -- \
    python3 components.flux_calculator_amd/bench/group_ab.py $A > /dev/null
  FCX_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \
    TCC_EA0_RDREQ_128B_sum --kernel-trace --output-format csv -d $O/$b/rdreq -o run -- \
    python3 components.flux_calculator_amd/bench/group_ab.py $A > /dev/null
  FCX_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/$b/write -o run -- \
    python3 components.flux_calculator_amd/bench/group_ab.py $A > /dev/null
done
echo done > $O/DONE
