#!/bin/bash
# crossing-record layouts in ONE process over the SAME arrays (bench/inproc_ab.py --group):
# ref = whole-line records written by one wave + one fix-up launch for the group;
# gfix = two-writer records + one fix-up launch; head = two-writer records + a fix-up per member
set -euo pipefail
O=gpurun_out/r04/inproc1; mkdir -p $O
B=components.flux_calculator_amd/bench
timeout -k 10 400 python3 $B/inproc_ab.py --group --types 2 --rounds 8 --steps 20 --warmup 40 --lib head=ab/head/libfcx.so --lib gfix=ab/gfix/libfcx.so > $O/t2.json
timeout -k 10 400 python3 $B/inproc_ab.py --group --rounds 8 --steps 20 --warmup 40 --opts nohalo:atmos_halo=0 --lib head_nohalo=ab/head/libfcx.so@atmos_halo=0 --lib gfix_nohalo=ab/gfix/libfcx.so@atmos_halo=0 --lib head=ab/head/libfcx.so > $O/t1.json
timeout -k 10 400 python3 $B/inproc_ab.py --group --precision f32 --rounds 8 --steps 20 --warmup 40 --opts nohalo:atmos_halo=0 --lib gfix_nohalo=ab/gfix/libfcx.so@atmos_halo=0 --lib head=ab/head/libfcx.so > $O/f32.json
