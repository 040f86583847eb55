#!/bin/bash
# build_variant.sh OUTDIR [hipcc -D flags...] -- an A/B copy of libfcx.so built with extra
# compile-time flags (measurement tool; the product library is built by the Makefile).
set -e
HERE="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$1"; shift
mkdir -p "$OUT/obj"
FLAGS="-DFCX_AB_BUILD --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -I$HERE/csrc -I$HERE/../include"
/opt/rocm/bin/hipcc $FLAGS "$@" -c "$HERE/csrc/fcx_kernels.hip" -o "$OUT/obj/fcx_kernels.o" &
/opt/rocm/bin/hipcc $FLAGS "$@" -c "$HERE/csrc/fcx_engine.hip" -o "$OUT/obj/fcx_engine.o" &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libfcx.so" "$OUT/obj/fcx_kernels.o" "$OUT/obj/fcx_engine.o"
python3 "$HERE/tools/unversion_needed.py" "$OUT/libfcx.so"
