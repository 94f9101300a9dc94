#!/bin/bash
# Diagnostic library variant: one translation unit recompiled with extra defines, linked with the
# default objects of every other unit (build/obj). usage: build_diag_variant.sh <out.so> <tu.hip> -DX=1 ...
set -e
cd "$(dirname "$0")/.."
OUT=$1; TU=$2; shift 2
OBJ=build/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -fno-slp-vectorize "$@" \
  -c quad-periodic-mpc_amd/csrc/$TU -o /tmp/diag_$(basename $OUT).o
objs=$(ls $OBJ/*.o | grep -v "/$TU.o$" | grep -v "_CMPC")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $objs /tmp/diag_$(basename $OUT).o
echo "$OUT"
