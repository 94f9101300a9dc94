#!/bin/bash
# Diagnostic library variant: one translation unit recompiled with extra defines, linked with the
# default objects of every other unit (build/obj). Same flags as quad-periodic-mpc_amd/build.py.
# usage: build_diag_variant.sh <out.so> <tu.hip> -DX=1 ...
set -e
cd "$(dirname "$0")/.."
OUT=$1; TU=$2; shift 2
OBJ=build/obj
FLAGS=$(python3 -c "import importlib,sys; sys.path.insert(0,'.'); print(' '.join(importlib.import_module('quad-periodic-mpc_amd.build').FLAGS))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS "$@" \
  -c quad-periodic-mpc_amd/csrc/$TU -o /tmp/diag_$(basename $OUT).o
objs=$(ls $OBJ/*.o | grep -v "/$TU.o$" | grep -v "_CMPC")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $objs /tmp/diag_$(basename $OUT).o
echo "$OUT"
