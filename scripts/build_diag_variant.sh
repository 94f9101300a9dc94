#!/bin/bash
# Diagnostic library variant: some translation units recompiled with extra defines, linked with
# the default objects of every other unit (build/obj). Same flags as quad-periodic-mpc_amd/build.py.
# usage: build_diag_variant.sh <out.so> <tu.hip> -DX=1 ...            (one unit)
#        build_diag_variant.sh <out.so> "tu1.hip:-DX=1 -DY=2" "tu2.hip:-DZ=3"   (several)
set -e
cd "$(dirname "$0")/.."
OUT=$1; shift
OBJ=build/obj
FLAGS=$(python3 -c "import importlib,sys; sys.path.insert(0,'.'); print(' '.join(importlib.import_module('quad-periodic-mpc_amd.build').FLAGS))")
specs=()
if [[ "$1" == *:* ]]; then specs=("$@"); else specs=("$1:${*:2}"); fi
objs=$(ls $OBJ/*.o | grep -v "_CMPC")
extra=""
for sp in "${specs[@]}"; do
  TU=${sp%%:*}; DEFS=${sp#*:}
  o=/tmp/diag_$(basename $OUT)_$TU.o
  X=""; [[ "$TU" == *.cpp ]] && X="-x hip"
  /opt/rocm/bin/hipcc $X --offload-arch=gfx950 $FLAGS $DEFS -c quad-periodic-mpc_amd/csrc/$TU -o $o
  objs=$(echo "$objs" | grep -v "/$TU.o$")
  extra="$extra $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $objs $extra
echo "$OUT"
