#!/bin/bash
# A/B helper: link a library whose translation unit <tu> comes from git revision <rev>, every
# other unit from build/obj (the current tree). usage: build_rev_variant.sh <rev> <tu.hip> <out.so>
set -e
cd "$(dirname "$0")/.."
REV=$1; TU=$2; OUT=$3
TMP=quad-periodic-mpc_amd/csrc/_rev_${TU}
git show "$REV:quad-periodic-mpc_amd/csrc/$TU" > "$TMP"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -fno-slp-vectorize \
  -c "$TMP" -o /tmp/rev_$$.o
rm -f "$TMP"
objs=$(ls build/obj/*.o | grep -v "/$TU.o$" | grep -v "_CMPC")
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $objs /tmp/rev_$$.o
echo "$OUT"
