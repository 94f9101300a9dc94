#!/bin/bash
# Config 5: side stream of the 144 / 192 classes (CMPC_SPARSE_SIDE, two digits), same library.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/sparse_side; mkdir -p "$OUT"
for v in 11 10 01 00 11; do
  echo "== CMPC_SPARSE_SIDE=$v"
  CMPC_SPARSE_SIDE=$v timeout -k 10 200 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline --no-extras > "$OUT/c5_$v.log" 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(round(d['value']/1e6,3), d['ms_per_step'])" "$OUT/c5_$v.log"
done
