#!/bin/bash
# Config 4 at world 1 with 1 / 2 / 4 pipeline pieces, and the per-rank loads of 2 / 4 / 8 ranks
# (131072 / 65536 / 32768 records) in 1 or 2 pieces. Each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-c4_chunks}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 -u bench.py --config 4 --no-cpu-baseline --no-extras --steps 20 --warmup 3"
for gb in 262144 131072 65536 32768; do
  for c in 1 2 4; do
    [ $((gb / c)) -lt 16384 ] && continue
    timeout -k 10 300 $B --global-batch $gb --chunks $c > "$OUT/c4_${gb}_${c}.log" 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), 'M', d['ms_per_step'])" "$OUT/c4_${gb}_${c}.log" $gb $c
  done
done
