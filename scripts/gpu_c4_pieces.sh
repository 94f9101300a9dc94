#!/bin/bash
# Config-4 per-rank load on ONE GPU (world 1 solves the same pieces a rank of a G-GPU run solves):
# global batch 262144 / G for G = 1, 2, 4, 8, cut into 1, 2 or 4 pipeline pieces.
# usage: scripts/gpu_c4_pieces.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-c4pieces}
mkdir -p "$OUT"
for gb in 32768 65536 131072 262144; do
  for ch in 1 2 4; do
    timeout -k 10 120 python3 -u bench.py --config 4 --global-batch $gb --chunks $ch --steps 20 --warmup 3 \
      --no-cpu-baseline --no-extras > "$OUT/c4_${gb}_${ch}.log" 2>&1 || { tail -5 "$OUT/c4_${gb}_${ch}.log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4_${gb}_${ch}.log').read().strip().splitlines()[-1]); print('global', $gb, 'chunks', $ch, 'QP/s', d['value'], 'ms/step', d['ms_per_step'])"
  done
done
