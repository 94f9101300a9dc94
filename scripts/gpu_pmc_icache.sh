#!/bin/bash
# Instruction-cache counter passes on the config-3 bench (one rocprofv3 --pmc run per pass).
# usage: scripts/gpu_pmc_icache.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-icache}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for ctrs in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES" \
            "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES"; do
  i=$((i+1))
  echo "=== pass $i: $ctrs"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/p$i" -o run --output-format csv -- python3 bench.py --config 3 --no-cpu-baseline --no-extras --steps 2 --warmup 1 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
find "$OUT" -name "*counter_collection.csv" | head
