#!/bin/bash
# SQ counter passes on the bench workload (one rocprofv3 --pmc run per pass, kernel trace only).
# usage: scripts/gpu_pmc_sq.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sq}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  echo "=== pass $i: $ctrs"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/p$i" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 scripts/pmc_sq_summary.py "$OUT"
