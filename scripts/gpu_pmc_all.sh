#!/bin/bash
# Counter passes for the bench workloads: per case, FETCH_SIZE and WRITE_SIZE in separate runs
# (HBM bytes, MI355X_MICROARCH.md §HBM), then two SQ passes (VALU / LDS / wait mix), each its own
# rocprofv3 --kernel-trace --pmc run with a hard time limit. Summarised by scripts/pmc_collect.py.
# usage: scripts/gpu_pmc_all.sh <tag> [case ...]   cases: cfg2 cfg3 cfg5 n16
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pmc}
shift || true
CASES=${*:-cfg3 cfg5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PASS_fetch="FETCH_SIZE"
PASS_write="WRITE_SIZE"
PASS_sq1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
PASS_sq2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for c in $CASES; do
  case $c in
    cfg2) args="--config 2" ;;
    cfg3) args="--config 3" ;;
    cfg5) args="--config 5" ;;
    n16) args="--horizon 16 --random-contact-frac 0" ;;
    *) echo "unknown case $c"; exit 1 ;;
  esac
  mkdir -p "$OUT/$c"
  for p in fetch write sq1 sq2; do
    v="PASS_$p"
    echo "=== $c/$p ($(date +%T))"
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc ${!v} -d "$OUT/$c/$p" -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-extras --steps 2 --warmup 1 $args > "$OUT/$c/$p.log" 2>&1 \
      || { echo "$c/$p failed"; tail -5 "$OUT/$c/$p.log"; exit 1; }
  done
done
echo "=== done"
