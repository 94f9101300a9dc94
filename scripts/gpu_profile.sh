#!/bin/bash
# Profiling session: rocprofv3 kernel trace + stats of the bench workloads (configs 3, 2,
# 5 and N = 16 trot), then the PMC counter passes (scripts/gpu_pmc_all.sh). Each GPU step has its
# own time limit; the script stops at the first failure.
# usage: scripts/gpu_profile.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in cfg3 cfg2 cfg5 n16; do
  case $c in
    cfg3) args="--config 3 --steps 20" ;;
    cfg2) args="--config 2 --steps 100" ;;
    cfg5) args="--config 5 --steps 10 --warmup 2" ;;
    n16) args="--horizon 16 --random-contact-frac 0 --steps 20" ;;
  esac
  echo "=== stats $c ($(date +%T))"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-extras $args > "$OUT/rocprof_$c.log" 2>&1 || { echo "stats $c failed"; tail -5 "$OUT/rocprof_$c.log"; exit 1; }
  cut -d, -f1-4 "$OUT/prof_$c/run_kernel_stats.csv" | head -12
done
bash scripts/gpu_pmc_all.sh ${TAG}_pmc cfg3 cfg2 cfg5 n16
