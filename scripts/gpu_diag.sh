#!/bin/bash
# Per-kernel time split of several workloads (rocprofv3 --kernel-trace --stats), no tests.
# usage: scripts/gpu_diag.sh <tag> ; writes gpurun_out/<tag>/<case>/...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-diag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, timeout, bench args...
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  return $rc
}
run cfg3 300 || exit 1
run n16 300 --horizon 16 || exit 1
run cfg5 400 --config5 || exit 1
run n20trot 400 --horizon 20 --random-contact-frac 0 || exit 1
find "$OUT" -name "*kernel_stats.csv" | sort
