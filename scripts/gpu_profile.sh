#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench (+ CPU baseline), rocprofv3 kernel stats, and the
# two HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs, --kernel-trace only).
# Every GPU step has its own time limit; the script stops at the first failure, never retries.
# usage: scripts/gpu_profile.sh <tag> [extra bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-prof}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 12 "$OUT/$name.log"
  return $rc
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
step bench 600 python -u bench.py "$@" || exit 1
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 "$@" || exit 1
step pmc_fetch 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" || exit 1
step pmc_write 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" || exit 1
find "$OUT" -name "*.csv" | head -20
