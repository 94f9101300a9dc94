#!/bin/bash
# Fast GPU iteration: golden parity summary, GPU test suite, bench (each step time-limited;
# stop at the first failure, never retry).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -n 25
  return $rc
}
step parity 300 python -u scripts/parity_quick.py || exit 1
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
step bench 300 python -u bench.py --no-cpu-baseline --steps 20
