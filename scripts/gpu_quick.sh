#!/bin/bash
# Quick GPU iteration: parity tests then bench (each step time-limited, stop on crash).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench 600 python bench.py --no-cpu-baseline
