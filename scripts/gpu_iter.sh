#!/bin/bash
# Fast GPU iteration: GPU parity tests, per-class diagnostics, bench (no CPU baseline).
# Each GPU step has its own time limit; the script stops at the first failure, never retries.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # name, timeout, cmd...
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 12
  return $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
step diag 300 python -u scripts/diag_classes.py || exit 1
step bench 300 python -u bench.py --no-cpu-baseline || exit 1
step bench_c5 300 python -u bench.py --no-cpu-baseline --config5 --steps 50 || exit 1
if [ -f quad-periodic-mpc_amd/libcmpc_prof.so ]; then
  step phase 200 python -u scripts/phase_prof.py || exit 1
fi
