#!/bin/bash
# One GPU session: smoke, GPU parity tests, then the bench lines of every BASELINE config that
# fits one GPU (3 = default, 2, 5, and 4's 1-GPU point). Each GPU step has its own time limit;
# the script stops at the first failure and never retries.
# usage: scripts/gpu_session.sh <tag> [--no-tests]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-session}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-600
  return $rc
}
if [ "${2:-}" != "--no-tests" ]; then
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
fi
step bench_c3 600 python -u bench.py || exit 1
step bench_c2 300 python -u bench.py --config 2 --steps 200 || exit 1
step bench_c4_1gpu 600 python -u bench.py --config 4 --steps 10 --no-cpu-baseline || exit 1
step bench_c5 900 python -u bench.py --config 5 --steps 10 --warmup 2 || exit 1
