#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; stop at the first crash/timeout (exit codes other
# than 0/1 from pytest), never retry.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench 600 python bench.py || exit 1
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 20 || exit 1
find gpurun_out/prof -name "*stats*" | head
