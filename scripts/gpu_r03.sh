#!/bin/bash
# Round-3 GPU session: smoke, GPU parity tests, the default bench line (config 3 + configs 2, 5,
# N=16 in other_configs), then rocprofv3 kernel stats for configs 3 and 5. Each GPU step has its
# own time limit; the script stops at the first failure and never retries.
# usage: scripts/gpu_r03.sh <tag> [--no-tests] [--no-prof]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r03}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=1; PROF=1
for a in "$@"; do
  case $a in --no-tests) TESTS=0 ;; --no-prof) PROF=0 ;; esac
done
step() {  # name, timeout, cmd...
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-1500
  return $rc
}
if [ $TESTS = 1 ]; then
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread || exit 1
fi
step bench 900 python -u bench.py || exit 1
if [ $PROF = 1 ]; then
  step rocprof_c3 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 20 || exit 1
  step rocprof_c5 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv -- python3 bench.py --config 5 --no-cpu-baseline --no-extras --steps 5 --warmup 2 || exit 1
  for c in c3 c5; do
    f=$(find "$OUT/prof_$c" -name "*kernel_stats.csv" | head -n 1)
    [ -n "$f" ] && cut -d, -f1-4 "$f" | cut -c1-160
  done
fi
exit 0
