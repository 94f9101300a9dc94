#!/bin/bash
# Round-5 session: smoke, GPU tests (all, no -x), the default bench, the class-cost probe, then
# config-3 A/B of library variants (built by scripts/build_diag_variant.sh, chosen by CMPC_LIB).
# usage: scripts/gpu_r05.sh <tag> [--no-tests] [--probe] [variant.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r05}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=1
if [ "${1:-}" = "--no-tests" ]; then TESTS=0; shift; fi
PROBE=0
if [ "${1:-}" = "--probe" ]; then PROBE=1; shift; fi
if [ $TESTS = 1 ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $OUT/pytest.log | tail -30
  [ $rc -le 1 ] || exit 1
  timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail -5 $OUT/bench.log; exit 1; }
  python3 scripts/bench_summary.py $OUT/bench.log
fi
if [ $PROBE = 1 ]; then
  timeout -k 10 300 python3 -u scripts/class_cost_probe.py > $OUT/class_cost.log 2>&1 || { echo probe failed; tail -5 $OUT/class_cost.log; exit 1; }
  cat $OUT/class_cost.log
fi
i=0
for lib in "" "$@"; do
  i=$((i + 1))
  for rep in 1 2; do
    if [ -n "$lib" ]; then export CMPC_LIB=$lib; else unset CMPC_LIB; fi
    timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > $OUT/ab_${i}_$rep.log 2>&1 || { echo "ab $lib failed"; tail -3 $OUT/ab_${i}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/ab_${i}_$rep.log').read().strip().splitlines()[-1]); r=d['roofline']; print('${lib:-default}', d['value'], d['ms_per_step'], r['avg_launch_ms'], r.get('tail_avg_ms'))"
  done
done
