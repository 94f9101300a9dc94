#!/bin/bash
# Cost of the bench's per-solve HIP timing events: the same bench leg with the events recorded on
# every solve (default) and with none (CMPC_BENCH_NO_EVENTS=1), alternating, two runs each.
# usage: scripts/gpu_events_ab.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for ev in on off; do
    if [ $ev = off ]; then export CMPC_BENCH_NO_EVENTS=1; else unset CMPC_BENCH_NO_EVENTS; fi
    timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras "$@" > $OUT/${ev}_$rep.log 2>&1 || { echo "bench $ev failed"; tail -3 $OUT/${ev}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${ev}_$rep.log').read().strip().splitlines()[-1]); print('events $ev', d['value'], d['ms_per_step'])"
  done
done
