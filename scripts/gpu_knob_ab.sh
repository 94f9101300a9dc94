#!/bin/bash
# A/B of one environment knob read by a -DCMPC_DIAG_KNOBS=1 build (cmpc_kernels.h diag_knob):
# the same variant library with and without the knob set, alternating, two runs each.
# usage: scripts/gpu_knob_ab.sh <tag> <variant.so> <KNOB=value> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; LIB=$2; KV=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export CMPC_LIB=$LIB
for rep in 1 2; do
  for mode in off on; do
    if [ $mode = on ]; then export "$KV"; else unset "${KV%%=*}"; fi
    timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras "$@" > $OUT/${mode}_$rep.log 2>&1 || { echo "bench $mode failed"; tail -3 $OUT/${mode}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${mode}_$rep.log').read().strip().splitlines()[-1]); print('$KV $mode', d['value'], d['ms_per_step'])"
  done
done
