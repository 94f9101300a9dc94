#!/bin/bash
# Stage split of a wide class by diagnostic builds (timing only: the variants' results are not
# solutions): the default library, then each CMPC_LIB variant given, on one bench workload.
# usage: scripts/gpu_stage_split.sh "<bench args>" variants/a.so variants/b.so ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGS=$1; shift
for v in default "$@"; do
  if [ "$v" = default ]; then unset CMPC_LIB; else export CMPC_LIB=$PWD/$v; fi
  echo -n "$v: "
  timeout -k 10 200 python -u bench.py $ARGS --no-cpu-baseline --no-extras 2>/dev/null | python3 -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][0]); print(round(d['value']/1e6,3), 'M', d['ms_per_step'], 'ms tail', d['roofline']['tail_avg_ms'])" || exit 1
done
