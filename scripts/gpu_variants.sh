#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lib in variants/*.so; do
  echo "=== $lib"
  CMPC_LIB=$PWD/$lib timeout -k 10 300 python scripts/parity_quick.py > gpurun_out/par_$(basename $lib).log 2>&1
  rc=$?; tail -n 2 gpurun_out/par_$(basename $lib).log
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
  CMPC_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_$(basename $lib).log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$(basename $lib).log').read().strip().splitlines()[-1]); r=d['roofline']; print('value', d['value'], 'c1_ms', r['avg_launch_ms'], 'c2_ms', r['class2_avg_launch_ms'])"
done
