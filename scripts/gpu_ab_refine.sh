#!/bin/bash
# A/B of refinement variants: N = 16 trot and config 5 bench lines, and the refinement accuracy
# probe, per library (default + the given variants/*.so).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-abr}; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for lib in "" "$@"; do
  i=$((i + 1))
  if [ -n "$lib" ]; then export CMPC_LIB=$lib; else unset CMPC_LIB; fi
  for a in "--horizon 16 --random-contact-frac 0" "--config 5 --steps 10 --warmup 2"; do
    timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras $a > $OUT/b_$i.log 2>&1 || { echo "bench $lib $a failed"; tail -3 $OUT/b_$i.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_$i.log').read().strip().splitlines()[-1]); print('${lib:-default}', '$a'.split()[1], round(d['value']/1e6,3), d['ms_per_step'])"
  done
  timeout -k 10 200 python3 -u scripts/refine_probe.py 2>&1 | grep -v ERROR | cut -c1-110 || exit 1
done
