#!/bin/bash
# A/B of library variants on config 5 (N=20 + estimator), bench protocol.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abc5
i=0
for kv in "$@"; do
  i=$((i + 1))
  env $kv timeout -k 10 150 python3 -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/abc5/bench_$i.log 2>&1 || { tail -5 gpurun_out/abc5/bench_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abc5/bench_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$kv', d['value'], d['ms_per_step'], r.get('avg_launch_ms'))"
done
