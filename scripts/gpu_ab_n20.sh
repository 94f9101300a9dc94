#!/bin/bash
# A/B of library variants on N=20 trot (all instances in the 128-row wide class), bench protocol.
# usage: scripts/gpu_ab_n20.sh "ENV=..." ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab20
i=0
for kv in "$@"; do
  i=$((i + 1))
  env $kv timeout -k 10 120 python3 -u bench.py --horizon 20 --random-contact-frac 0 --steps 10 --no-cpu-baseline --no-extras > gpurun_out/ab20/bench_$i.log 2>&1 || { tail -5 gpurun_out/ab20/bench_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab20/bench_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$kv', d['value'], d['ms_per_step'], r['avg_launch_ms'])"
done
