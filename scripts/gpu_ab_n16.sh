#!/bin/bash
# A/B of library variants on N=16 trot (the reference's deployed horizon; every instance in the
# 96-row wide class), bench protocol.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab16
i=0
for kv in "$@"; do
  i=$((i + 1))
  env $kv timeout -k 10 120 python3 -u bench.py --horizon 16 --random-contact-frac 0 --steps 10 --no-cpu-baseline --no-extras > gpurun_out/ab16/bench_$i.log 2>&1 || { tail -5 gpurun_out/ab16/bench_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab16/bench_$i.log').read().strip().splitlines()[-1]); print('$kv', d['value'], d['ms_per_step'])"
done
