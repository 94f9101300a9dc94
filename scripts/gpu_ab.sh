#!/bin/bash
# GPU parity tests, then the bench under each given environment setting (A/B of launch knobs),
# e.g.  scripts/gpu_ab.sh "CMPC_SIDE_PRIORITY=0" "CMPC_SIDE_PRIORITY=1"
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -1 gpurun_out/ab/pytest.log
i=0
for kv in "$@"; do
  i=$((i + 1))
  env $kv timeout -k 10 120 python3 -u bench.py --no-cpu-baseline > gpurun_out/ab/bench_$i.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab/bench_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$kv', d['value'], d['ms_per_step'], r['avg_launch_ms'], r.get('tail_avg_ms'))"
done
