#!/bin/bash
# GPU tests, then config 5 with exact grids (default at N >= 11) and with device-bounded grids
# (CMPC_EXACT_GRID=0), then config 3 and N=16 trot.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02d/pytest.log 2>&1 || { tail -30 gpurun_out/r02d/pytest.log; exit 1; }
tail -1 gpurun_out/r02d/pytest.log
bash scripts/gpu_ab_c5.sh CMPC_X=exact CMPC_EXACT_GRID=0 || exit 1
bash scripts/gpu_ab.sh CMPC_X=cfg3 || exit 1
timeout -k 10 120 python3 -u bench.py --horizon 16 --random-contact-frac 0 --steps 10 --no-cpu-baseline --no-extras > gpurun_out/r02d/n16.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r02d/n16.log').read().strip().splitlines()[-1]); print('n16', d['value'], d['ms_per_step'])"
