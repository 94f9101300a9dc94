#!/bin/bash
# w128 stage split at N = 20 trot (stop-after builds), N = 10 batch-size sweep (config mix), the
# default bench line (config 3 + other configs + scaling model). Each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r03_c}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1; local t=$2; shift 2; echo "=== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -n 10 | cut -c1-400; return $rc; }
step phase_n20 300 bash scripts/gpu_phase_n20.sh || exit 1
step sweep_mix 300 python3 -u scripts/occupancy_sweep.py --horizon 10 --random-contact-frac 0.25 || exit 1
step bench 900 python3 -u bench.py || exit 1
