#!/bin/bash
# Kernel-level timing (rocprofv3 --kernel-trace --stats) of a short bench run, then the class-1
# stage breakdown when the diagnostic library is present. Each GPU step is time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-stats}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 > "$OUT/rocprof.log" 2>&1 || exit $?
cut -d, -f1-4 "$OUT"/prof/run_kernel_stats.csv
if [ -f quad-periodic-mpc_amd/libcmpc_prof.so ]; then
  timeout -k 10 200 python3 -u scripts/phase_prof.py > "$OUT/phase.log" 2>&1 || exit $?
  grep -v amdgpu.ids "$OUT/phase.log"
fi
