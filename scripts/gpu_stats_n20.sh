#!/bin/bash
# Kernel-level timing of the config-5 bench (N = 20 + estimator), rocprofv3 --kernel-trace --stats.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-n20stats}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config5 --steps 10 > "$OUT/rocprof.log" 2>&1 || exit $?
cut -d, -f1-4 "$OUT"/prof/run_kernel_stats.csv
