#!/bin/bash
# Round-2 final profile: kernel-trace stats of config 3 and config 5 (rocprofv3 --kernel-trace
# --stats), then the counter passes of scripts/gpu_pmc_all.sh (cfg3, cfg5, n16). Every GPU step
# is time-limited; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in 3 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$c" -o run --output-format csv -- \
    python3 bench.py --config $c --no-cpu-baseline --no-extras --steps 20 > "$OUT/rocprof_c$c.log" 2>&1 || exit $?
  cut -d, -f1-4 "$OUT"/prof_c$c/run_kernel_stats.csv | head -8
done
bash scripts/gpu_pmc_all.sh "${TAG}_pmc" cfg3 cfg5 n16
