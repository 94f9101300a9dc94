#!/bin/bash
# Kernel trace of small-batch bench runs: per solve its makespan and the idle gap before the next
# solve's class-1 kernel (scripts/trace_timeline.py --gaps).
# usage: scripts/gpu_gap_probe.sh <tag> [batch ...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-gap}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for b in ${*:-4096 32768}; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d "$OUT/tr_$b" -o run --output-format csv -- \
    python3 bench.py --config 3 --batch $b --steps 60 --no-cpu-baseline --no-extras > "$OUT/tr_$b.log" 2>&1 || { echo "trace $b failed"; tail -5 "$OUT/tr_$b.log"; exit 1; }
  f=$(ls "$OUT"/tr_$b/*/run_kernel_trace.csv "$OUT"/tr_$b/run_kernel_trace.csv 2>/dev/null | head -1)
  if [ $b -ge 16384 ]; then anc="c1_kernel<60"; else anc="c1_kernel<64"; fi
  echo "== batch $b"
  python3 scripts/trace_timeline.py "$f" --anchor "$anc" --steps 4 --gaps | tee "$OUT/gaps_$b.txt"
  python3 scripts/trace_timeline.py "$f" --anchor "$anc" --steps 2 >> "$OUT/gaps_$b.txt"
done
