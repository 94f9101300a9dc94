#!/bin/bash
# Round-6 probe: CPU baseline timing on the box, small-batch solve anatomy + kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r06_p}
mkdir -p "$OUT"
export TMPDIR=/tmp
lscpu > $OUT/lscpu.txt 2>&1 || true
timeout -k 10 300 python3 -u scripts/cpu_probe.py > $OUT/cpu_probe.log 2>&1 || { echo cpu probe failed; tail -5 $OUT/cpu_probe.log; }
cat $OUT/cpu_probe.log
timeout -k 10 200 python3 -u scripts/small_batch_probe.py 4096 32768 65536 262144 > $OUT/sb.log 2>&1 || { echo sb failed; tail -5 $OUT/sb.log; exit 1; }
cat $OUT/sb.log
timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 -u scripts/small_batch_probe.py 4096 32768 > $OUT/sb_tr.log 2>&1 || { echo trace failed; tail -5 $OUT/sb_tr.log; exit 1; }
f=$(ls $OUT/tr/*/run_kernel_trace.csv $OUT/tr/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/trace_timeline.py $f --anchor cmpc_solve_c1 --steps 3 > $OUT/timeline.txt 2>&1
tail -40 $OUT/timeline.txt
