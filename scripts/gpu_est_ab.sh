#!/bin/bash
# Estimator layout A/B: per library, the rocprofv3 kernel-trace stats of config 5 (estimator launch
# time) and one counter pass (LDS bank conflicts per LDS instruction, VALU instructions per wave).
# usage: scripts/gpu_est_ab.sh <tag> default variants/a.so ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i + 1))
  if [ "$v" = default ]; then unset CMPC_LIB; else export CMPC_LIB=$PWD/$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/s$i" -o run --output-format csv -- \
    python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline --no-extras > "$OUT/s$i.log" 2>&1 || { echo "stats $v failed"; exit 1; }
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES \
    -d "$OUT/p$i" -o run --output-format csv -- \
    python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/p$i.log" 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 - "$OUT" "$i" "$v" <<'PY'
import csv, sys, collections
out, i, v = sys.argv[1:4]
est = [r for r in csv.DictReader(open(f"{out}/s{i}/run_kernel_stats.csv")) if "estimate" in r["Name"]][0]
acc = collections.defaultdict(float)
for r in csv.DictReader(open(f"{out}/p{i}/run_counter_collection.csv")):
    if "estimate" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(f"{v:24s} estimator {float(est['AverageNs'])/1e3:8.1f} us  conflicts/LDS instr "
      f"{acc['SQ_LDS_BANK_CONFLICT']/max(acc['SQ_ACTIVE_INST_LDS'],1):.3f}  VALU/wave "
      f"{acc['SQ_INSTS_VALU']/max(acc['SQ_WAVES'],1):.0f}")
PY
done
