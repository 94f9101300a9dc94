#!/bin/bash
# Round-3 A/B session: batch-size sweeps at N = 10 (pure class 1, then the config mix), config 5
# under the wide-class order / exact-grid switches, N = 16 / 20 trot, rocprof stats of config 5.
# Each GPU step has its own time limit; the script stops at the first failure, never retries.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r03_ab1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -n 12 | cut -c1-400
  return $rc
}
ms() {  # bench line -> value / ms / roofline launch + tail
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r.get('avg_launch_ms'), r.get('tail_avg_ms'), d.get('status_counts'))" "$1"
}
step sweep_n10_trot 300 python3 -u scripts/occupancy_sweep.py --horizon 10 || exit 1
step sweep_n10_mix 300 python3 -u scripts/occupancy_sweep.py --horizon 10 --random-contact-frac 0.25 || exit 1
B="python3 -u bench.py --no-cpu-baseline --no-extras"
step c5_default 300 $B --config 5 --steps 10 --warmup 2 || exit 1
step c5_order1 300 env CMPC_WIDE_ORDER=1 $B --config 5 --steps 10 --warmup 2 || exit 1
step c5_exact 300 env CMPC_EXACT_GRID=1 $B --config 5 --steps 10 --warmup 2 || exit 1
step c5_order1_exact 300 env CMPC_WIDE_ORDER=1 CMPC_EXACT_GRID=1 $B --config 5 --steps 10 --warmup 2 || exit 1
step n20_trot 300 $B --horizon 20 --random-contact-frac 0 --steps 10 --warmup 2 || exit 1
step n16_trot 300 $B --horizon 16 --random-contact-frac 0 --steps 10 --warmup 2 || exit 1
step c3 300 $B --steps 20 || exit 1
step c2 300 $B --config 2 --steps 100 || exit 1
for f in c5_default c5_order1 c5_exact c5_order1_exact n20_trot n16_trot c3 c2; do ms "$OUT/$f.log"; done
step rocprof_c5 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv -- python3 bench.py --config 5 --no-cpu-baseline --no-extras --steps 5 --warmup 2 || exit 1
f=$(find "$OUT/prof_c5" -name "*kernel_stats.csv" | head -n 1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | cut -c1-160
exit 0
