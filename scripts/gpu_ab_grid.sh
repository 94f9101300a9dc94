#!/bin/bash
# A/B: wide classes launched over the worst-case grid (default) vs exact grids read back from the
# device (CMPC_EXACT_GRID=1, one host round trip per solve). No tests; each run time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_grid
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, env value, bench args...
  local name=$1 ex=$2; shift 2
  CMPC_EXACT_GRID=$ex timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  python3 - "$OUT/$name.log" "$name" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"] or {}
        print(f'{sys.argv[2]:14s} {d["value"]/1e6:8.3f} M QP/s  {d["ms_per_step"]:8.3f} ms  c1 {r.get("class1_avg_launch_ms")}  tail {r.get("tail_avg_ms")}')
PY
}
run c3_default 0 --steps 30
run c3_exact 1 --steps 30
run n20_default 0 --horizon 20 --random-contact-frac 0 --steps 5 --warmup 2
run n20_exact 1 --horizon 20 --random-contact-frac 0 --steps 5 --warmup 2
run c5_default 0 --config 5 --steps 5 --warmup 2
run c5_exact 1 --config 5 --steps 5 --warmup 2
run n16_default 0 --horizon 16 --random-contact-frac 0 --steps 10 --warmup 2
run n16_exact 1 --horizon 16 --random-contact-frac 0 --steps 10 --warmup 2
timeout -k 10 300 python -u scripts/split_bench.py --horizon 20 --random-contact-frac 0 --reps 5 > "$OUT/split_n20.log" 2>&1; tail -8 "$OUT/split_n20.log"
