#!/bin/bash
# The refinement switch (cmpc_batch_set_refine) A/B: its parity test (counts in the ledger), then
# N = 16 trot and config 5 timed with the refinement on (product) and off, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r05_ref}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k "refine_switch or deployed_horizon" > "$OUT/pytest.log" 2>&1
echo "pytest rc=$?"; grep -E "passed|failed" "$OUT/pytest.log" | tail -2; grep -A12 "parity ledger" "$OUT/pytest.log"
for rep in 1 2; do
  for w in n16 cfg5; do
    case $w in
      n16) args="--horizon 16 --random-contact-frac 0 --steps 20" ;;
      cfg5) args="--config 5 --steps 10 --warmup 2" ;;
    esac
    for r in on off; do
      extra=""; [ $r = off ] && extra="--no-refine"
      timeout -k 10 200 python3 -u bench.py $args $extra --no-cpu-baseline --no-extras > "$OUT/b.log" 2>&1 || { echo "$w $r failed"; tail -3 "$OUT/b.log"; exit 1; }
      python3 -c "
import json
d = json.loads([l for l in open('$OUT/b.log') if l.startswith('{')][-1])
print('$rep $w refine $r', round(d['value'] / 1e6, 3), 'M', d['ms_per_step'], 'ms')" | tee -a "$OUT/ab.log"
    done
  done
done
