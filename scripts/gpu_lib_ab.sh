#!/bin/bash
# Same-box A/B of library builds: each workload timed under every CMPC_LIB in turn, the whole
# rotation repeated (ABAB...), so drift over the session hits every build alike.
# usage: scripts/gpu_lib_ab.sh <tag> <reps> default variants/a.so variants/b.so ...
# workloads: config 3, config 2, N = 16 trot, config 5 (bench.py --no-extras, one line each);
# WL="cfg3 b32768 ..." picks others (bNNN: config 3's mix at batch NNN)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for w in ${WL:-cfg3 cfg2 n16 cfg5}; do
    case $w in
      b*) args="--config 3 --batch ${w#b} --steps 50" ;;
      cfg3) args="--config 3 --steps 50" ;;
      cfg2) args="--config 2 --steps 200" ;;
      n16) args="--horizon 16 --random-contact-frac 0 --steps 20" ;;
      cfg5) args="--config 5 --steps 10 --warmup 2" ;;
    esac
    for v in "$@"; do
      if [ "$v" = default ]; then unset CMPC_LIB; else export CMPC_LIB=$PWD/$v; fi
      timeout -k 10 200 python3 -u bench.py $args --no-cpu-baseline --no-extras > "$OUT/b.log" 2>&1 || { echo "$w $v failed"; tail -5 "$OUT/b.log"; exit 1; }
      python3 -c "
import json
d = json.loads([l for l in open('$OUT/b.log') if l.startswith('{')][-1])
r = d['roofline']
print('$rep $w %-28s' % '$v', round(d['value'] / 1e6, 3), 'M', d['ms_per_step'], 'ms  launch', r.get('avg_launch_ms'), 'tail', r.get('tail_avg_ms'))" | tee -a "$OUT/ab.log"
    done
  done
done
