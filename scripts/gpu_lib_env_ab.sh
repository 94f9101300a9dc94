#!/bin/bash
# Same-box A/B of (library, environment) pairs over batch sizes, rotated within each repetition.
# usage: scripts/gpu_lib_env_ab.sh <tag> "<batches | cfg5 n16>" <reps> "lib.so|KNOB=v" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; BATCHES=$2; REPS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for b in $BATCHES; do
    for spec in "$@"; do
      lib=${spec%%|*}; kv=${spec#*|}
      case $b in
        cfg5) args="--config 5 --steps 10 --warmup 2" ;;
        n16) args="--horizon 16 --random-contact-frac 0 --steps 20" ;;
        *) args="--config 3 --batch $b --steps $(( b >= 16384 ? 50 : 200 ))" ;;
      esac
      if [ "$lib" = default ]; then unset CMPC_LIB; else export CMPC_LIB=$PWD/$lib; fi
      if [ "$kv" = "-" ] || [ "$kv" = "$spec" ]; then envs=""; else envs="$kv"; fi
      env $envs timeout -k 10 150 python3 -u bench.py $args --no-cpu-baseline --no-extras > "$OUT/b.log" 2>&1 || { echo "$b $spec failed"; tail -3 "$OUT/b.log"; exit 1; }
      python3 -c "
import json
d = json.loads([l for l in open('$OUT/b.log') if l.startswith('{')][-1])
r = d['roofline']
print('$rep %6s %-40s' % ('$b', '$spec'), round(d['value'] / 1e6, 3), 'M', d['ms_per_step'], 'ms launch', r.get('avg_launch_ms'), 'tail', r.get('tail_avg_ms'))" | tee -a "$OUT/ab.log"
    done
  done
done
