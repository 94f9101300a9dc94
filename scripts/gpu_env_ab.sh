#!/bin/bash
# A/B of environment settings (knobs of a -DCMPC_DIAG_KNOBS=1 build, cmpc_kernels.h diag_knob) on
# one library, over several batch sizes, the settings rotated within each repetition.
# usage: scripts/gpu_env_ab.sh <tag> <lib.so> "<batches | cfg5 n16 n16r>" <reps> "KNOB=v ..." ...
#        (a setting "-" runs with no knob set)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; LIB=$2; BATCHES=$3; REPS=$4; shift 4
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export CMPC_LIB=$PWD/$LIB
for rep in $(seq 1 "$REPS"); do
  for b in $BATCHES; do
    for kv in "$@"; do
      case $b in
        cfg5) args="--config 5 --steps 10 --warmup 2" ;;
        n16) args="--horizon 16 --random-contact-frac 0 --steps 20" ;;
        n16r) args="--horizon 16 --steps 20" ;;
        *) args="--config 3 --batch $b --steps $(( b >= 16384 ? 50 : 200 ))" ;;
      esac
      if [ "$kv" = "-" ]; then envs=""; else envs="$kv"; fi
      env $envs timeout -k 10 150 python3 -u bench.py $args --no-cpu-baseline --no-extras > "$OUT/b.log" 2>&1 || { echo "$b $kv failed"; tail -3 "$OUT/b.log"; exit 1; }
      python3 -c "
import json
d = json.loads([l for l in open('$OUT/b.log') if l.startswith('{')][-1])
r = d['roofline']
print('$rep %6s %-34s' % ('$b', '$kv'), round(d['value'] / 1e6, 3), 'M', d['ms_per_step'], 'ms launch', r.get('avg_launch_ms'), 'tail', r.get('tail_avg_ms'))" | tee -a "$OUT/ab.log"
    done
  done
done
