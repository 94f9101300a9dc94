#!/bin/bash
# GPU tests on the default library (TESTS=0 skips), then the bench lines of configs 3 / 2 / 5 and
# N = 16 / 20 trot under each environment setting given (e.g. CMPC_WIDE_FORM=1; "default" = none).
# usage: scripts/gpu_ab_env.sh <tag> [VAR=value ...]. Each step time-limited; stops at a failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-ab_env}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -n 3 | cut -c1-300
  return $rc
}
ms() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,3), 'M', d['ms_per_step'], r.get('avg_launch_ms'), r.get('tail_avg_ms'), d.get('status_counts'))" "$1"; }
if [ "${TESTS:-1}" = 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread || exit 1
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
B="python3 -u bench.py --no-cpu-baseline --no-extras"
for setting in default "$@"; do
  tag=${setting//=/_}
  if [ "$setting" = default ]; then envp=""; else envp="env $setting"; fi
  step c3_$tag 300 $envp $B --steps 30 || exit 1
  step c2_$tag 300 $envp $B --config 2 --steps 200 || exit 1
  step c3h_$tag 300 $envp $B --batch 32768 --steps 30 || exit 1
  step n16_$tag 300 $envp $B --horizon 16 --random-contact-frac 0 --steps 10 --warmup 2 || exit 1
  step n20_$tag 300 $envp $B --horizon 20 --random-contact-frac 0 --steps 10 --warmup 2 || exit 1
  step c5_$tag 300 $envp $B --config 5 --steps 10 --warmup 2 || exit 1
done
for f in "$OUT"/c3_* "$OUT"/c3h_* "$OUT"/c2_* "$OUT"/n16_* "$OUT"/n20_* "$OUT"/c5_*; do ms "$f"; done
if [ "${PROF:-1}" = 1 ]; then
  step rocprof_c5 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv -- python3 bench.py --config 5 --no-cpu-baseline --no-extras --steps 5 --warmup 2 || exit 1
  f=$(find "$OUT/prof_c5" -name "*kernel_trace.csv" | head -n 1)
  [ -n "$f" ] && python3 scripts/trace_timeline.py "$f" --steps 1
  step rocprof_c3 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 20 || exit 1
  f=$(find "$OUT/prof_c3" -name "*kernel_trace.csv" | head -n 1)
  [ -n "$f" ] && python3 scripts/trace_timeline.py "$f" --steps 1
fi
exit 0
