#!/bin/bash
# GPU tests on the default library, then A/B: default vs variants (CMPC_LIB), configs 3/2/5,
# N = 16 / 20 trot, and the class-1 stage breakdown. Each step time-limited; stops at a failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r03_ab2}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1; local t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -n 4 | cut -c1-300
  return $rc
}
ms() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,3), 'M', d['ms_per_step'], r.get('avg_launch_ms'), r.get('tail_avg_ms'), d.get('status_counts'))" "$1"; }
if [ "${TESTS:-1}" = 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread || exit 1
fi
B="python3 -u bench.py --no-cpu-baseline --no-extras"
for lib in default "$@"; do
  tag=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset CMPC_LIB; else export CMPC_LIB=$PWD/$lib; fi
  step c3_$tag 300 $B --steps 30 || exit 1
  step c2_$tag 300 $B --config 2 --steps 200 || exit 1
  step n16_$tag 300 $B --horizon 16 --random-contact-frac 0 --steps 10 --warmup 2 || exit 1
  step n20_$tag 300 $B --horizon 20 --random-contact-frac 0 --steps 10 --warmup 2 || exit 1
  step c5_$tag 300 $B --config 5 --steps 10 --warmup 2 || exit 1
done
unset CMPC_LIB
for f in "$OUT"/c3_* "$OUT"/c2_* "$OUT"/n16_* "$OUT"/n20_* "$OUT"/c5_*; do ms "$f"; done
if [ -f variants/libphase.so ]; then
  step phase_b256 300 python3 -u scripts/phase_prof.py --lib $PWD/variants/libphase.so --batch 256 --reps 20 || exit 1
  if [ -f variants/libplace.so ]; then step place 300 env CMPC_LIB=$PWD/variants/libplace.so python3 -u scripts/place_prof.py --batches 256,4096,65536 || exit 1; fi
fi
step rocprof_c5 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv -- python3 bench.py --config 5 --no-cpu-baseline --no-extras --steps 5 --warmup 2 || exit 1
f=$(find "$OUT/prof_c5" -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/trace_timeline.py "$f" --steps 1
exit 0
