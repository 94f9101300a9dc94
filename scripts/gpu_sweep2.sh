#!/bin/bash
# batch-size sweep (config mix) with the classify pass on the handle's stream and beside class 1,
# then the class-1 stage breakdown at 65536. Each step time-limited; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-sweep2}
mkdir -p "$OUT"
export TMPDIR=/tmp
S="python3 -u scripts/occupancy_sweep.py --horizon 10 --random-contact-frac 0.25 --batches 4096,8192,16384,32768,65536,131072"
CMPC_CLASSIFY_SIDE=0 timeout -k 10 300 $S > "$OUT/sweep_main.log" 2>&1 || exit 1
CMPC_CLASSIFY_SIDE=1 timeout -k 10 300 $S > "$OUT/sweep_side.log" 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/phase_prof.py --lib $PWD/variants/libphase.so --batch 65536 > "$OUT/phase_65536.log" 2>&1 || exit 1
grep -h "N=" "$OUT/sweep_main.log" "$OUT/sweep_side.log" | cut -c1-150
grep -v amdgpu "$OUT/phase_65536.log"
