#!/bin/bash
# class-1 latency by active-set iterations (placement variant) + stage breakdown (phase variant)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-place2}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1; local t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; grep -v amdgpu.ids "$OUT/$name.log" | tail -n 12 | cut -c1-900; return $rc; }
step place_trot 300 env CMPC_LIB=$PWD/variants/libplace.so python3 -u scripts/place_prof.py --batches 256,65536 || exit 1
step place_mix 300 env CMPC_LIB=$PWD/variants/libplace.so python3 -u scripts/place_prof.py --batches 65536 --random-contact-frac 0.25 || exit 1
step phase 300 python3 -u scripts/phase_prof.py --lib $PWD/variants/libphase.so || exit 1
step phase_b256 300 python3 -u scripts/phase_prof.py --lib $PWD/variants/libphase.so --batch 256 --reps 20 || exit 1
